"""The CLI keeps the reference's flags and stdout lines, so the reference's
experiment harness (automated.py:33-38 summary regex, restated below) parses
our output unchanged."""
import re
import subprocess

import pytest

pytestmark = pytest.mark.gpu

# automated.py:33-38
SUMMARY = re.compile(
    r"Found solution with rel prec res norm = (\d\.?\d*e(?:\+|-)\d+|\d+\.?\d*) when k = (\d+) and i = (\d+)\n"
    r"  total iterations = (\d+)\n"
    r"  ilu took (\d\.?\d*e(?:\+|-)\d+|\d+\.?\d*)s; gmres took (\d\.?\d*e(?:\+|-)\d+|\d+\.?\d*)s\n"
    r"  resNorm = (\d\.?\d*e(?:\+|-)\d+|\d+\.?\d*); errNorm = (\d\.?\d*e(?:\+|-)\d+|\d+\.?\d*)\n")


@pytest.mark.parametrize("engine", ["fused", "surface"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "single-prec", "single"])
def test_cli_stdout_matches_harness_regex(mpg, engine, mode):
    tol = "1e-5" if mode == "single" else "1e-9"
    out = subprocess.run([str(mpg.CLI), "--matrix", "laplace:12", "--rlen", "30", "--mode", mode, "--orth", "cgs",
                          "--prec", "jacobi", "--tol", tol, "--engine", engine, "--gpu"],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    m = SUMMARY.search(out)
    assert m, out
    assert int(m.group(4)) % 30 == 0 and int(m.group(2)) == 0
    assert out.startswith("||x|| = ")
    assert ("Doing Mixed Precision test" in out) == (mode == "mixed")


def test_cli_rejects_like_the_reference(mpg):
    r = subprocess.run([str(mpg.CLI), "--matrix", "laplace:4", "--rlen", "10", "--orth", "householder"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "Unknown Orthogonalization" in r.stdout
    r = subprocess.run([str(mpg.CLI), "--rlen", "10"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "No value suplied for A" in r.stdout


def test_cli_default_preconditioner_is_ilu(mpg):
    """With no --prec the reference CLI uses ILU(0) (gmres_perf_test.cpp:322);
    the run converges and prints the harness lines."""
    out = subprocess.run([str(mpg.CLI), "--matrix", "laplace:10", "--rlen", "30", "--mode", "mixed", "--tol", "1e-9",
                          "--gpu"], capture_output=True, text=True, timeout=120, check=True).stdout
    m = SUMMARY.search(out)
    assert m, out
    assert float(m.group(1)) <= 1e-9


def test_cli_bpath_right_hand_side(mpg, tmp_path):
    """--bpath: b from a Matrix Market file, x_true = 0 (gmres_perf_test.cpp
    :412-421), so ||x|| prints 0 and errNorm is the solution's norm; the CLI
    solve equals the library solve with that b."""
    import numpy as np

    A = mpg.gen_spec("laplace:10")
    xt = mpg.rand_vect(A.nrows, 5)
    b = mpg.host_spmv(A, xt)
    p = tmp_path / "b.mtx"
    p.write_text("%%MatrixMarket matrix array real general\n" + f"{A.nrows} 1\n" +
                 "".join(f"{v:.17g}\n" for v in b))
    assert np.array_equal(mpg.load_mtx_vector(str(p), A.nrows), b)
    out = subprocess.run([str(mpg.CLI), "--matrix", "laplace:10", "--bpath", str(p), "--rlen", "30", "--mode", "mixed",
                          "--orth", "cgs", "--prec", "jacobi", "--tol", "1e-9", "--gpu"],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    assert out.startswith("||x|| = 0\n"), out[:80]
    assert f"||b|| = {np.linalg.norm(b):.6g}" in out
    m = SUMMARY.search(out)
    assert m, out
    got = mpg.solve(A, b, np.zeros(A.nrows), engine="fused", mode="mixed", orth="cgs", prec="jacobi", rlen=30,
                    tol=1e-9)
    assert int(m.group(3)) == got.restarts and int(m.group(4)) == got.total_iters
    assert abs(float(m.group(8)) - np.linalg.norm(got.x)) <= 1e-5 * np.linalg.norm(got.x)  # errNorm, x_true = 0


def test_cli_ngpus(mpg):
    """--ngpus N row-partitions the fused solve over N GPUs of the process
    (mpg_solve_multi_gpu): the reference's stdout lines at N = 1, and a clear
    failure when more GPUs are asked for than are visible."""
    args = [str(mpg.CLI), "--matrix", "laplace:12", "--rlen", "30", "--mode", "mixed", "--orth", "cgs",
            "--prec", "jacobi", "--tol", "1e-9", "--gpu"]
    out = subprocess.run(args + ["--ngpus", "1"], capture_output=True, text=True, timeout=120, check=True).stdout
    m = SUMMARY.search(out)
    assert m and "Doing Mixed Precision test" in out, out
    ref = SUMMARY.search(subprocess.run(args, capture_output=True, text=True, timeout=120, check=True).stdout)
    assert m.group(4) == ref.group(4)  # the same iteration count as the one-GPU solve
    n = mpg.device_count() + 1
    r = subprocess.run(args + ["--ngpus", str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "visible" in r.stderr, (r.stdout, r.stderr)
