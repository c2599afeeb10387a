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
