"""Condition-number estimator (include/mpgmres/condest.h; the reference's
condest.cpp:34-179).

CPU: the oracle restatement (oracle/cpu_condest.cpp) against numpy singular
values on symmetric inputs (power iteration on A converges to sigma_max
there; the LSQR search gives an upper bound of sigma_min), and the CLI's
argument handling, which exits before touching a GPU.
GPU: the A^T CSR behind transposed spmv (mpg_csr_transpose) bit-exact
against a stable argsort, and whole estimates against the oracle.

Parity tolerance (GPU vs oracle, parity unpinned by reference fixtures —
the reference ships none for condest): sigma_max 1e-10 relative (power
iteration contracts rounding differences); sigma_min 1e-6 relative (LSQR
trajectories from different fp64 summation orders); the step at which the
stopping test fires within +-1.
"""
import ctypes as C
import subprocess

import numpy as np
import pytest

from tests.conftest import REPO

CLI = REPO / "icl-mixed-precision-gmres_amd" / "bin" / "condest"

MATS = {
    "lap3d-6": lambda mpg: mpg.gen_laplace3d(6),
    "stencil27-4x3": lambda mpg: mpg.gen_stencil27(4, 3),
    "band500": lambda mpg: mpg.gen_band(500, 5, 4, seed=3),
}


@pytest.mark.parametrize("mat", ["lap3d-6", "stencil27-4x3"])
def test_oracle_condest_brackets_svd(mpg, oracle, mat):
    A = MATS[mat](mpg)
    r = oracle.condest(mpg, A, 42, 100000)
    s = np.linalg.svd(A.to_scipy().toarray(), compute_uv=False)
    assert r["power_iters"] == int(np.ceil((np.log(2 * A.nrows) ** 2 - np.log(0.1 * 1e-24)) / 0.1))
    assert r["sigma_max"] == pytest.approx(s[0], rel=1e-9)
    assert s[-1] * (1 - 1e-12) <= r["sigma_min"] <= 1.1 * s[-1]
    assert r["finish_t"] > 0 and r["iters"] == int(np.ceil(r["finish_t"] * 1.25)) + 1
    assert r["cond"] == pytest.approx(r["sigma_max"] / r["sigma_min"])


def test_oracle_condest_max_iters_bounds_the_search(mpg, oracle):
    A = mpg.gen_laplace3d(6)
    r = oracle.condest(mpg, A, 42, 5)
    assert r["iters"] == 6 and r["finish_t"] == 0  # the for loop ran t = 1..5


def _cli(*args):
    return subprocess.run([str(CLI), *args], capture_output=True, text=True, timeout=60)


def test_cli_reference_argument_handling(tmp_path):
    assert CLI.exists(), "build with make -C icl-mixed-precision-gmres_amd"
    r = _cli()
    assert r.returncode == 1 and r.stdout.strip() == "No value suplied for A"
    r = _cli("--bogus")
    assert r.returncode == 1 and r.stdout.strip() == "Unknown flag--bogus"
    # without --gpu the reference prints this and does nothing (condest.cpp:217-223)
    r = _cli("--matrix", "laplace:4")
    assert r.returncode == 0 and r.stdout.strip() == "CPU not currently supported"


# ---------------------------------------------------------------- GPU


def _transpose_expected(A):
    perm = np.argsort(A.col, kind="stable").astype(np.int32)
    row_of = np.repeat(np.arange(A.nrows, dtype=np.int32), np.diff(A.rowptr))
    rp = np.concatenate([[0], np.cumsum(np.bincount(A.col, minlength=A.ncols))]).astype(np.int32)
    return rp, row_of[perm], perm


def _dup_matrix(mpg):
    """duplicates in a row, an empty row and an empty column"""
    rp = np.array([0, 3, 3, 5, 7], np.int32)
    ci = np.array([1, 1, 3, 0, 1, 3, 1], np.int32)
    return mpg.Csr(4, 4, rp, ci, np.arange(1.0, 8.0))


@pytest.mark.gpu
@pytest.mark.parametrize("mat", ["dups", "band500", "stencil27-4x3", "random"])
def test_csr_transpose_bit_exact(hip, mpg, mat):
    if mat == "dups":
        A = _dup_matrix(mpg)
    elif mat == "random":
        import scipy.sparse as sp

        S = sp.random(3000, 2500, density=0.004, format="csr", random_state=7)
        S.sort_indices()
        A = mpg.Csr(3000, 2500, S.indptr.astype(np.int32), S.indices.astype(np.int32), S.data)
    else:
        A = MATS[mat](mpg)
    rp, ci, va = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
    rpt, cit, perm = hip.buf(A.ncols + 1, np.int32), hip.buf(A.nnz, np.int32), hip.buf(A.nnz, np.int32)
    vt = hip.buf(A.nnz, np.float64)
    hip.call("mpg_csr_transpose", A.nrows, A.ncols, A.nnz, rp.p, ci.p, rpt.p, cit.p, perm.p)
    hip.call("mpg_gather_b64", A.nnz, perm.p, va.p, vt.p)
    e_rp, e_ci, e_perm = _transpose_expected(A)
    assert np.array_equal(rpt.get(), e_rp)
    assert np.array_equal(cit.get(), e_ci)
    assert np.array_equal(perm.get(), e_perm)
    assert np.array_equal(vt.get(), A.val[e_perm])


@pytest.mark.gpu
def test_csr_transpose_empty(hip, mpg):
    rp = hip.buf(np.zeros(4, np.int32))
    rpt = hip.buf(np.full(6, -1, np.int32))
    hip.call("mpg_csr_transpose", 3, 5, 0, rp.p, None, rpt.p, None, None)
    assert np.array_equal(rpt.get(), np.zeros(6, np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("mat", list(MATS))
def test_condest_matches_oracle(mpg, oracle, mat):
    A = MATS[mat](mpg)
    ref = oracle.condest(mpg, A, 42, 100000)
    got = mpg.condest(A, 42, 100000)
    assert got["power_iters"] == ref["power_iters"]
    assert got["sigma_max"] == pytest.approx(ref["sigma_max"], rel=1e-10)
    assert got["sigma_min"] == pytest.approx(ref["sigma_min"], rel=1e-6)
    assert abs(got["finish_t"] - ref["finish_t"]) <= 1
    assert got["iters"] == int(np.ceil(got["finish_t"] * 1.25)) + 1
    assert got["stop_reason"] == ref["stop_reason"] == 0


@pytest.mark.gpu
def test_condest_cli_lines():
    r = subprocess.run([str(CLI), "--matrix", "laplace:6", "--gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert lines[0].startswith("sigma_max = ")
    assert any(x.endswith(": finishing") and x.startswith("t = ") for x in lines)
    assert lines[-2].endswith(" iterations total")
    assert lines[-1].startswith("Computed cond(A) = ")
    cond = float(lines[-1].split("=")[1])
    assert 15 < cond < 25  # the 6^3 Laplacian: 19.2
