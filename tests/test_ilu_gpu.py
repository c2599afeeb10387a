"""ILU(0) and ILU-Jacobi on the MI355X (include/mpgmres/ilu.h) against the
CPU oracle (oracle/cpu_gmres.cpp: the reference's ilu0_impl with its pivot
positions filled in, MKL sparse triangular solves, the generic
ilusv_jacobi).

Tolerances:
- factors: bit-exact. The GPU runs the same fp64 operation sequence per
  entry (uncontracted products, elimination steps in column order) and
  rounds to fp32 once, like the oracle;
- triangular solves: fp64 row sums rounded once (MKL's own order differs):
  1e-12 relative for fp64, 4 ulp-scale (2e-6 relative) for fp32;
- ILU-Jacobi: the oracle sums in the factor precision, the GPU in fp64:
  1e-13 / 1e-5 relative.
"""
import ctypes as C

import numpy as np
import pytest

from tests.golden.make_golden import convdiff

pytestmark = pytest.mark.gpu


def _random_diag_sparse(mpg, n, per_row, seed):
    """Irregular pattern, explicit diagonal, diagonally dominant."""
    g = np.random.default_rng(seed)
    rp, ci, va = [0], [], []
    for i in range(n):
        cols = set(g.integers(0, n, per_row).tolist()) - {i}
        cols = sorted(cols | {i})
        off = g.uniform(-1, 1, len(cols))
        row = [(c, v) for c, v in zip(cols, off) if c != i]
        diag = 1.0 + sum(abs(v) for _, v in row)
        row.append((i, diag if i % 7 else -diag))
        row.sort()
        ci += [c for c, _ in row]
        va += [v for _, v in row]
        rp.append(len(ci))
    return mpg.Csr(n, n, np.array(rp, np.int32), np.array(ci, np.int32), np.array(va))


MATS = {
    "convdiff32": lambda mpg: convdiff(mpg, 32),
    "lap3d-20": lambda mpg: mpg.gen_laplace3d(20),
    "band3000": lambda mpg: mpg.gen_band(3000, 5, 4, seed=3),
    "random2000": lambda mpg: _random_diag_sparse(mpg, 2000, 6, 11),
}


class Ilu:
    def __init__(self, hip, A, dt):
        self.hip, self.A, self.dt = hip, A, dt
        lib = hip.lib
        lib.mpg_ilu_values_dev.restype = C.c_void_p
        lib.mpg_ilu_diag_dev.restype = C.c_void_p
        self.drp, self.dci, self.dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
        self.csr = C.c_void_p()
        hip.check(lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, self.drp.p, self.dci.p,
                                     C.byref(self.csr)))
        self.h = C.c_void_p()
        hip.check(lib.mpg_ilu0_create(hip.ctx, self.csr, self.dv.p, 0 if dt == np.float64 else 1, C.byref(self.h)),
                  "mpg_ilu0_create")

    def factors(self):
        lib, n = self.hip.lib, self.A.nrows
        lu = np.empty(self.A.nnz, self.dt)
        di = np.empty(n, np.int32)
        self.hip.check(lib.mpg_memcpy_d2h(self.hip.ctx, lu.ctypes.data, C.c_void_p(lib.mpg_ilu_values_dev(self.h)),
                                          lu.nbytes))
        self.hip.check(lib.mpg_memcpy_d2h(self.hip.ctx, di.ctypes.data, C.c_void_p(lib.mpg_ilu_diag_dev(self.h)),
                                          di.nbytes))
        return lu, di

    def apply(self, x, kind, steps=1):
        dx = self.hip.buf(x.astype(self.dt))
        if kind == "ilu":
            self.hip.check(self.hip.lib.mpg_ilu_solve(self.hip.ctx, self.h, dx.p), "mpg_ilu_solve")
        else:
            self.hip.check(self.hip.lib.mpg_ilu_jacobi_solve(self.hip.ctx, self.h, steps, dx.p), "ilu_jacobi")
        out = dx.get()
        assert self.hip.lib.mpg_ilu_fault(self.h) == 0
        return out

    def close(self):
        self.hip.lib.mpg_ilu_destroy(self.h)
        self.hip.lib.mpg_csr_destroy(self.csr)


@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("mat", list(MATS))
def test_ilu0_factors_bit_exact(hip, mpg, oracle, mat, dt):
    A = MATS[mat](mpg)
    L = Ilu(hip, A, dt)
    try:
        lu, di = L.factors()
        ref_lu, ref_di = oracle.ilu0(A, dt)
        assert np.array_equal(di, ref_di)
        assert np.array_equal(lu, ref_lu), np.max(np.abs(lu - ref_lu))
    finally:
        L.close()


@pytest.mark.parametrize("kind,steps", [("ilu", 1), ("ilu_jacobi", 1), ("ilu_jacobi", 4)])
@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("mat", list(MATS))
def test_ilu_apply_matches_oracle(hip, mpg, oracle, mat, dt, kind, steps):
    A = MATS[mat](mpg)
    x = mpg.rand_vect(A.nrows, 5).astype(dt)
    L = Ilu(hip, A, dt)
    try:
        got = L.apply(x, kind, steps)
        ref = oracle.ilu_apply(A, x, kind, steps, dt)
        if kind == "ilu":
            rtol = 1e-12 if dt == np.float64 else 2e-6
        else:
            rtol = 1e-13 if dt == np.float64 else 1e-5
        np.testing.assert_allclose(got, ref, rtol=rtol, atol=rtol * np.abs(ref).max())
    finally:
        L.close()


def test_ilu_large_stencil_consistent(hip, mpg):
    """60^3 Laplacian (216k rows, ~180 dependency levels): the sync-free
    factorisation and solves run to completion with no fault, and
    L U y = x holds for y = M^-1 x (checked with the factors)."""
    import scipy.sparse as sp

    A = mpg.gen_laplace3d(60)
    L = Ilu(hip, A, np.float64)
    try:
        x = mpg.rand_vect(A.nrows, 9)
        y = L.apply(x, "ilu")
        lu, di = L.factors()
        F = sp.csr_matrix((lu, A.col, A.rowptr), shape=(A.nrows, A.nrows))
        low = sp.tril(F, -1) + sp.identity(A.nrows)
        up = sp.triu(F)
        r = low @ (up @ y) - x
        assert np.abs(r).max() <= 1e-12 * np.abs(x).max()
    finally:
        L.close()


@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("mat", ["band3000", "band-wide", "random2000", "lap3d-20", "grid-3000x2"])
def test_ilu_serial_solve_matches_levels(hip, mpg, monkeypatch, mat, dt):
    """Serial-chain solves (one workgroup, for schedules with few rows per
    level) and level-scheduled solves give identical results: both sum each
    row in fp64 in CSR order and round once. Banded matrices take the serial
    path; the random pattern and the 3-D Laplacian (wide levels) and a 3000x2 grid (dependencies
    3000 rows back, beyond the serial kernel's LDS ring) keep the levels."""
    extra = {"band-wide": lambda: mpg.gen_band(9000, 31, 29, seed=5), "grid-3000x2": lambda: mpg.gen_laplace3d(3000, 2, 1)}
    A = extra[mat]() if mat in extra else MATS[mat](mpg)
    x = mpg.rand_vect(A.nrows, 7).astype(dt)
    out = {}
    for env in ("1", "0"):
        monkeypatch.setenv("MPG_ILU_SERIAL", env)
        L = Ilu(hip, A, dt)
        try:
            out[env] = (L.apply(x, "ilu"), hip.lib.mpg_ilu_solve_mode(L.h))
        finally:
            L.close()
    assert out["0"][1] == 0
    assert out["1"][1] == (3 if mat.startswith("band") else 0)
    assert np.array_equal(out["1"][0], out["0"][0])


@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
def test_ilu_level_solve_tag_pattern_and_nan_inputs(hip, mpg, monkeypatch, dt):
    """The level-scheduled solves use a signalling-NaN bit pattern as the
    'not yet solved' tag of their output. A right-hand side holding exactly
    that pattern, a quiet NaN and an Inf must neither hang a poll nor fault:
    the rows they reach come out NaN/Inf, and every other row keeps the bits
    of the serial chain (which has no tag). The matrix is two decoupled
    1500-row bands, the special values all go into the second one, so the
    first block's rows stay finite."""
    B = mpg.gen_band(1500, 5, 4, seed=3)
    A = mpg.Csr(3000, 3000, np.concatenate([B.rowptr, B.rowptr[1:] + B.nnz]).astype(np.int32),
                np.concatenate([B.col, B.col + 1500]).astype(np.int32), np.concatenate([B.val, B.val]))
    x = mpg.rand_vect(A.nrows, 5).astype(dt)
    tag = np.array([0x7FF5A5A5A5A5A5A5 if dt == np.float64 else 0x7FA5A5A5],
                   np.uint64 if dt == np.float64 else np.uint32).view(dt)[0]
    x[1600] = tag
    x[2000] = np.nan
    x[2500] = np.inf
    out = {}
    for env in ("1", "0"):  # serial chain, then the level schedule (tagged)
        monkeypatch.setenv("MPG_ILU_SERIAL", env)
        L = Ilu(hip, A, dt)
        try:
            out[env] = (L.apply(x, "ilu"), hip.lib.mpg_ilu_solve_mode(L.h))  # apply asserts no fault
        finally:
            L.close()
    assert out["1"][1] == 3 and out["0"][1] == 0
    s, lv = out["1"][0], out["0"][0]
    assert np.isnan(lv[1500:]).any() and np.isfinite(lv[:1500]).all()
    assert np.array_equal(np.isnan(s), np.isnan(lv))
    ok = ~np.isnan(s)
    assert np.array_equal(s[ok], lv[ok])
    bits = lv.view(np.uint64 if dt == np.float64 else np.uint32)
    assert not (bits == np.array([tag]).view(bits.dtype)[0]).any()  # no tag left in the output


def test_ilu_rejects_missing_diagonal(hip, mpg):
    A = mpg.Csr(3, 3, np.array([0, 1, 2, 3], np.int32), np.array([1, 1, 2], np.int32), np.ones(3))
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
    csr, h = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, 3, 3, 3, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        assert hip.lib.mpg_ilu0_create(hip.ctx, csr, dv.p, 0, C.byref(h)) == -5  # MPG_ERR_UNSUPPORTED
    finally:
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("engine", ["surface", "fused"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "single-prec"])
@pytest.mark.parametrize("prec", ["ilu", "ilu_jacobi"])
def test_ilu_solve_live_oracle(mpg, oracle, engine, mode, prec):
    """Whole GMRES(30) solves with ILU / ILU-Jacobi(3) on the 24^3 Laplacian
    against the oracle run on the same inputs (tests/parity.py classes)."""
    from tests.parity import compare_mkl

    A = mpg.gen_laplace3d(24)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec=prec, rlen=30, tol=1e-10, max_restarts=60, jacobi_steps=3)
    got = mpg.solve(A, b, xt, engine=engine, **opts)
    # two-sided: MKL (pinned branch) at 1/4/8 threads and the loop kernels; ILU-Jacobi's
    # last cycle ends at 6.5e-14 under MKL, 2.8e-13 on the loops (GPU 2.7e-13)
    runs = compare_mkl(oracle, mpg, A, b, xt, got, opts, f"lap24-{mode}-{prec}-{engine}",
                       runs=_ILU_ORACLE.setdefault((mode, prec), {}))
    assert runs[1].status == "converged"


_ILU_ORACLE = {}


@pytest.mark.parametrize("engine", ["surface", "fused"])
def test_ilu_solve_fault_fails_the_solve(mpg, engine, monkeypatch):
    """A level-scheduled triangular solve whose bounded wait expires records
    a fault and leaves x partly solved; the engines read the sticky fault
    word (fused: every restart-cycle boundary; surface: after every apply)
    and fail the solve with MPG_ERR_BREAKDOWN instead of iterating on a wrong
    M^-1 w. A 1-tick wait bound makes every real wait fault."""
    A = mpg.gen_laplace3d(24)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="ilu", rlen=30, tol=1e-10, max_restarts=60)
    monkeypatch.setenv("MPG_ILU_SERIAL", "0")
    monkeypatch.setenv("MPG_ILU_WAIT_TICKS", "1")
    with pytest.raises(RuntimeError, match=r"solve failed \(-6\).*ILU triangular solve fault"):
        mpg.solve(A, b, xt, engine=engine, **opts)
    monkeypatch.delenv("MPG_ILU_WAIT_TICKS")
    got = mpg.solve(A, b, xt, engine=engine, **opts)  # a fresh factor has a clear fault word
    assert got.status == "converged"
