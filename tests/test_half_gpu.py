"""fp16 Arnoldi values (mode mixed-half, BASELINE config 5) on matrices
outside fp16's range. IEEE fp16 holds magnitudes in [6.0e-8, 65504]; a
stiffness matrix's entries (bcsstk17: translations and rotations in one
system) span far more. mpg_csr_half_values (capi.h) scales each row that
needs it by a power of two and the SpMV unscales its fp64 row sum exactly,
so:
  * rows already in range keep the unscaled copy's bits (BAND, Laplacians,
    the C4 stand-in: every GPU solve of round 2 is unchanged);
  * an out-of-range matrix solves to tol like the oracle's fp32-value
    mixed solve (the reference has no fp16 mode);
  * without scaling (half_unscaled) the set-up fails with MPG_ERR_RANGE
    instead of running on Inf/NaN values.
Test matrix: the 27-point 3-dof stencil under a symmetric dof scaling
S A S, S = diag(1e-3, 1, 1e4) per node: SPD, entries from ~1e-11 to 5e9."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ERR_RANGE = -7


def stiff(mpg, nx=20, s=(1e-3, 1.0, 1e4)):
    A = mpg.gen_stencil27(nx, 3)
    rows = np.repeat(np.arange(A.nrows), np.diff(A.rowptr))
    sc = np.asarray(s)
    return mpg.Csr(A.nrows, A.ncols, A.rowptr, A.col, A.val * sc[rows % 3] * sc[A.col % 3])


def _half_values(hip, A, drp, dci, csr, scale):
    dv = hip.buf(A.val)
    dh, de = hip.buf(A.nnz, np.uint16), hip.buf(A.nrows + 64, np.int8)
    stats = (C.c_int64 * 4)()
    st = hip.lib.mpg_csr_half_values(hip.ctx, csr, dv.p, scale, dh.p, de.p if scale else None, stats)
    return st, dh, de, list(stats)


def _csr(hip, A):
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p,
                                     C.byref(csr)))
    return drp, dci, csr


def test_in_range_rows_keep_the_plain_cast_bits(hip, mpg):
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    drp, dci, csr = _csr(hip, A)
    try:
        st, dh, de, stats = _half_values(hip, A, drp, dci, csr, 1)
        assert st == 0 and stats == [0, stats[1], 0, 0], stats
        assert not de.get()[:A.nrows].any()
        plain = hip.buf(A.nnz, np.uint16)
        hip.call("mpg_copy_f64f16", A.nnz, hip.buf(A.val).p, plain.p)
        assert np.array_equal(dh.get(), plain.get())
        # = numpy's fp64 -> fp32 -> fp16 rounding
        assert np.array_equal(dh.get(), A.val.astype(np.float32).astype(np.float16).view(np.uint16))
    finally:
        hip.lib.mpg_csr_destroy(csr)


def test_scaled_values_and_spmv(hip, mpg):
    """Each scaled row's values are the fp16 rounding of a * 2^e (checked
    against numpy), and the scaled SpMV is within fp16 rounding of the fp64
    product; the plain cast reports the overflow and fails."""
    A = stiff(mpg, 12)
    n = A.nrows
    drp, dci, csr = _csr(hip, A)
    try:
        st, dh, de, stats = _half_values(hip, A, drp, dci, csr, 0)
        assert st == ERR_RANGE and stats[2] > 0, stats
        assert b"overflow" in hip.lib.mpg_ctx_last_error(hip.ctx)
        st, dh, de, stats = _half_values(hip, A, drp, dci, csr, 1)
        assert st == 0 and stats[0] > 0 and stats[2] == 0 and stats[3] == 0, stats
        e = de.get()[:n].astype(np.int64)
        rows = np.repeat(np.arange(n), np.diff(A.rowptr))
        want = np.ldexp(A.val, e[rows]).astype(np.float32).astype(np.float16).view(np.uint16)
        assert np.array_equal(dh.get(), want)
        h = dh.get().view(np.float16).astype(np.float64)
        rmax = np.maximum.reduceat(np.abs(h), A.rowptr[:-1])
        # (a row maximum just under 2^15 may round up to it)
        assert np.all((rmax >= 2.0 ** -2) & (rmax <= 2.0 ** 15)), (rmax.min(), rmax.max())
        assert np.all(e[np.arange(n) % 3 == 2] < 0)  # the 1e4-scaled dof's rows were brought down
        x = np.random.default_rng(4).uniform(-1, 1, n).astype(np.float32)
        dx, dy = hip.buf(x), hip.buf(n, np.float32)
        hip.call("mpg_csr_spmv_f16f32_scaled", csr, C.c_float(1.0), dh.p, de.p, dx.p, C.c_float(0.0), dy.p)
        y = dy.get().astype(np.float64)
        sp = A.to_scipy()
        exact = sp @ x.astype(np.float64)
        bound = 2.0 ** -10 * (abs(sp) @ np.abs(x.astype(np.float64)))
        assert np.all(np.abs(y - exact) <= bound)
        # the same copy through the plain f16 SpMV is off by exactly 2^e per row
        dz = hip.buf(n, np.float32)
        hip.call("mpg_csr_spmv_f16f32", csr, C.c_float(1.0), dh.p, dx.p, C.c_float(0.0), dz.p)
        z = dz.get().astype(np.float64)
        ok = np.isfinite(z) & (np.abs(z) < 1e30) & (np.abs(z) > 1e-30)
        np.testing.assert_allclose(np.ldexp(z[ok], -e[ok]), y[ok], rtol=2e-7)
    finally:
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("orth", ["cgs", "mgs"])
def test_stiff_matrix_mixed_half_converges(mpg, oracle, orth):
    A = stiff(mpg, 20)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=100)
    ref = oracle.solve(mpg, A, b, xt, mode="mixed", **opts)
    assert ref.status == "converged"
    eng = mpg.Engine(A, b, xt, mode="mixed-half", **opts)
    hs = eng.half_stats()
    eng.close()
    assert hs["rows_scaled"] == A.nrows // 3 and hs["overflowed"] == 0, hs
    got = {}
    for fmt in ("sell", "csr"):
        got[fmt] = mpg.solve(A, b, xt, engine="fused", mode="mixed-half", spmv_format=fmt, **opts)
        g = got[fmt]
        assert g.status == "converged" and g.backward_error[-1] <= opts["tol"], (fmt, g.status)
        assert g.restarts <= 3 * ref.restarts + 2, (g.restarts, ref.restarts)
    # the SELL and CSR Arnoldi SpMVs unscale the same fp64 row sums (the
    # fp64 residual prologues differ in the last bits, so whole solves are
    # compared to fp32 rounding)
    s, c = got["sell"], got["csr"]
    assert abs(s.restarts - c.restarts) <= 1
    np.testing.assert_allclose(s.step_res[:30], c.step_res[:30], rtol=1e-4)


def test_stiff_matrix_unscaled_cast_is_an_error(mpg):
    A = stiff(mpg, 12)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    with pytest.raises(RuntimeError, match="overflow"):
        mpg.solve(A, b, xt, engine="fused", mode="mixed-half", orth="cgs", prec="jacobi", rlen=30, tol=1e-10,
                  max_restarts=10, half_unscaled=True)


@pytest.mark.parametrize("fmt", ["sell", "csr"])
def test_in_range_matrix_solve_unchanged_by_scaling(mpg, fmt):
    """BAND (|a| <= 11): no row is scaled, so the scaled and plain casts give
    one solve, bit for bit."""
    A = mpg.gen_band(150_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="fused", mode="mixed-half", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3,
                spmv_format=fmt)
    a = mpg.solve(A, b, xt, **opts)
    c = mpg.solve(A, b, xt, half_unscaled=True, **opts)
    assert a.total_iters == c.total_iters == 90
    assert np.array_equal(a.step_res, c.step_res) and np.array_equal(a.x, c.x)


def _row_scaled(mpg, A, lo=-6.0, hi=6.0, seed=3):
    """D A with D = diag(10^u), u ~ U(lo, hi) per row: every row's own range
    stays small, but most rows leave fp16's and are scaled by a power of 2."""
    d = 10.0 ** np.random.default_rng(seed).uniform(lo, hi, A.nrows)
    rows = np.repeat(np.arange(A.nrows), np.diff(A.rowptr))
    return mpg.Csr(A.nrows, A.ncols, A.rowptr, A.col, A.val * d[rows])


@pytest.mark.parametrize("which", ["band-pair", "stencil27-stepped"])
def test_row_scaled_unscaling_on_every_sell_kernel(mpg, which):
    """the scaled fp16 rows must also run through the paired
    uniform SELL kernel (k_step_sell2, BAND) and the stepped copy with
    CSR-summed slices (C4's structure), not only the single-slice int16
    kernel. Each layout is asserted; the fp16 SELL solve is compared with the
    CSR-tile solve of the same scaled copy (both unscale the same fp64 row
    sums; the prologues differ in the last fp64 bits, as above)."""
    if which == "band-pair":
        A = _row_scaled(mpg, mpg.gen_band(200_000, 5, 4, seed=7))
    else:
        A = _row_scaled(mpg, mpg.gen_stencil27(105, 3, ny=105, nz=8))
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed-half", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=2)
    eng = mpg.Engine(A, b, xt, spmv_format="sell", **opts)
    lay, cols, hs = eng.spmv_layout(), eng.sell_columns(), eng.half_stats()
    eng.close()
    assert hs["rows_scaled"] > A.nrows // 2 and hs["overflowed"] == 0 and hs["exp_out_of_range"] == 0, hs
    if which == "band-pair":
        assert lay["format"] == "sell" and lay["slices_per_wave"] == 2 and cols["form"] == "int16", (lay, cols)
    else:
        assert lay["format"] == "sell" and cols["form"] == "stepped" and cols["csr_slices"] > 0, (lay, cols)
    s = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
    c = mpg.solve(A, b, xt, engine="fused", spmv_format="csr", **opts)
    assert s.total_iters == c.total_iters == 60
    assert np.all(np.isfinite(s.step_res)) and s.nonfinite_steps == 0
    np.testing.assert_allclose(s.step_res, c.step_res, rtol=1e-4)
    np.testing.assert_allclose(s.cyc_r_norm, c.cyc_r_norm, rtol=1e-4)
