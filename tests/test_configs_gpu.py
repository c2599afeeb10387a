"""Every BASELINE.json config at its stated size on one MI355X, against the
oracle (the kernels_mkl.cpp restatement) run live on the same inputs where
it finishes in seconds, and through size-independent properties where it
does not (SURVEY §8(a) config shorthand):

  C1  bcsstk17 stand-in through the MM loader    tests/test_c1_standin.py
  C2  LAP-1M (100^3 7-point), fp64 GMRES(30)     live oracle, CGS and MGS
  C3  LAP-1M, fp32 inner + fp64 outer            live oracle, CGS / CGSR / MGS
  C4  Queen_4147 stand-in (27-point, 3 dof)      live oracle at 40^3 x 3 and
                                                 at 105 x 105 x 8 x 3 (the
                                                 stepped-int16 W = 4 SELL form
                                                 full-size C4 runs on), its
                                                 full-size SpMV against CSR and
                                                 MKL, properties at 111^3 x 3
  C5  BAND-100M fp16 values + fp64 IR            full size, converges to tol

Reference SpMV / drivers: kernels_mkl.cpp:326-352, gmres.cpp:24-245,
gmres_perf_test.cpp:53-182, 413-416. Tolerances: tests/parity.py."""
import numpy as np
import pytest

from tests.parity import as_ref, compare

pytestmark = pytest.mark.gpu


def _problem(mpg, A):
    xt = mpg.rand_vect(A.nrows, 42)
    return A, xt, mpg.host_spmv(A, xt)


@pytest.fixture(scope="module")
def lap1m(mpg):
    return _problem(mpg, mpg.gen_laplace3d(100))


@pytest.mark.parametrize("mode,orth", [("baseline", "cgs"), ("baseline", "mgs"), ("mixed", "cgs"),
                                       ("mixed", "cgsr"), ("mixed", "mgs")])
def test_c2_c3_lap1m_fixed_cycles(mpg, oracle, lap1m, mode, orth):
    """3 restart cycles at tol = 0 (aborts at check_initial of cycle 4):
    every step's |s(k+1)| and every cycle's backward error against the oracle."""
    A, xt, b = lap1m
    assert A.nrows == 1_000_000 and A.nnz == 6_940_000
    opts = dict(mode=mode, orth=orth, prec="identity", rlen=30, tol=0.0, max_restarts=3)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    got = mpg.solve(A, b, xt, engine="fused", **opts)
    assert got.status == ref.status == "aborted" and got.total_iters == 90
    compare(as_ref(ref), got, mode, 0.0, 30, f"lap1m-{mode}-{orth}")
    if mode != "baseline":  # fp32 Arnoldi: the whole history, not just cycle 0
        np.testing.assert_allclose(got.step_res, ref.step_res, rtol=1e-3, atol=1e-6 * ref.minvb_norm)


@pytest.mark.parametrize("mode", ["baseline", "mixed"])
def test_c2_c3_lap1m_converges_like_oracle(mpg, oracle, lap1m, mode):
    A, xt, b = lap1m
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=1e-6, max_restarts=200)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    assert ref.status == "converged"
    for engine in ("fused", "surface"):
        got = mpg.solve(A, b, xt, engine=engine, **opts)
        compare(as_ref(ref), got, mode, opts["tol"], 30, f"lap1m-{mode}-conv-{engine}")


@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("mixed", "mgs"), ("baseline", "cgs")])
def test_c4_stencil27_live_oracle(mpg, oracle, mode, orth):
    """The Queen_4147 stand-in's structure (27-point, 3 unknowns per node,
    24-81 entries per row, columns beyond int16 reach at this size too) at
    40^3 x 3 = 192,000 rows, where the oracle runs in seconds."""
    A, xt, b = _problem(mpg, mpg.gen_stencil27(40, 3))
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=100)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    assert ref.status == "converged"
    for engine in ("fused", "surface"):
        got = mpg.solve(A, b, xt, engine=engine, **opts)
        compare(as_ref(ref), got, mode, opts["tol"], 30, f"stencil27-40-{mode}-{orth}-{engine}")


@pytest.fixture(scope="module")
def c4_stepped(mpg):
    """105 x 105 x 8 nodes x 3 dof = 264,600 rows, 19,397,862 nnz: a plane
    spans 3 * 105^2 = 33,075 rows, beyond the int16 slice-relative form, so
    the SELL copy takes the stepped int16 form at W = 4 as full-size C4 does
    (profiles/r02g_configs.jsonl), including slices summed from the copy's
    sub-CSR (those straddling the first and last boundary planes)."""
    A = mpg.gen_stencil27(105, 3, ny=105, nz=8)
    assert A.nrows == 264_600 and A.nnz == 19_397_862
    return _problem(mpg, A)


@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("mixed", "mgs"), ("baseline", "cgs"), ("mixed", "cgsr")])
def test_c4_stepped_layout_live_oracle(mpg, oracle, c4_stepped, mode, orth):
    """C4's full-size SpMV layouts in whole solves against the live oracle:
    the stepped SELL copy (int16 columns, W = 4, CSR-summed boundary slices)
    and the node-block copy on the fused engine, and the operator surface
    (whose SELL copy is built by the same builder), asserting the layout the
    engine really ran."""
    A, xt, b = c4_stepped
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=100)
    eng = mpg.Engine(A, b, xt, spmv_format="sell", **opts)
    lay, cols = eng.spmv_layout(), eng.sell_columns()
    eng.close()
    assert lay["format"] == "sell" and lay["vec_width"] == 4 and lay["col_bytes"] == 2 and not lay["window"], lay
    assert cols["form"] == "stepped" and 1 <= cols["csr_slices"] <= A.nrows // 64 // 100, cols
    eng = mpg.Engine(A, b, xt, spmv_format="node", **opts)
    assert eng.spmv_layout()["format"] == "node" and eng.spmv_layout()["stored"] == A.nnz
    eng.close()
    ref = oracle.solve(mpg, A, b, xt, **opts)
    assert ref.status == "converged"
    for engine, fmt in (("fused", "sell"), ("fused", "node"), ("surface", "auto")):
        got = mpg.solve(A, b, xt, engine=engine, spmv_format=fmt, **opts)
        compare(as_ref(ref), got, mode, opts["tol"], 30, f"c4-stepped-{mode}-{orth}-{engine}-{fmt}")


def test_c4_full_size_spmv_sell_vs_csr_vs_mkl(hip, mpg, oracle):
    """One fp32 SpMV of full-size C4 (stencil27(111, 3): 4,102,893 rows,
    326,382,219 nnz) through the SELL copy (stepped int16, W = 4) against the
    CSR SpMV (the same fp64 row sums in CSR order: identical bits) and the
    oracle's mkl_sparse_s_mv (kernels_mkl.cpp:326-352; fp32 accumulation, so
    within 2 * row_nnz * eps32 * (|A| |x|)_i)."""
    import ctypes as C

    A = mpg.gen_stencil27(111, 3)
    n = A.nrows
    assert n == 4_102_893 and A.nnz == 326_382_219
    x = mpg.rand_vect(n, 7).astype(np.float32)
    v32 = A.val.astype(np.float32)
    drp, dci, dv, dx = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(v32), hip.buf(x)
    dy_sell, dy_csr = hip.buf(n, np.float32), hip.buf(n, np.float32)
    csr, sell = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, 1, dv.p, 0, C.byref(sell)))
        assert sell.value
        form, exc, imp = C.c_int32(), C.c_int64(), C.c_int64()
        hip.check(hip.lib.mpg_sell_columns(sell, C.byref(form), C.byref(exc), C.byref(imp)))
        w, cb, stored, win = C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32()
        hip.check(hip.lib.mpg_sell_layout(sell, C.byref(w), C.byref(cb), C.byref(stored), C.byref(win)))
        assert form.value == 2 and w.value == 4 and cb.value == 2 and exc.value >= 1, (form.value, w.value, exc.value)
        hip.call("mpg_sell_spmv_f32", sell, C.c_float(1.0), dx.p, C.c_float(0.0), dy_sell.p)
        hip.call("mpg_csr_spmv_f32", csr, C.c_float(1.0), dv.p, dx.p, C.c_float(0.0), dy_csr.p)
        y_sell, y_csr = dy_sell.get(), dy_csr.get()
        assert np.array_equal(y_sell, y_csr)
        y_mkl = oracle.spmv(A, x, dtype=np.float32)
        scale = oracle.spmv(mpg.Csr(n, n, A.rowptr, A.col, np.abs(v32).astype(np.float64)),
                            np.abs(x).astype(np.float64))
        row_nnz = np.diff(A.rowptr)
        eps32 = np.finfo(np.float32).eps
        bad = np.abs(y_sell.astype(np.float64) - y_mkl.astype(np.float64)) > 2 * row_nnz * eps32 * scale
        assert not bad.any(), np.flatnonzero(bad)[:10]
    finally:
        if sell.value:
            hip.lib.mpg_sell_destroy(sell)
        hip.lib.mpg_csr_destroy(csr)


def _restart_properties(got, rlen, floor_rel):
    """Size-independent checks of a restarted GMRES run with an fp64 outer
    residual: (1) within a cycle the Arnoldi residual |s(k+1)| never grows
    (GMRES minimises it over a growing space; fp32 rounding allowed); (2)
    the preconditioned true residual norm beta = ||M r|| (what GMRES with a
    left preconditioner minimises) never grows from one restart to the
    next; (3)
    each cycle's last Arnoldi residual predicts the next restart's true
    preconditioned residual (beta) while both sit above the fp32 floor."""
    s = np.asarray(got.step_res)
    cyc = np.asarray(got.step_cycle)
    for c in np.unique(cyc):
        sc = s[cyc == c]
        assert np.all(np.diff(sc) <= 1e-5 * sc[:-1]), f"cycle {c}: Arnoldi residual grew"
    beta = np.asarray(got.cyc_beta)
    assert np.all(np.diff(beta) <= 1e-5 * beta[:-1]), f"preconditioned residual grew: {beta}"
    for c in range(len(beta) - 1):
        last = s[cyc == c][-1]
        if beta[c + 1] > floor_rel * beta[0]:
            assert abs(last - beta[c + 1]) <= 0.05 * beta[c + 1], (c, last, beta[c + 1])


def test_c4_stencil27_full_size_properties(mpg):
    """C4 at its stated size on one GPU (111^3 nodes x 3 dof = 4,102,893
    rows, 326,382,219 nnz): mixed CGS GMRES(30), 4 cycles at tol = 0, the
    restart properties above, and the true residual of the returned x
    recomputed on the host."""
    A = mpg.gen_stencil27(111, 3)
    assert A.nrows == 4_102_893 and A.nnz == 326_382_219
    A, xt, b = _problem(mpg, A)
    got = mpg.solve(A, b, xt, engine="fused", mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0,
                    max_restarts=4)
    assert got.status == "aborted" and got.total_iters == 120
    _restart_properties(got, 30, 1e-5)
    r = b - mpg.host_spmv(A, got.x)
    assert abs(np.linalg.norm(r) - got.res_norm) <= 1e-6 * np.linalg.norm(b)
    assert got.res_norm < 1e-3 * np.linalg.norm(b)


def test_c5_band100m_half_values_full_size(mpg):
    """C5 at its stated size (BAND-100M: n = 1e7, 99,999,975 nnz) with fp16
    Arnoldi values, fp32 vectors and fp64 iterative refinement: converges to
    tol with the error bound of the 300k-row test, takes the restart path
    the fp32-value solve takes (±1), and satisfies the restart properties."""
    A, xt, b = _problem(mpg, mpg.gen_band(10_000_000, 5, 4, seed=7))
    assert A.nnz == 99_999_975
    opts = dict(engine="fused", orth="cgs", prec="identity", rlen=30, tol=1e-10, max_restarts=60)
    half = mpg.solve(A, b, xt, mode="mixed-half", **opts)
    assert half.status == "converged" and half.backward_error[-1] <= 1e-10
    assert half.err_norm <= 1e-6 * np.linalg.norm(xt)
    single = mpg.solve(A, b, xt, mode="mixed", **opts)
    assert single.status == "converged"
    assert abs(half.restarts - single.restarts) <= 1
    # (the fp16 Arnoldi matrix differs from A by ~5e-4 relative, so its
    # residual estimate does not predict the fp64 residual: property 3 off)
    _restart_properties(half, 30, 1.0)
