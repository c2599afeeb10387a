"""Stepped int16 SELL columns (sell_tile.hpp): a 7-point Laplacian on a
190 x 190 x 6 grid has column offsets of +-36,100, beyond the int16
slice-relative form, so its copy stores int16 offsets against one base per
(slice, step, element). A tridiagonal matrix with two far entries in one
slice (element 0 of one row 40,000 below its row, of the next 40,000 above)
spreads beyond 16 bits there, so that slice alone is summed from the CSR
arrays. Sums run in CSR
order with the same arithmetic in every form, so the stepped copy, the
int32 copy (MPG_SELL_STEPPED=0) and the CSR SpMV give the same bits for
fp32/fp16 values (fp64: the CSR tile's staged products, a few ulps), and
whole solves are bit-identical between the column forms and within the
parity tolerances of the oracle (tests/parity.py)."""
import ctypes as C

import numpy as np
import pytest

from tests.parity import as_ref, compare

pytestmark = pytest.mark.gpu
F64_EPS = np.finfo(np.float64).eps


def _wide(mpg):
    return mpg.gen_laplace3d(190, 190, 6)


def _far(mpg, n=200_000):
    """tridiagonal, diagonally dominant; row 64000 also reads column 24000,
    row 64001 holds only column 104001 (slice 1000: a spread of 80,000)"""
    rows = []
    for r in range(n):
        if r == 64001:
            rows.append([(104001, 0.5)])
            continue
        e = [(c, -1.0) for c in (r - 1, r + 1) if 0 <= c < n] + [(r, 4.0)]
        if r == 64000:
            e.append((24000, 0.25))
        rows.append(sorted(e))
    rp = np.zeros(n + 1, dtype=np.int32)
    rp[1:] = np.cumsum([len(x) for x in rows])
    col = np.array([c for x in rows for c, _ in x], dtype=np.int32)
    val = np.array([v for x in rows for _, v in x], dtype=np.float64)
    return mpg.Csr(n, n, rp, col, val)


@pytest.mark.parametrize("stepped", ["1", "0"])
@pytest.mark.parametrize("kind", ["wide", "far"])
def test_sell_stepped_columns_spmv(hip, mpg, stepped, kind, monkeypatch):
    monkeypatch.setenv("MPG_SELL_STEPPED", stepped)
    A = _wide(mpg) if kind == "wide" else _far(mpg)
    n = A.nrows
    g = np.random.default_rng(3)
    x = g.uniform(-1, 1, n)
    y0 = g.uniform(-1, 1, n)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    sells = []
    try:
        cases = [("f64", 0, A.val, np.float64, -1.0, 1.0), ("f32", 1, A.val.astype(np.float32), np.float32, 1.0, 0.0),
                 ("f16f32", 2, A.val.astype(np.float16).view(np.uint16), np.float32, 2.0, -0.5)]
        for name, vt, vals, xdt, alpha, beta in cases:
            dv = hip.buf(vals)
            sell = C.c_void_p()
            hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 0, C.byref(sell)))
            assert sell.value
            sells.append(sell)
            form, exc, imp = C.c_int32(), C.c_int64(), C.c_int64()
            hip.check(hip.lib.mpg_sell_columns(sell, C.byref(form), C.byref(exc), C.byref(imp)))
            if stepped == "1":
                assert form.value == 2 and exc.value == (0 if kind == "wide" else 1), (form.value, exc.value)
            else:
                assert form.value == 0
            dx = hip.buf(x.astype(xdt))
            dy_sell, dy_csr = hip.buf(y0.astype(xdt)), hip.buf(y0.astype(xdt))
            hip.call(f"mpg_sell_spmv_{name}", sell, xdt(alpha), dx.p, xdt(beta), dy_sell.p)
            hip.call(f"mpg_csr_spmv_{name}", csr, xdt(alpha), dv.p, dx.p, xdt(beta), dy_csr.p)
            if name == "f64":
                scale = np.abs(y0) + abs(A.to_scipy()) @ np.abs(x)
                assert np.all(np.abs(dy_sell.get() - dy_csr.get()) <= 4 * F64_EPS * scale), name
            else:
                assert np.array_equal(dy_sell.get(), dy_csr.get()), name
    finally:
        for h in sells:
            hip.lib.mpg_sell_destroy(h)
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("mode", ["mixed", "baseline", "mixed-half"])
def test_stepped_columns_solve(mpg, oracle, mode, monkeypatch):
    A = _wide(mpg)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=1e-9 if mode != "mixed-half" else 1e-6,
                max_restarts=25)
    got = {}
    for st in ("1", "0"):
        monkeypatch.setenv("MPG_SELL_STEPPED", st)
        eng = mpg.Engine(A, b, xt, spmv_format="sell", **opts)
        assert eng.spmv_layout()["col_bytes"] == (2 if st == "1" else 4)
        eng.close()
        got[st] = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
    s, i = got["1"], got["0"]
    assert s.status == i.status and s.total_iters == i.total_iters
    assert np.array_equal(s.step_res, i.step_res) and np.array_equal(s.x, i.x)
    if mode != "mixed-half":
        ref = oracle.solve(mpg, A, b, xt, **opts)
        compare(as_ref(ref), s, mode, opts["tol"], 30, f"stepped-{mode}")
    else:
        assert s.status == "converged" and s.backward_error[-1] <= opts["tol"]


@pytest.mark.parametrize("xcd", ["1", "0"])
def test_xcd_ordered_slices_match_oracle(mpg, oracle, xcd, monkeypatch):
    """XCD-ordered slices (MPG_SELL_XCD) only change which workgroup sums
    which rows: every row's sum is the same; the prologue's per-workgroup
    norm partials group differently (last-bit changes in the norms)."""
    monkeypatch.setenv("MPG_SELL_XCD", xcd)
    A = mpg.gen_laplace3d(60)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    for mode in ("baseline", "mixed"):
        opts = dict(mode=mode, orth="cgs", prec="identity", rlen=30, tol=1e-10, max_restarts=60)
        got = mpg.solve(A, b, xt, engine="fused", **opts)
        ref = oracle.solve(mpg, A, b, xt, **opts)
        compare(as_ref(ref), got, mode, opts["tol"], 30, f"xcd{xcd}-{mode}")


def test_stepped_exception_slice_solve(mpg, monkeypatch):
    """The fused engine's Arnoldi SpMV and residual prologue on a stepped copy
    with one CSR-summed slice: the same bits as the int32 copy."""
    A = _far(mpg)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    for mode in ("mixed", "baseline"):
        opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
        got = {}
        for st in ("1", "0"):
            monkeypatch.setenv("MPG_SELL_STEPPED", st)
            got[st] = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
        assert got["1"].total_iters == got["0"].total_iters == 90
        assert np.array_equal(got["1"].step_res, got["0"].step_res) and np.array_equal(got["1"].x, got["0"].x)


@pytest.mark.parametrize("implicit", ["1", "0"])
def test_implicit_slices_spmv(hip, mpg, implicit, monkeypatch):
    """Implicit slices (every row of the slice with the same column offsets:
    all but the first and last slice of a banded matrix) read no columns;
    their sums are the CSR sums in CSR order, so fp32/fp16 results equal the
    CSR SpMV's bits and the copy without implicit slices gives the same bits
    in every precision."""
    monkeypatch.setenv("MPG_SELL_IMPLICIT", implicit)
    A = mpg.gen_band(200_000, 5, 4, seed=11)
    n = A.nrows
    g = np.random.default_rng(5)
    x = g.uniform(-1, 1, n)
    y0 = g.uniform(-1, 1, n)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    sells = []
    try:
        cases = [("f64", 0, A.val, np.float64, -1.0, 1.0), ("f32", 1, A.val.astype(np.float32), np.float32, 1.0, 0.0),
                 ("f16f32", 2, A.val.astype(np.float16).view(np.uint16), np.float32, 2.0, -0.5)]
        for name, vt, vals, xdt, alpha, beta in cases:
            dv = hip.buf(vals)
            sell = C.c_void_p()
            hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 0, C.byref(sell)))
            sells.append(sell)
            form, exc, imp = C.c_int32(), C.c_int64(), C.c_int64()
            hip.check(hip.lib.mpg_sell_columns(sell, C.byref(form), C.byref(exc), C.byref(imp)))
            assert form.value == 1 and imp.value == (n // 64 - 2 if implicit == "1" else 0), imp.value
            dx = hip.buf(x.astype(xdt))
            dy_sell, dy_csr = hip.buf(y0.astype(xdt)), hip.buf(y0.astype(xdt))
            hip.call(f"mpg_sell_spmv_{name}", sell, xdt(alpha), dx.p, xdt(beta), dy_sell.p)
            hip.call(f"mpg_csr_spmv_{name}", csr, xdt(alpha), dv.p, dx.p, xdt(beta), dy_csr.p)
            if name == "f64":
                scale = np.abs(y0) + abs(A.to_scipy()) @ np.abs(x)
                assert np.all(np.abs(dy_sell.get() - dy_csr.get()) <= 4 * F64_EPS * scale), name
            else:
                assert np.array_equal(dy_sell.get(), dy_csr.get()), name
    finally:
        for h in sells:
            hip.lib.mpg_sell_destroy(h)
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("mode", ["mixed", "baseline", "mixed-half"])
@pytest.mark.parametrize("orth", ["cgs", "mgs"])
def test_implicit_slices_solve(mpg, mode, orth, monkeypatch):
    """The fused engine's Arnoldi SpMV and residual prologue with and without
    implicit slices: the same bits."""
    A = mpg.gen_band(120_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    got = {}
    for imp in ("1", "0"):
        monkeypatch.setenv("MPG_SELL_IMPLICIT", imp)
        got[imp] = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
    assert got["1"].total_iters == got["0"].total_iters == 90
    assert np.array_equal(got["1"].step_res, got["0"].step_res) and np.array_equal(got["1"].x, got["0"].x)
    assert got["1"].res_norm == got["0"].res_norm


def test_sell_copy_owns_its_flagged_rows(hip, mpg):
    """mpg_sell_create's copy owns every byte it reads (capi.h): the flagged
    slices of a stepped copy are summed from the copy's own sub-CSR, so the
    caller may overwrite and free the CSR arrays, the CSR handle and the value
    array once the copy exists (the copy used to borrow them)."""
    A = _far(mpg)
    n = A.nrows
    g = np.random.default_rng(9)
    x = g.uniform(-1, 1, n)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    cases = [("f64", 0, A.val, np.float64), ("f32", 1, A.val.astype(np.float32), np.float32),
             ("f16f32", 2, A.val.astype(np.float16).view(np.uint16), np.float32)]
    sells, want, dvs = [], [], []
    try:
        for name, vt, vals, xdt in cases:
            dv = hip.buf(vals)
            dvs.append(dv)
            sell = C.c_void_p()
            hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 0, C.byref(sell)))
            sells.append(sell)
            form, exc, imp = C.c_int32(), C.c_int64(), C.c_int64()
            hip.check(hip.lib.mpg_sell_columns(sell, C.byref(form), C.byref(exc), C.byref(imp)))
            assert form.value == 2 and exc.value == 1
            dx, dy = hip.buf(x.astype(xdt)), hip.buf(n, xdt)
            hip.call(f"mpg_csr_spmv_{name}", csr, xdt(1.0), dv.p, dx.p, xdt(0.0), dy.p)
            want.append(dy.get())
        # poison, then free, everything the copies were built from
        hip.check(hip.lib.mpg_memcpy_h2d(hip.ctx, dci.p, np.full(A.nnz, 7, np.int32).ctypes.data, A.nnz * 4), "h2d")
        hip.check(hip.lib.mpg_memcpy_h2d(hip.ctx, drp.p, np.zeros(n + 1, np.int32).ctypes.data, (n + 1) * 4), "h2d")
        for dv in dvs:
            junk = np.full(dv.nbytes, 0xFF, np.uint8)  # NaN in every precision
            hip.check(hip.lib.mpg_memcpy_h2d(hip.ctx, dv.p, junk.ctypes.data, dv.nbytes), "h2d")
        hip.sync()
        hip.lib.mpg_csr_destroy(csr)
        csr = None
        for dv in dvs:
            dv.free()
        dci.free()
        drp.free()
        for (name, _, _, xdt), sell, y in zip(cases, sells, want):
            dx, dy = hip.buf(x.astype(xdt)), hip.buf(n, xdt)
            hip.call(f"mpg_sell_spmv_{name}", sell, xdt(1.0), dx.p, xdt(0.0), dy.p)
            got = dy.get()
            if name == "f64":
                scale = abs(A.to_scipy()) @ np.abs(x)
                assert np.all(np.abs(got - y) <= 4 * F64_EPS * scale), name
            else:
                assert np.array_equal(got, y), name
    finally:
        for h in sells:
            hip.lib.mpg_sell_destroy(h)
        if csr is not None:
            hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("kind", ["lap", "wide", "stencil27"])
def test_shared_column_blocks_same_bits(mpg, kind, monkeypatch):
    """Slices whose 2-byte column blocks are identical keep one block
    (SellCopy::coff): most slices of a stencil share. Every slice still
    decodes with its own first row (and bases, stepped form), so the fused
    solve gives the same bits as with every block stored (MPG_SELL_SHARE=0)."""
    A = {"lap": lambda: mpg.gen_laplace3d(60), "wide": lambda: _wide(mpg),
         "stencil27": lambda: mpg.gen_stencil27(105, 3, ny=105, nz=4)}[kind]()
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = {}
    for sh in ("1", "0"):
        monkeypatch.setenv("MPG_SELL_SHARE", sh)
        for mode in ("mixed", "baseline"):
            opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3, spmv_format="sell")
            eng = mpg.Engine(A, b, xt, **opts)
            cols = eng.sell_columns()
            eng.close()
            # (implicit slices read a pattern, not a block: they neither store nor share one)
            stored = -(-A.nrows // 64) - cols["implicit_slices"]
            shared = cols["shared_slices"]
            assert (shared > stored // 2) if sh == "1" else shared == 0, (kind, sh, shared, stored)
            got[sh, mode] = mpg.solve(A, b, xt, engine="fused", **opts)
    for mode in ("mixed", "baseline"):
        a, c = got["1", mode], got["0", mode]
        assert a.total_iters == c.total_iters == 90
        assert np.array_equal(a.step_res, c.step_res) and np.array_equal(a.x, c.x), mode


def test_shared_column_blocks_surface_spmv(hip, mpg, monkeypatch):
    """The stand-alone SELL SpMV (operator surface) on a copy with shared
    column blocks: the CSR SpMV's bits (fp32 values)."""
    import ctypes as C

    A = mpg.gen_laplace3d(50)
    n = A.nrows
    x = np.random.default_rng(2).uniform(-1, 1, n).astype(np.float32)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr, sell = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        dv = hip.buf(A.val.astype(np.float32))
        hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, 1, dv.p, 0, C.byref(sell)))
        assert hip.lib.mpg_sell_shared_slices(sell) > (n // 64) // 2
        dx, y1, y2 = hip.buf(x), hip.buf(n, np.float32), hip.buf(n, np.float32)
        hip.call("mpg_sell_spmv_f32", sell, C.c_float(1.0), dx.p, C.c_float(0.0), y1.p)
        hip.call("mpg_csr_spmv_f32", csr, C.c_float(1.0), dv.p, dx.p, C.c_float(0.0), y2.p)
        assert np.array_equal(y1.get(), y2.get())
    finally:
        if sell.value:
            hip.lib.mpg_sell_destroy(sell)
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("kind,mode", [("lap", "mixed"), ("lap", "baseline"), ("band", "mixed"),
                                       ("band", "mixed-half")])
def test_sell_schedules_same_bits(mpg, kind, mode, monkeypatch):
    """The SELL step kernel's schedules are the same sums in the same order:
    two slices per wave (k_step_sell2, 8- or exact 10-entry batches) or one
    (MPG_SELL_PAIR=0), computed or loaded slice offsets (MPG_SELL_UNIFORM),
    the first batch gathered before or after the fold's scale is known
    (MPG_SELL_PREGATHER). Every combination gives the fused solve's bits."""
    # (n a multiple of 64: every slice as wide, so the pair kernel applies)
    A = mpg.gen_laplace3d(48) if kind == "lap" else mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=3, spmv_format="sell")
    runs = {}
    for pair, uni, pg in (("1", "1", "1"), ("1", "1", "0"), ("0", "1", "1"), ("0", "0", "1")):
        monkeypatch.setenv("MPG_SELL_PAIR", pair)
        monkeypatch.setenv("MPG_SELL_UNIFORM", uni)
        monkeypatch.setenv("MPG_SELL_PREGATHER", pg)
        eng = mpg.Engine(A, b, xt, **opts)
        lay = eng.spmv_layout()
        eng.close()
        assert lay["format"] == "sell" and lay["slices_per_wave"] == (2 if pair == "1" else 1), lay
        runs[pair, uni, pg] = mpg.solve(A, b, xt, engine="fused", **opts)
    ref = runs["1", "1", "1"]
    assert ref.total_iters == 90
    for key, r in runs.items():
        assert np.array_equal(r.step_res, ref.step_res) and np.array_equal(r.x, ref.x), key


@pytest.mark.parametrize("stepped", ["1", "0"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "mixed-half"])
def test_pipelined_batches_same_bits(mpg, stepped, mode, monkeypatch):
    """The software-pipelined batch loop of the one-slice-per-wave SpMV
    (MPG_SELL_PIPE: batch q's gathers, then batch q + U's loads) sums the
    same operands in the same order as the plain loop: the same solve bits,
    on stepped and int32 columns, with and without a CSR-summed slice."""
    monkeypatch.setenv("MPG_SELL_STEPPED", stepped)
    for make in (_wide, _far):
        A = make(mpg)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
        got = {}
        for pipe in ("1", "0"):
            monkeypatch.setenv("MPG_SELL_PIPE", pipe)
            got[pipe] = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
        p, q = got["1"], got["0"]
        assert p.total_iters == q.total_iters == 90
        assert np.array_equal(p.step_res, q.step_res) and np.array_equal(p.x, q.x)
