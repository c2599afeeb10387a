"""Per-kernel parity of the gfx950 HIP kernels (through the C-ABI) against
the CPU oracle (MKL semantics of kernels_mkl.cpp) and an fp64 NumPy
reference.

Tolerances (stated per kernel): the HIP reductions accumulate in fp64, so
fp32 results are within ~1 ulp of the exactly rounded value; MKL's fp32
reductions are not (their error grows with n), hence fp32 comparisons are
made against the fp64 reference with an ulp bound and against the oracle
with a looser relative bound. Elementwise kernels are bit-exact.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

F32_EPS = np.finfo(np.float32).eps
F64_EPS = np.finfo(np.float64).eps

SIZES = [0, 1, 63, 64, 65, 1000, 4097, 1_000_003]


def rng(seed=0):
    return np.random.default_rng(seed)


def assert_ulp(got, exp, scale, ulps=1):
    """|got - exp| <= ulps * ulp(scale), scale = |y| + |a x|: axpy may be
    contracted to one FMA (single rounding, as MKL's and cuBLAS's vector
    axpy), numpy rounds the product first; they differ by at most one
    rounding of the product."""
    exp = np.asarray(exp)
    assert np.all(np.abs(got - exp) <= ulps * np.spacing(np.abs(scale)))


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("t", ["f64", "f32"])
def test_dot_nrm2(hip, oracle, n, t):
    dt = np.float64 if t == "f64" else np.float32
    g = rng(n)
    x = g.uniform(-1, 1, n).astype(dt)
    y = g.uniform(-1, 1, n).astype(dt)
    dx, dy, out = hip.buf(x), hip.buf(y), hip.buf(2, dt)
    hip.call(f"mpg_dot_{t}", n, dx.p, dy.p, out.at(0))
    hip.call(f"mpg_nrm2_{t}", n, dx.p, out.at(1))
    got = out.get()
    ref_dot = float(np.dot(x.astype(np.longdouble), y.astype(np.longdouble)))
    ref_nrm = float(np.sqrt(np.sum(x.astype(np.longdouble) ** 2)))
    scale = float(np.sum(np.abs(x.astype(np.float64) * y)))
    if t == "f64":
        assert abs(got[0] - ref_dot) <= 1e-14 * max(scale, 1e-300) + 1e-300
        assert abs(got[1] - ref_nrm) <= 1e-14 * max(ref_nrm, 1e-300)
        if n:
            assert abs(got[0] - oracle.dot(x, y)) <= 1e-12 * max(scale, 1e-300)
            assert abs(got[1] - oracle.nrm2(x)) <= 1e-12 * ref_nrm
    else:
        # fp64 accumulation, one rounding: within 1 ulp (+ fp64 sum error)
        assert abs(got[0] - ref_dot) <= F32_EPS * abs(ref_dot) + 1e-13 * scale + 1e-38
        assert abs(got[1] - ref_nrm) <= F32_EPS * ref_nrm + 1e-38
        if n:
            assert abs(got[0] - oracle.dot(x, y)) <= 1e-5 * max(scale, 1e-30)
            assert abs(got[1] - oracle.nrm2(x)) <= 1e-5 * ref_nrm
    # host-result variants agree bit for bit with the device-result ones
    import ctypes as C

    hv = (C.c_double if t == "f64" else C.c_float)()
    hip.call(f"mpg_dot_{t}_host", n, dx.p, dy.p, C.byref(hv))
    assert dt(hv.value) == got[0]
    # nrm2 to the host: one launch on a 16-B aligned vector (last-workgroup
    # ticket, result stored into pinned memory), repeated so the ticket's
    # reset is exercised; the two-launch form on a vector that is not aligned
    for _ in range(3):
        hv.value = -1
        hip.call(f"mpg_nrm2_{t}_host", n, dx.p, C.byref(hv))
        assert dt(hv.value) == got[1]
    if n > 1:
        hip.call(f"mpg_nrm2_{t}", n - 1, dx.at(1), out.at(1))
        hip.call(f"mpg_nrm2_{t}_host", n - 1, dx.at(1), C.byref(hv))
        assert dt(hv.value) == out.get()[1]


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_blas1_elementwise(hip, t):
    dt = np.float64 if t == "f64" else np.float32
    n = 100_003
    g = rng(1)
    x = g.uniform(-1, 1, n).astype(dt)
    y = g.uniform(-1, 1, n).astype(dt)
    a = dt(0.7312)
    dx, dy, da = hip.buf(x), hip.buf(y), hip.buf(np.array([a], dt))
    hip.call(f"mpg_axpy_{t}", n, a, dx.p, dy.p)
    with np.errstate(all="ignore"):
        exp = (y + a * x).astype(dt)
    scale = (np.abs(y) + np.abs(a * x)).astype(dt)
    assert_ulp(dy.get(), exp, scale)
    dy2 = hip.buf(y)
    hip.call(f"mpg_naxpy_dev_{t}", n, da.p, dx.p, dy2.p)
    assert_ulp(dy2.get(), (y - a * x).astype(dt), scale)
    dy3 = hip.buf(y)
    hip.call(f"mpg_axpy_dev_{t}", n, da.p, dx.p, dy3.p)
    assert np.array_equal(dy3.get(), dy.get())
    dz = hip.buf(n, dt)
    hip.call(f"mpg_scal_copy_{t}", n, a, dx.p, dz.p)
    assert np.array_equal(dz.get(), (a * x).astype(dt))
    hip.call(f"mpg_scal_recip_copy_dev_{t}", n, da.p, dx.p, dz.p)
    assert np.array_equal(dz.get(), ((dt(1) / a) * x).astype(dt))
    hip.call(f"mpg_scal_{t}", n, a, dx.p)
    assert np.array_equal(dx.get(), (a * x).astype(dt))
    # gdmv: y = beta*y + alpha*d*x, in place (Jacobi apply)
    d = g.uniform(0.5, 2, n).astype(dt)
    dd, dw = hip.buf(d), hip.buf(y)
    hip.call(f"mpg_gdmv_{t}", n, dt(1), dd.p, dw.p, dt(0), dw.p)
    assert np.array_equal(dw.get(), (dt(0) * y + dt(1) * d * y).astype(dt))


def test_copy_casts_and_fill(hip):
    n = 5001
    x = rng(2).normal(size=n) * 1e3
    dx = hip.buf(x)
    d32, d64, d16 = hip.buf(n, np.float32), hip.buf(n, np.float64), hip.buf(n, np.uint16)
    hip.call("mpg_copy_f64f32", n, dx.p, d32.p)
    assert np.array_equal(d32.get(), x.astype(np.float32))
    hip.call("mpg_copy_f32f64", n, d32.p, d64.p)
    assert np.array_equal(d64.get(), x.astype(np.float32).astype(np.float64))
    hip.call("mpg_copy_f64f16", n, dx.p, d16.p)
    assert np.array_equal(d16.get().view(np.float16), x.astype(np.float16))
    # strided fill of a 7 x 5 block with lda 9
    blk = hip.buf(9 * 5, np.float64)
    hip.call("mpg_fill_f64", blk.p, 7, 5, 9, 2.5)
    got = blk.get().reshape(5, 9)
    assert np.all(got[:, :7] == 2.5) and np.all(got[:, 7:] == 0)


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_givens(hip, oracle, t):
    dt = np.float64 if t == "f64" else np.float32
    cases = [(3.0, 4.0), (-3.0, 4.0), (1e-3, -2.0), (0.0, 0.0), (5.0, 0.0), (0.0, -7.0), (1.5, 1.5)]
    for a, b in cases:
        buf = hip.buf(np.array([a, b, 0, 0], dt))
        hip.call(f"mpg_rotg_{t}", buf.at(0), buf.at(1), buf.at(2), buf.at(3))
        got = buf.get()
        ref = oracle.rotg(a, b, dt)
        tol = 4 * (F64_EPS if t == "f64" else F32_EPS)
        assert got[1] == 0
        assert np.allclose(got, ref, rtol=tol, atol=0), (a, b, got, ref)
    # column rotation: k previous rotations applied to a[0..k]
    k = 9
    g = rng(3)
    col = g.normal(size=k + 1).astype(dt)
    th = g.uniform(0, 2 * np.pi, k)
    c, s = np.cos(th).astype(dt), np.sin(th).astype(dt)
    dcol, dc, ds = hip.buf(col), hip.buf(c), hip.buf(s)
    hip.call(f"mpg_rot_vec_{t}", k, dcol.p, dc.p, ds.p)
    exp = col.copy()
    for j in range(k):
        a1, a2 = exp[j], exp[j + 1]
        exp[j] = dt(dt(c[j] * a1) + dt(s[j] * a2))
        exp[j + 1] = dt(dt(c[j] * a2) - dt(s[j] * a1))
    assert np.array_equal(dcol.get(), exp)


@pytest.mark.parametrize("t", ["f64", "f32"])
@pytest.mark.parametrize("rows,cols", [(1_000_000, 31), (100_003, 1), (5000, 40), (31, 31), (7, 3)])
def test_gemv_panels(hip, oracle, t, rows, cols):
    dt = np.float64 if t == "f64" else np.float32
    g = rng(rows + cols)
    lda = rows + (64 if rows > 64 else 0)
    Afull = np.zeros((lda, cols), dt, order="F")
    Afull[:rows] = g.uniform(-1, 1, (rows, cols))
    A = Afull[:rows]
    xT = g.uniform(-1, 1, rows).astype(dt)
    xN = g.uniform(-1, 1, cols).astype(dt)
    y0 = g.uniform(-1, 1, rows).astype(dt)
    dA = hip.buf(Afull.ravel(order="F"))
    dxT, dxN, dyT, dyN = hip.buf(xT), hip.buf(xN), hip.buf(cols, dt), hip.buf(y0)
    hip.call(f"mpg_gemv_{t}", 1, rows, cols, dt(1), dA.p, lda, dxT.p, dt(0), dyT.p)
    hip.call(f"mpg_gemv_{t}", 0, rows, cols, dt(-1), dA.p, lda, dxN.p, dt(1), dyN.p)
    A64 = A.astype(np.float64)
    refT = A64.T @ xT.astype(np.float64)
    refN = y0.astype(np.float64) - A64 @ xN.astype(np.float64)
    eps = F64_EPS if t == "f64" else F32_EPS
    scaleT = np.abs(A64).T @ np.abs(xT.astype(np.float64))
    scaleN = np.abs(y0) + np.abs(A64) @ np.abs(xN.astype(np.float64))
    assert np.all(np.abs(dyT.get() - refT) <= 2 * eps * np.abs(refT) + 1e-12 * scaleT)
    # fp64 sum of `cols` products, rounded to T, then y - t rounded again
    assert np.all(np.abs(dyN.get() - refN) <= (2 * eps + cols * F64_EPS) * scaleN)
    orefT = oracle.gemv(True, A, xT)
    assert np.allclose(dyT.get(), orefT, rtol=0, atol=(1e-12 if t == "f64" else 1e-5) * scaleT.max())


@pytest.mark.parametrize("t", ["f64", "f32"])
@pytest.mark.parametrize("n", [1, 2, 10, 30, 100])
def test_trsv_upper(hip, oracle, t, n):
    dt = np.float64 if t == "f64" else np.float32
    g = rng(n)
    ld = n + 1  # H(0:k, 0:k) inside an (m+1) x m array
    H = np.zeros((ld, n), dt, order="F")
    H[:n] = np.triu(g.uniform(-1, 1, (n, n))) + np.diag(g.uniform(2, 3, n))
    y = g.uniform(-1, 1, n).astype(dt)
    dH, dy = hip.buf(H.ravel(order="F")), hip.buf(y)
    hip.call(f"mpg_trsv_{t}", 1, 0, n, dH.p, ld, dy.p)
    got = dy.get()
    ref = oracle.trsv_upper(np.asfortranarray(H[:n]), y)
    tol = 64 * (F64_EPS if t == "f64" else F32_EPS)
    assert np.allclose(got, ref, rtol=tol, atol=tol)
    # lower and transposed forms against numpy
    L = np.asfortranarray(np.tril(g.uniform(-1, 1, (n, n))) + np.diag(g.uniform(2, 3, n))).astype(dt)
    for upper, trans, M in [(0, 0, L), (1, 1, np.asfortranarray(H[:n])), (0, 1, L)]:
        dM, dv = hip.buf(M.ravel(order="F")), hip.buf(y)
        hip.call(f"mpg_trsv_{t}", upper, trans, n, dM.p, n, dv.p)
        op = M.T if trans else M
        exp = np.linalg.solve(op.astype(np.float64), y.astype(np.float64))
        assert np.allclose(dv.get(), exp, rtol=1e3 * tol, atol=1e3 * tol)


def test_small_d2h_reads(hip, monkeypatch):
    """Small device -> host reads (<= 4 KiB: the kernel that stores into the
    pinned staging block for whole aligned words, the runtime copy otherwise)
    return the bytes written by the kernel just before them on the stream."""
    import ctypes as C

    n = 2048
    g = rng(7)
    for form in ("1", "0"):
        monkeypatch.setenv("MPG_D2H_KERNEL", form)
        for it in range(3):
            x = g.uniform(-1, 1, n).astype(np.float32)
            dx, dy = hip.buf(x), hip.buf(n, np.float32)
            hip.call("mpg_scal_copy_f32", n, 2.0, dx.p, dy.p)
            full = dy.get()
            assert np.array_equal(full, x * np.float32(2))
            for off, nbytes in ((0, 4), (0, 120), (4, 4096 - 4), (0, 4096), (1, 7), (2, 6), (0, 3), (12, 4097)):
                out = np.zeros(nbytes, np.uint8)
                hip.check(hip.lib.mpg_memcpy_d2h(hip.ctx, out.ctypes.data, C.c_void_p(dy.ptr.value + off), C.c_size_t(nbytes)),
                          "d2h")
                assert np.array_equal(out, full.view(np.uint8)[off:off + nbytes]), (form, off, nbytes)


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_trsv_wave_same_bits(hip, t, monkeypatch):
    """The one-wave LDS-staged trsv (n <= 64) against the workgroup form
    (MPG_TRSV_WAVE=0): the same bits in all four (upper, trans) forms, at
    n = 1 ... 64 and ld > n; n = 65 takes the workgroup form either way."""
    dt = np.float64 if t == "f64" else np.float32
    for n in (1, 2, 7, 30, 31, 63, 64, 65):
        g = rng(100 + n)
        ld = n + 3
        M = np.zeros((ld, n), dt, order="F")
        M[:n] = g.uniform(-1, 1, (n, n)) + np.diag(g.uniform(2, 3, n))
        y = g.uniform(-1, 1, n).astype(dt)
        y[n // 2] = 0  # a zero right-hand entry: the skipped update
        for upper in (1, 0):
            for trans in (0, 1):
                got = {}
                for wave in ("1", "0"):
                    monkeypatch.setenv("MPG_TRSV_WAVE", wave)
                    dM, dv = hip.buf(M.ravel(order="F")), hip.buf(y)
                    hip.call(f"mpg_trsv_{t}", upper, trans, n, dM.p, ld, dv.p)
                    got[wave] = dv.get()
                assert np.array_equal(got["1"].view(np.uint8), got["0"].view(np.uint8)), (n, upper, trans)
                tri = np.triu(M[:n]) if upper else np.tril(M[:n])
                op = (tri.T if trans else tri).astype(np.float64)
                exp = np.linalg.solve(op, y.astype(np.float64))
                tol = 1e3 * 64 * (F64_EPS if t == "f64" else F32_EPS)
                assert np.allclose(got["1"], exp, rtol=tol, atol=tol)


def _spmv_case(mpg, kind):
    if kind == "band":
        return mpg.gen_band(200_000, 5, 4, seed=11)
    if kind == "laplace":
        return mpg.gen_laplace3d(40, 30, 20)
    if kind == "longrows":  # rows longer than one LDS chunk + empty rows
        import scipy.sparse as sp

        g = rng(5)
        n = 3000
        dens = np.where(np.arange(n) % 500 == 0, 0.9, 0.003)
        rows, cols = [], []
        for i in range(n):
            if i % 777 == 5:
                continue  # empty row
            c = np.nonzero(g.random(n) < dens[i])[0]
            rows += [i] * len(c)
            cols += list(c)
        M = sp.csr_matrix((g.uniform(-1, 1, len(rows)), (rows, cols)), shape=(n, n))
        M.sort_indices()
        return mpg.Csr(n, n, M.indptr.astype(np.int32), M.indices.astype(np.int32), M.data.astype(np.float64))
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["band", "laplace", "longrows"])
def test_spmv(hip, mpg, oracle, kind):
    import ctypes as C

    A = _spmv_case(mpg, kind)
    n = A.nrows
    g = rng(7)
    x = g.uniform(-1, 1, n)
    y0 = g.uniform(-1, 1, n)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        S = A.to_scipy()
        absS = abs(S)
        # fp64: y = -A x + y0 (the residual form)
        dv, dx, dy = hip.buf(A.val), hip.buf(x), hip.buf(y0)
        hip.call("mpg_csr_spmv_f64", csr, -1.0, dv.p, dx.p, 1.0, dy.p)
        ref = y0 - S @ x
        scale = np.abs(y0) + absS @ np.abs(x)
        assert np.all(np.abs(dy.get() - ref) <= 4 * F64_EPS * scale)
        assert np.allclose(dy.get(), oracle.spmv(A, x, -1.0, 1.0, y0), rtol=0, atol=1e-13 * scale.max())
        # fp32: y = A x (Arnoldi form); fp64 accumulation, one rounding
        v32, x32 = A.val.astype(np.float32), x.astype(np.float32)
        dv32, dx32, dy32 = hip.buf(v32), hip.buf(x32), hip.buf(n, np.float32)
        hip.call("mpg_csr_spmv_f32", csr, np.float32(1), dv32.p, dx32.p, np.float32(0), dy32.p)
        S32 = S.copy()
        S32.data = v32.astype(np.float64)
        ref32 = S32 @ x32.astype(np.float64)
        sc32 = abs(S32) @ np.abs(x32.astype(np.float64))
        assert np.all(np.abs(dy32.get() - ref32) <= F32_EPS * np.abs(ref32) + 1e-14 * sc32)
        orc = oracle.spmv(A, x32, 1.0, 0.0, dtype=np.float32)
        assert np.allclose(dy32.get(), orc, rtol=0, atol=1e-5 * max(sc32.max(), 1e-30))
        # fp16 values, fp32 vectors
        v16 = A.val.astype(np.float16)
        dv16, dyh = hip.buf(v16.view(np.uint16)), hip.buf(n, np.float32)
        hip.call("mpg_csr_spmv_f16f32", csr, np.float32(1), dv16.p, dx32.p, np.float32(0), dyh.p)
        S16 = S.copy()
        S16.data = v16.astype(np.float64)
        ref16 = S16 @ x32.astype(np.float64)
        assert np.all(np.abs(dyh.get() - ref16) <= F32_EPS * np.abs(ref16) + 1e-14 * (abs(S16) @ np.abs(x32)))
    finally:
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("kind", ["band", "laplace", "longrows"])
def test_sell_spmv(hip, mpg, oracle, kind):
    """The SELL-64 copy (format 2: always, so the irregular longrows case is
    sliced too) against the CSR SpMV on the same inputs. Both sum in fp64 in
    CSR order and round once; for fp32/fp16 values the fp64 products are
    exact, so the results agree to the last bit. With fp64 values the SELL
    sum contracts product and add into one FMA while the CSR tile rounds the
    product it stages in LDS: a few ulps of the row's scale apart."""
    import ctypes as C

    A = _spmv_case(mpg, kind)
    n = A.nrows
    g = rng(9)
    x = g.uniform(-1, 1, A.ncols)
    y0 = g.uniform(-1, 1, n)
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    sells = []
    try:
        v32 = A.val.astype(np.float32)
        v16 = A.val.astype(np.float16).view(np.uint16)
        cases = [("f64", 0, A.val, np.float64, -1.0, 1.0), ("f32", 1, v32, np.float32, 1.0, 0.0),
                 ("f16f32", 2, v16, np.float32, 2.0, -0.5)]
        for name, vt, vals, xdt, alpha, beta in cases:
            dv = hip.buf(vals)
            sell = C.c_void_p()
            hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 2, C.byref(sell)))
            assert sell.value
            sells.append(sell)
            dx = hip.buf(x.astype(xdt))
            dy_sell, dy_csr = hip.buf(y0.astype(xdt)), hip.buf(y0.astype(xdt))
            hip.call(f"mpg_sell_spmv_{name}", sell, xdt(alpha), dx.p, xdt(beta), dy_sell.p)
            hip.call(f"mpg_csr_spmv_{name}", csr, xdt(alpha), dv.p, dx.p, xdt(beta), dy_csr.p)
            if name == "f64":
                scale = np.abs(y0) + abs(A.to_scipy()) @ np.abs(x)
                assert np.all(np.abs(dy_sell.get() - dy_csr.get()) <= 4 * F64_EPS * scale), name
            else:
                assert np.array_equal(dy_sell.get(), dy_csr.get()), name
        # format 0 declines the slices when padding would not pay
        auto = C.c_void_p()
        dv = hip.buf(A.val)
        hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, 0, dv.p, 0, C.byref(auto)))
        if kind == "longrows":
            assert not auto.value
        else:
            assert auto.value
            sells.append(auto)
    finally:
        for h in sells:
            hip.lib.mpg_sell_destroy(h)
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_jacobi_setup(hip, mpg, oracle, t):
    import ctypes as C

    dt = np.float64 if t == "f64" else np.float32
    A = mpg.gen_band(50_000, 3, 2, seed=3)
    A.val[::97] *= 1e-9  # tiny diagonals get boosted to eps*||A||_inf
    n = A.nrows
    drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, n, n, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        dv, dd = hip.buf(A.val.astype(dt)), hip.buf(n, dt)
        hip.call(f"mpg_jacobi_setup_{t}", csr, dv.p, dd.p)
        assert np.array_equal(dd.get(), oracle.jacobi(A, dt))
    finally:
        hip.lib.mpg_csr_destroy(csr)


class ScalarOp(C.Structure):
    """mpg_scalar_op (include/mpgmres/capi.h)"""
    _fields_ = [("op", C.c_int32), ("f64", C.c_int32), ("k", C.c_int32), ("reserved", C.c_int32),
                ("alpha", C.c_double), ("p", C.c_void_p * 4)]


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_scalar_program_matches_single_ops(hip, t):
    """One mpg_scalar_program launch runs the Givens step of an Arnoldi step
    (rot_vec over k earlier rotations, rotg, rot of s) plus a scalar copy and
    both scalar scal forms, with the same bits as the single-operator calls."""
    dt = np.float64 if t == "f64" else np.float32
    f64 = 1 if t == "f64" else 0
    k = 7
    g = rng(11)
    col0 = g.normal(size=k + 2).astype(dt)
    th = g.uniform(0, 2 * np.pi, k)
    c0, s0 = np.cos(th).astype(dt), np.sin(th).astype(dt)
    sv0 = np.zeros(k + 2, dt)
    sv0[k] = dt(g.normal())
    out = {}
    for how in ("program", "single"):
        # (dt zeros: np.append with Python ints promotes float32 to float64)
        col = hip.buf(np.concatenate([col0, np.zeros(1, dt)]))
        c, s = hip.buf(np.concatenate([c0, np.zeros(2, dt)])), hip.buf(np.concatenate([s0, np.zeros(2, dt)]))
        sv = hip.buf(sv0)
        rec, scal = hip.buf(np.zeros(3, dt)), hip.buf(np.array([dt(0.37)], dt))
        if how == "program":
            ops = (ScalarOp * 6)()
            specs = [(2, k, 0.0, [col.p, None, c.p, s.p]),
                     (0, 0, 0.0, [col.at(k), col.at(k + 1), c.at(k), s.at(k)]),
                     (1, 0, 0.0, [sv.at(k), sv.at(k + 1), c.at(k), s.at(k)]),
                     (3, 0, 0.0, [sv.at(k + 1), rec.at(0), None, None]),
                     (4, 0, 1.7, [rec.at(0), rec.at(1), None, None]),
                     (5, 0, 0.0, [rec.at(1), rec.at(2), scal.p, None])]
            for i, (op, kk, alpha, ps) in enumerate(specs):
                ops[i].op, ops[i].f64, ops[i].k, ops[i].alpha = op, f64, kk, alpha
                for j, q in enumerate(ps):
                    ops[i].p[j] = q.value if q is not None else None
            hip.check(hip.lib.mpg_scalar_program(hip.ctx, ops, 6), "mpg_scalar_program")
        else:
            hip.call(f"mpg_rot_vec_{t}", k, col.p, c.p, s.p)
            hip.call(f"mpg_rotg_{t}", col.at(k), col.at(k + 1), c.at(k), s.at(k))
            hip.call(f"mpg_rot_{t}", sv.at(k), sv.at(k + 1), c.at(k), s.at(k))
            hip.call(f"mpg_copy_{t}{t}", C.c_int64(1), sv.at(k + 1), rec.at(0))
            alpha = C.c_double(1.7) if t == "f64" else C.c_float(1.7)
            hip.call(f"mpg_scal_scalar_{t}", alpha, rec.at(0), rec.at(1))
            hip.call(f"mpg_scal_scalar_dev_{t}", scal.p, rec.at(1), rec.at(2))
        out[how] = [b.get() for b in (col, c, s, sv, rec)]
    for a, b in zip(out["program"], out["single"]):
        assert np.array_equal(a, b)
    assert out["program"][4][0] != 0
    with pytest.raises(RuntimeError):
        hip.check(hip.lib.mpg_scalar_program(hip.ctx, (ScalarOp * 9)(), 9), "too long")


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_scalar_program_rides_sell_spmv(hip, mpg, t):
    """mpg_sell_spmv_prog_*: the Givens program run by one extra workgroup of
    a SELL SpMV launch gives the bits of its own launch, and the SpMV's y the
    bits of the plain SpMV (the operator surface hands the next step's SpMV
    the queued program when their operands do not overlap)."""
    dt = np.float64 if t == "f64" else np.float32
    vt = 0 if t == "f64" else 1
    f64 = 1 if t == "f64" else 0
    A = mpg.gen_band(20_000, 5, 4, seed=3)
    g = rng(5)
    x, y0 = g.uniform(-1, 1, A.ncols).astype(dt), g.uniform(-1, 1, A.nrows).astype(dt)
    k = 11
    col0 = g.normal(size=k + 2).astype(dt)
    th = g.uniform(0, 2 * np.pi, k)
    c0, s0 = np.cos(th).astype(dt), np.sin(th).astype(dt)
    sv0 = np.zeros(k + 2, dt)
    sv0[k] = dt(g.normal())
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val.astype(dt))
    csr, sell = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 2, C.byref(sell)))
    out = {}
    try:
        for how in ("ride", "apart"):
            # (dt zeros: np.append with Python ints promotes float32 to float64)
            col = hip.buf(np.concatenate([col0, np.zeros(1, dt)]))
            c, s = hip.buf(np.concatenate([c0, np.zeros(2, dt)])), hip.buf(np.concatenate([s0, np.zeros(2, dt)]))
            sv = hip.buf(sv0)
            rec = hip.buf(np.zeros(1, dt))
            dx, dy = hip.buf(x), hip.buf(y0)
            ops = (ScalarOp * 4)()
            specs = [(2, k, [col.p, None, c.p, s.p]), (0, 0, [col.at(k), col.at(k + 1), c.at(k), s.at(k)]),
                     (1, 0, [sv.at(k), sv.at(k + 1), c.at(k), s.at(k)]), (3, 0, [sv.at(k + 1), rec.at(0), None, None])]
            for i, (op, kk, ps) in enumerate(specs):
                ops[i].op, ops[i].f64, ops[i].k, ops[i].alpha = op, f64, kk, 0.0
                for j, q in enumerate(ps):
                    ops[i].p[j] = q.value if q is not None else None
            if how == "ride":
                hip.call(f"mpg_sell_spmv_prog_{t}", sell, 1.0, dx.p, 0.5, dy.p, C.cast(ops, C.c_void_p), 4)
            else:
                hip.check(hip.lib.mpg_scalar_program(hip.ctx, ops, 4), "mpg_scalar_program")
                hip.call(f"mpg_sell_spmv_{t}", sell, 1.0, dx.p, 0.5, dy.p)
            out[how] = [b.get() for b in (col, c, s, sv, rec, dy)]
    finally:
        hip.lib.mpg_sell_destroy(sell)
        hip.lib.mpg_csr_destroy(csr)
    for a, b in zip(out["ride"], out["apart"]):
        assert np.array_equal(a, b)
    assert out["ride"][4][0] != 0


@pytest.mark.parametrize("t", ["f64", "f32"])
@pytest.mark.parametrize("which", ["band", "lap", "stencil27", "fem27"])
def test_sell_spmv_norm_matches_separate_launches(hip, mpg, t, which):
    """Round 5 (the operator surface's add_vector riding the next SpMV):
    mpg_sell_spmv_norm_* -- h = T(sqrt(sum of the ||w||^2 partials)),
    v = T(T(1)/h w), y = T(A v), workgroup 0 storing h before the riding
    Givens program that reads it -- gives the bits of mpg_scal_recip_nrm2_*
    followed by mpg_sell_spmv_prog_*, on every SELL kernel form: the
    two-slice window kernel (BAND), the two-slice gather kernel (7-point
    Laplacian), the stepped-int16 kernel with CSR-summed slices (27-point
    stencil) and int32 columns (fem27 forced to SELL)."""
    dt = np.float64 if t == "f64" else np.float32
    CT = C.c_double if t == "f64" else C.c_float
    vt = 0 if t == "f64" else 1
    f64 = 1 if t == "f64" else 0
    A = {"band": lambda: mpg.gen_band(20_000, 5, 4, seed=3), "lap": lambda: mpg.gen_laplace3d(30),
         "stencil27": lambda: mpg.gen_stencil27(105, 3, ny=105, nz=4), "fem27": lambda: mpg.gen_spec("fem27:16:3:70:13")}[which]()
    g = rng(23)
    n = A.nrows
    w = g.uniform(-1, 1, n).astype(dt)
    k = 7
    col0 = g.normal(size=k + 2).astype(dt)  # H(:,k); h = H(k+1,k) is written by the normalisation
    th = g.uniform(0, 2 * np.pi, k)
    c0, s0 = np.cos(th).astype(dt), np.sin(th).astype(dt)
    sv0 = np.zeros(k + 2, dt)
    sv0[k] = dt(g.normal())
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val.astype(dt))
    csr, sell = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    hip.check(hip.lib.mpg_sell_create(hip.ctx, csr, vt, dv.p, 2, C.byref(sell)))
    out = {}
    try:
        assert sell.value
        for how in ("ride", "apart", "ride-noprog", "apart-noprog"):
            # (dt zeros: np.append with Python ints promotes float32 to float64)
            col = hip.buf(np.concatenate([col0, np.zeros(1, dt)]))
            c, s = hip.buf(np.concatenate([c0, np.zeros(2, dt)])), hip.buf(np.concatenate([s0, np.zeros(2, dt)]))
            sv = hip.buf(sv0)
            rec = hip.buf(np.zeros(1, dt))
            dw, dvk, dy = hip.buf(w), hip.buf(n, dt), hip.buf(np.full(n, 7.0, dt))
            ops = (ScalarOp * 4)()
            specs = [(2, k, [col.p, None, c.p, s.p]), (0, 0, [col.at(k), col.at(k + 1), c.at(k), s.at(k)]),
                     (1, 0, [sv.at(k), sv.at(k + 1), c.at(k), s.at(k)]), (3, 0, [sv.at(k + 1), rec.at(0), None, None])]
            for i, (op, kk, ps) in enumerate(specs):
                ops[i].op, ops[i].f64, ops[i].k, ops[i].alpha = op, f64, kk, 0.0
                for j, q in enumerate(ps):
                    ops[i].p[j] = q.value if q is not None else None
            nops = 0 if how.endswith("noprog") else 4
            np_ = C.c_int32()
            hip.call(f"mpg_nrm2_partials_{t}", C.c_int64(n), dw.p, C.byref(np_))
            if how.startswith("ride"):
                hip.call(f"mpg_sell_spmv_norm_{t}", sell, np_, col.at(k + 1), dw.p, dvk.p, CT(1.0), dy.p,
                         C.cast(ops, C.c_void_p), nops)
            else:
                hip.call(f"mpg_scal_recip_nrm2_{t}", np_, col.at(k + 1), C.c_int64(n), dw.p, dvk.p)
                hip.call(f"mpg_sell_spmv_prog_{t}", sell, CT(1.0), dvk.p, CT(0.0), dy.p, C.cast(ops, C.c_void_p), nops)
            out[how] = [b.get() for b in (col, c, s, sv, rec, dvk, dy)]
    finally:
        hip.lib.mpg_sell_destroy(sell)
        hip.lib.mpg_csr_destroy(csr)
    for a, b in zip(out["ride"], out["apart"]):
        assert np.array_equal(a, b)
    for a, b in zip(out["ride-noprog"], out["apart-noprog"]):
        assert np.array_equal(a, b)
    h = np.sqrt(np.sum(w.astype(np.float64) ** 2))
    got_h = out["ride-noprog"][0][k + 1]
    assert abs(got_h - h) <= 1e-6 * h, (got_h, h, col0, out["ride-noprog"][0], out["apart-noprog"][0])
    assert out["ride"][4][0] != 0 and np.all(np.isfinite(out["ride"][6]))


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_split_reductions_match_one_call(hip, t):
    """Stage 1 / stage 2 split reductions and the consumers that fold stage 2
    in (the operator surface's deferred reductions) give the one-call forms'
    bits: nrm2 -> 1/h scal, dot -> naxpy, gemv^T -> gemv."""
    dt = np.float64 if t == "f64" else np.float32
    CT = C.c_double if t == "f64" else C.c_float
    g = rng(17)
    n = 300_001
    x, y = g.normal(size=n).astype(dt), g.normal(size=n).astype(dt)
    dx, dy = hip.buf(x), hip.buf(y)
    np_ = C.c_int32()
    # nrm2 -> scal_recip
    h1, h2 = hip.buf(1, dt), hip.buf(1, dt)
    o1, o2 = hip.buf(n, dt), hip.buf(n, dt)
    hip.call(f"mpg_nrm2_{t}", C.c_int64(n), dx.p, h1.p)
    hip.call(f"mpg_scal_recip_copy_dev_{t}", C.c_int64(n), h1.p, dx.p, o1.p)
    hip.call(f"mpg_nrm2_partials_{t}", C.c_int64(n), dx.p, C.byref(np_))
    hip.call(f"mpg_scal_recip_nrm2_{t}", np_, h2.p, C.c_int64(n), dx.p, o2.p)
    assert np.array_equal(h1.get(), h2.get()) and np.array_equal(o1.get(), o2.get())
    # dot -> naxpy
    a1, a2 = hip.buf(1, dt), hip.buf(1, dt)
    z1, z2 = hip.buf(y), hip.buf(y)
    hip.call(f"mpg_dot_{t}", C.c_int64(n), dx.p, dy.p, a1.p)
    hip.call(f"mpg_naxpy_dev_{t}", C.c_int64(n), a1.p, dx.p, z1.p)
    hip.call(f"mpg_dot_partials_{t}", C.c_int64(n), dx.p, dy.p, C.byref(np_))
    hip.call(f"mpg_naxpy_dot_{t}", np_, a2.p, C.c_int64(n), dx.p, z2.p)
    assert np.array_equal(a1.get(), a2.get()) and np.array_equal(z1.get(), z2.get())
    # gemv^T -> gemv on a padded panel (16-B quad form), and the finish form
    rows, cols = 200_000, 17
    lda = (rows + 63) // 64 * 64
    V = g.normal(size=(cols, lda)).astype(dt)
    w = g.normal(size=rows).astype(dt)
    dV, dw1, dw2 = hip.buf(V.ravel()), hip.buf(w), hip.buf(w)
    c1, c2, c3 = hip.buf(cols, dt), hip.buf(cols, dt), hip.buf(cols, dt)
    hip.call(f"mpg_gemv_{t}", 1, C.c_int64(rows), C.c_int64(cols), CT(1.0), dV.p, C.c_int64(lda), dw1.p, CT(0.0), c1.p)
    hip.call(f"mpg_gemv_{t}", 0, C.c_int64(rows), C.c_int64(cols), CT(-1.0), dV.p, C.c_int64(lda), c1.p, CT(1.0), dw1.p)
    hip.call(f"mpg_gemv_t_partials_{t}", C.c_int64(rows), C.c_int64(cols), dV.p, C.c_int64(lda), dw2.p, C.byref(np_))
    hip.call(f"mpg_gemv_t_finish_{t}", np_, C.c_int64(cols), CT(1.0), CT(0.0), c3.p)
    hip.call(f"mpg_gemv_n_from_t_{t}", C.c_int64(rows), C.c_int64(cols), CT(-1.0), dV.p, C.c_int64(lda), np_, CT(1.0),
             c2.p, CT(1.0), dw2.p)
    assert np.array_equal(c1.get(), c2.get()) and np.array_equal(c1.get(), c3.get())
    assert np.array_equal(dw1.get(), dw2.get())


@pytest.mark.parametrize("t", ["f64", "f32"])
@pytest.mark.parametrize("which", ["stencil27", "fem27", "fem27p"])
def test_node_spmv_matches_csr(hip, mpg, t, which):
    """mpg_node_spmv_* (one record per 3 x 3 block, node_tile.hpp) forms the
    CSR tile's fp64 products and sums each row in CSR storage order: the bits
    of mpg_csr_spmv_* for beta = 0 and beta != 0, at the default two tiles per
    workgroup and at one; a band matrix gets padded blocks only (the same
    bits), and alt_bytes decides when a copy is built (node_wins)."""
    dt = np.float64 if t == "f64" else np.float32
    CT = C.c_double if t == "f64" else C.c_float
    vt = 0 if t == "f64" else 1
    A = {"stencil27": lambda: mpg.gen_stencil27(30, 3), "fem27": lambda: mpg.gen_spec("fem27:24:3:70:13"),
         "fem27p": lambda: mpg.gen_spec("fem27:24:3:70:13:32:5")}[which]()
    g = rng(5)
    n = A.nrows
    x = g.uniform(-1, 1, n).astype(dt)
    y0 = g.uniform(-1, 1, n).astype(dt)
    drp, dci, dv, dx = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val.astype(dt)), hip.buf(x)
    csr, node = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(-1), C.byref(node)))
        assert node.value
        nb, nt, by, pad = C.c_int64(), C.c_int32(), C.c_int64(), C.c_int64()
        hip.check(hip.lib.mpg_node_layout(node, C.byref(nb), C.byref(nt), C.byref(by), C.byref(pad)))
        assert nb.value * 9 == A.nnz and nt.value >= nb.value // 256 and pad.value == 0
        assert by.value == nb.value * (80 if t == "f64" else 40) + 4 * (n // 3 + 1) + 8 * (nt.value + 1)
        for tpw in ("2", "1"):
            os.environ["MPG_NODE_TPW"] = tpw
            try:
                for alpha, beta in ((1.0, 0.0), (-1.5, 0.75)):
                    dyn, dyc = hip.buf(y0), hip.buf(y0)
                    hip.call(f"mpg_node_spmv_{t}", node, CT(alpha), dx.p, CT(beta), dyn.p)
                    hip.call(f"mpg_csr_spmv_{t}", csr, CT(alpha), dv.p, dx.p, CT(beta), dyc.p)
                    assert np.array_equal(dyn.get(), dyc.get()), (tpw, alpha, beta)
            finally:
                os.environ.pop("MPG_NODE_TPW", None)
        # alt_bytes: built only against a copy that streams more
        hip.lib.mpg_node_destroy(node)
        node = C.c_void_p()
        hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(by.value // 2), C.byref(node)))
        assert not node.value
        hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(by.value + 1), C.byref(node)))
        assert node.value
    finally:
        hip.lib.mpg_node_destroy(node)
        hip.lib.mpg_csr_destroy(csr)
    # a band (no node structure): only padded blocks, the CSR bits all the same, and never
    # built against the CSR arrays' bytes
    B = mpg.gen_band(3000, 5, 4, seed=7)
    drp, dci, dv = hip.buf(B.rowptr), hip.buf(B.col), hip.buf(B.val.astype(dt))
    dxb = hip.buf(g.uniform(-1, 1, B.nrows).astype(dt))
    csr, node = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, B.nrows, B.ncols, B.nnz, B.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    try:
        hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(-1), C.byref(node)))
        assert node.value
        nb, bb, pad = C.c_int64(), C.c_int64(), C.c_int64()
        hip.check(hip.lib.mpg_node_layout(node, C.byref(nb), None, C.byref(bb), C.byref(pad)))
        assert pad.value == 9 * nb.value - B.nnz > 0
        dyn, dyc = hip.buf(np.zeros(B.nrows, dt)), hip.buf(np.zeros(B.nrows, dt))
        hip.call(f"mpg_node_spmv_{t}", node, CT(1.0), dxb.p, CT(0.0), dyn.p)
        hip.call(f"mpg_csr_spmv_{t}", csr, CT(1.0), dv.p, dxb.p, CT(0.0), dyc.p)
        assert np.array_equal(dyn.get(), dyc.get())
        hip.lib.mpg_node_destroy(node)
        node = C.c_void_p()
        # (a 9-wide band pads 5 blocks per node row to 27 entries: 40 % zeros, yet in fp32 fewer
        # bytes than CSR -- auto weighs it against the SELL copy's implicit slices instead)
        hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(bb.value * 9 // 10), C.byref(node)))
        assert not node.value
    finally:
        hip.lib.mpg_node_destroy(node)
        hip.lib.mpg_csr_destroy(csr)


@pytest.mark.parametrize("t", ["f64", "f32"])
def test_isolated_short_rows_sum_in_csr_order(hip, t):
    """A short row that mpg_csr_create leaves alone in its row block (the next
    row is longer than a stream-mode tile, or it is the matrix's last row) is
    summed in CSR order like every other short row -- the order of the SELL
    and node-block copies -- not by the long-row tree. Rows of 50
    entries alternate with rows of 2100: every short row is isolated. The
    short rows' y equals a host restatement of the CSR tile bit for bit: each
    product rounded to fp64 (exact for fp32 operands), added in CSR order in
    fp64, then rounded to the vector type."""
    dt = np.float64 if t == "f64" else np.float32
    CT = C.c_double if t == "f64" else C.c_float
    g = rng(11)
    nrows, ncols = 41, 2100
    lens = [50 if r % 2 == 0 else 2100 for r in range(nrows)]
    rowptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.concatenate([np.sort(g.choice(ncols, L, replace=False)) for L in lens]).astype(np.int32)
    val = g.uniform(-1, 1, rowptr[-1]).astype(dt)
    x = g.uniform(-1, 1, ncols).astype(dt)
    drp, dci, dv, dx, dy = hip.buf(rowptr), hip.buf(col), hip.buf(val), hip.buf(x), hip.buf(np.zeros(nrows, dt))
    csr = C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, nrows, ncols, int(rowptr[-1]), rowptr.ctypes.data, drp.p, dci.p,
                                     C.byref(csr)))
    try:
        assert hip.lib.mpg_csr_num_blocks(csr) == nrows  # every row alone in its block
        hip.call(f"mpg_csr_spmv_{t}", csr, CT(1.0), dv.p, dx.p, CT(0.0), dy.p)
        y = dy.get()
    finally:
        hip.lib.mpg_csr_destroy(csr)
    for r in range(0, nrows, 2):
        acc = 0.0
        for j in range(rowptr[r], rowptr[r + 1]):
            acc += float(val[j]) * float(x[col[j]])
        assert y[r] == dt(acc), (r, y[r], dt(acc))


@pytest.mark.parametrize("t", ["f64", "f32"])
@pytest.mark.parametrize("which", ["stencil27", "fem27", "fem27p"])
def test_node_spmv_rides_match_separate_launches(hip, mpg, t, which):
    """Round 6: the operator surface's rides on the node-block
    copy. mpg_node_spmv_norm_* (h = T(sqrt(sum of the ||w||^2 partials)),
    v = T(T(1)/h w), y = T(A v), workgroup 0 storing h before the riding
    Givens program reads it) gives the bits of mpg_scal_recip_nrm2_* then
    mpg_node_spmv_prog_*, and mpg_node_spmv_prog_* the bits of
    mpg_scalar_program then mpg_node_spmv_* -- whose y is mpg_csr_spmv_*'s."""
    dt = np.float64 if t == "f64" else np.float32
    CT = C.c_double if t == "f64" else C.c_float
    vt = 0 if t == "f64" else 1
    f64 = 1 if t == "f64" else 0
    A = {"stencil27": lambda: mpg.gen_stencil27(30, 3), "fem27": lambda: mpg.gen_spec("fem27:24:3:70:13"),
         "fem27p": lambda: mpg.gen_spec("fem27:24:3:70:13:32:5")}[which]()
    g = rng(29)
    n = A.nrows
    w = g.uniform(-1, 1, n).astype(dt)
    k = 7
    col0 = g.normal(size=k + 2).astype(dt)
    th = g.uniform(0, 2 * np.pi, k)
    c0, s0 = np.cos(th).astype(dt), np.sin(th).astype(dt)
    sv0 = np.zeros(k + 2, dt)
    sv0[k] = dt(g.normal())
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val.astype(dt))
    csr, node = C.c_void_p(), C.c_void_p()
    hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.ncols, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    hip.check(hip.lib.mpg_node_create(hip.ctx, csr, vt, dv.p, C.c_int64(-1), C.byref(node)))
    out = {}
    try:
        assert node.value
        for how in ("norm", "norm-apart", "norm-noprog", "norm-noprog-apart", "prog", "prog-apart", "csr"):
            col = hip.buf(np.concatenate([col0, np.zeros(1, dt)]))
            c, s = hip.buf(np.concatenate([c0, np.zeros(2, dt)])), hip.buf(np.concatenate([s0, np.zeros(2, dt)]))
            sv = hip.buf(sv0)
            rec = hip.buf(np.zeros(1, dt))
            dw, dvk, dy = hip.buf(w), hip.buf(n, dt), hip.buf(np.full(n, 7.0, dt))
            ops = (ScalarOp * 4)()
            specs = [(2, k, [col.p, None, c.p, s.p]), (0, 0, [col.at(k), col.at(k + 1), c.at(k), s.at(k)]),
                     (1, 0, [sv.at(k), sv.at(k + 1), c.at(k), s.at(k)]), (3, 0, [sv.at(k + 1), rec.at(0), None, None])]
            for i, (op, kk, ps) in enumerate(specs):
                ops[i].op, ops[i].f64, ops[i].k, ops[i].alpha = op, f64, kk, 0.0
                for j, q in enumerate(ps):
                    ops[i].p[j] = q.value if q is not None else None
            nops = 0 if "noprog" in how else 4
            if how.startswith("norm"):
                np_ = C.c_int32()
                hip.call(f"mpg_nrm2_partials_{t}", C.c_int64(n), dw.p, C.byref(np_))
                if how.endswith("apart"):
                    hip.call(f"mpg_scal_recip_nrm2_{t}", np_, col.at(k + 1), C.c_int64(n), dw.p, dvk.p)
                    hip.call(f"mpg_node_spmv_prog_{t}", node, CT(1.0), dvk.p, CT(0.0), dy.p, C.cast(ops, C.c_void_p),
                             nops)
                else:
                    hip.call(f"mpg_node_spmv_norm_{t}", node, np_, col.at(k + 1), dw.p, dvk.p, CT(1.0), dy.p,
                             C.cast(ops, C.c_void_p), nops)
            elif how == "prog":
                hip.call(f"mpg_node_spmv_prog_{t}", node, CT(1.0), dw.p, CT(0.5), dy.p, C.cast(ops, C.c_void_p), 4)
            elif how == "prog-apart":
                hip.check(hip.lib.mpg_scalar_program(hip.ctx, ops, 4), "mpg_scalar_program")
                hip.call(f"mpg_node_spmv_{t}", node, CT(1.0), dw.p, CT(0.5), dy.p)
            else:  # the CSR SpMV of the normalised vector of the "norm" run
                dvn = hip.buf(out["norm"][5])
                hip.call(f"mpg_csr_spmv_{t}", csr, CT(1.0), dv.p, dvn.p, CT(0.0), dy.p)
            out[how] = [b.get() for b in (col, c, s, sv, rec, dvk, dy)]
    finally:
        hip.lib.mpg_node_destroy(node)
        hip.lib.mpg_csr_destroy(csr)
    for ride, apart in (("norm", "norm-apart"), ("norm-noprog", "norm-noprog-apart"), ("prog", "prog-apart")):
        for a, b in zip(out[ride], out[apart]):
            assert np.array_equal(a, b), (ride, apart)
    assert np.array_equal(out["csr"][6], out["norm"][6])
    h = np.sqrt(np.sum(w.astype(np.float64) ** 2))
    assert abs(out["norm-noprog"][0][k + 1] - h) <= 1e-6 * h
    assert out["norm"][4][0] != 0 and out["prog"][4][0] != 0
