"""ORACLE — test infrastructure only.

Independent NumPy restatement of the reference's restarted GMRES(m), used to
cross-check the C++/MKL oracle (cpu_gmres.cpp) on small inputs. Pure
array arithmetic in the reference's precisions:
  gmres_baseline      gmres.cpp:24-133   (Type everywhere, M in PrecType)
  gmres_singleUpdate  gmres.cpp:135-245  (fp64 residual/update, fp32 cycle)
  CGS / MGS / CGSR    Orthogonalization.hpp:76-136
  first/add_vector    Orthogonalization.hpp:36-60 (reciprocal, then multiply)
  Givens              kernels_mkl.cpp:214-260 (reference-BLAS rotg, b := 0)
  Convergence (base)  IterUtil.hpp:17-81
  Jacobi              types.hpp:393-431
  ILU(0), ILU-Jacobi  kernels_mkl.cpp:416-500 (diag_inds filled), kernels.hpp:171-248
Only the base restart strategy is restated here. BLAS reductions use NumPy's
own summation order, so agreement with the MKL oracle is to round-off, not
bitwise.
"""
# Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
# University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
from __future__ import annotations

import numpy as np


def rotg(a, b, dt):
    a, b = dt(a), dt(b)
    roe = a if abs(a) > abs(b) else b
    scale = dt(abs(a) + abs(b))
    if scale == 0:
        return dt(0), dt(1), dt(0)
    r = dt(scale * np.sqrt(dt(a / scale) ** 2 + dt(b / scale) ** 2))
    r = r if roe >= 0 else -r
    return r, dt(a / r), dt(b / r)


def jacobi_diag(rowptr, col, val64, dt):
    n = len(rowptr) - 1
    v = val64.astype(dt)
    rows = np.add.reduceat(np.abs(v), rowptr[:-1]) if len(v) else np.zeros(n, dt)
    alpha = dt(np.max(rows).astype(dt) * dt(np.finfo(np.float32).eps))
    d = np.empty(n, dt)
    for i in range(n):
        j = rowptr[i]
        while j < rowptr[-1] - 1 and col[j] < i:
            j += 1
        a = v[j]
        d[i] = dt(1) / (max(a, alpha) if a >= 0 else min(a, -alpha))
    return d


def ilu0_factors(A, dt):
    """ILU(0) by the dictionary-of-rows IKJ form (an independent restatement
    of ilu0_impl, kernels_mkl.cpp:416-500, with diag_inds filled): rows 1..n-1,
    eliminations in increasing column order, pivots pushed to +-alpha with
    alpha = max row |sum| * eps(dt). Returns (L strict lower, U upper with
    the diagonal) as scipy CSR in dt."""
    import scipy.sparse as sp

    n = A.nrows
    rows = []
    for i in range(n):
        rows.append({int(c): float(v) for c, v in zip(A.col[A.rowptr[i]:A.rowptr[i + 1]],
                                                      A.val[A.rowptr[i]:A.rowptr[i + 1]])})
    alpha = max(sum(abs(v) for v in r.values()) for r in rows) * float(np.finfo(dt).eps)
    for i in range(1, n):
        ri = rows[i]
        for k in sorted(c for c in ri if c < i):
            f = ri[k] / rows[k][k]
            ri[k] = f
            for j, u in rows[k].items():
                if j > k and j in ri:
                    ri[j] -= f * u
        d = ri[i]
        ri[i] = (alpha if d < alpha else d) if d >= 0 else (-alpha if d > -alpha else d)
    lo, up = sp.lil_matrix((n, n)), sp.lil_matrix((n, n))
    for i, r in enumerate(rows):
        for j, v in r.items():
            (lo if j < i else up)[i, j] = v
    return lo.tocsr().astype(dt), up.tocsr().astype(dt)


def ilu_apply(Lo, Up, x, dt, kind="ilu", steps=1):
    """M^-1 x: exact unit-lower then upper solves, or `steps` Jacobi sweeps
    on each factor (ilusv_jacobi, kernels.hpp:219-248)."""
    from scipy.sparse.linalg import spsolve_triangular

    x = x.astype(dt)
    if kind == "ilu":
        n = Lo.shape[0]
        import scipy.sparse as sp

        y = spsolve_triangular((Lo + sp.identity(n, dtype=dt, format="csr")).astype(np.float64),
                               x.astype(np.float64), lower=True, unit_diagonal=True)
        return spsolve_triangular(Up.astype(np.float64), y, lower=False).astype(dt)
    b = x.copy()
    for _ in range(steps):
        t = (b - (x + (Lo @ x).astype(dt))).astype(dt)
        x = (x + t).astype(dt)
    b = x.copy()
    d = (dt(1) / Up.diagonal()).astype(dt)
    for _ in range(steps):
        t = (b - (Up @ x).astype(dt)).astype(dt)
        x = (x + d * t).astype(dt)
    return x


class _Problem:
    def __init__(self, A, dt):
        import scipy.sparse as sp
        self.A = sp.csr_matrix((A.val.astype(dt), A.col, A.rowptr), shape=(A.nrows, A.ncols))


def _orth(kind, V, k, w, h, dt):
    if kind == "mgs":
        for j in range(k + 1):
            h[j, k] = dt(np.dot(w, V[:, j]))
            w -= h[j, k] * V[:, j]
        return w
    Vk = V[:, : k + 1]
    h[: k + 1, k] = (Vk.T @ w).astype(dt)
    w = (w - Vk @ h[: k + 1, k]).astype(dt)
    if kind == "cgsr":
        c = (Vk.T @ w).astype(dt)
        w = (w - Vk @ c).astype(dt)
        h[: k + 1, k] += c
    return w


def _cycle(Aop, apply_m, w, m, orth, dt, minvb, history):
    """One Arnoldi cycle from the preconditioned residual w; returns (y, V, k)."""
    n = len(w)
    V = np.zeros((n, m + 1), dt, order="F")
    H = np.zeros((m + 1, m), dt, order="F")
    cs = np.zeros(m + 1, dt)
    sn = np.zeros(m + 1, dt)
    s = np.zeros(m + 1, dt)
    beta = dt(np.linalg.norm(w))
    V[:, 0] = (dt(1) / beta) * w if beta != 0 else 0
    s[0] = beta
    for k in range(m):
        w = apply_m(Aop(V[:, k]))
        w = _orth(orth, V, k, w.astype(dt), H, dt)
        hn = dt(np.linalg.norm(w))
        H[k + 1, k] = hn
        V[:, k + 1] = (dt(1) / hn) * w
        for j in range(k):
            a1, a2 = H[j, k], H[j + 1, k]
            H[j, k] = cs[j] * a1 + sn[j] * a2
            H[j + 1, k] = cs[j] * a2 - sn[j] * a1
        r, c, sv = rotg(H[k, k], H[k + 1, k], dt)
        H[k, k], H[k + 1, k], cs[k], sn[k] = r, 0, c, sv
        a1, a2 = s[k], s[k + 1]
        s[k] = c * a1 + sv * a2
        s[k + 1] = c * a2 - sv * a1
        history.append(abs(float(s[k + 1])))
    import scipy.linalg as sl
    y = sl.solve_triangular(H[:m, :m], s[:m], lower=False).astype(dt)
    return y, V


def solve(A, b, mode="mixed", orth="mgs", prec="identity", rlen=30, tol=1e-6, max_restarts=1000, jacobi_steps=1):
    """Returns dict(status, restarts, total_iters, cyc_r_norm, cyc_normalization, cyc_beta, step_res, x)."""
    n = A.nrows
    m = rlen
    T = np.float32 if mode in ("mixed", "single") else np.float64
    P = np.float32 if mode in ("mixed", "single", "single-prec") else np.float64
    d = jacobi_diag(A.rowptr, A.col, A.val, P) if prec == "jacobi" else None
    lu = ilu0_factors(A, P) if prec in ("ilu", "ilu_jacobi") else None

    def apply_m(v, into=T):
        if lu is not None:
            return ilu_apply(lu[0], lu[1], v.astype(P), P, prec, jacobi_steps).astype(into)
        if d is None:
            return v.astype(into)
        return (d * v.astype(P)).astype(into)

    # the solver matrix: fp32 values in mixed (inner) and in every baseline mode
    A32 = _Problem(A, np.float32).A
    A64 = _Problem(A, np.float64).A
    if mode == "mixed":
        Ain = A32
        Aout = A64
        X = np.float64
        a_norm = float(np.linalg.norm(A.val.astype(np.float32)))
        bb = b.astype(np.float64)
    else:
        Ain = A32.astype(T)
        Aout = Ain
        X = T
        a_norm = T(np.linalg.norm(Ain.data))
        bb = b.astype(T)
    x = np.zeros(n, X)
    b_norm = X(np.linalg.norm(bb))
    minvb = float(np.linalg.norm(apply_m(bb)))
    cyc_r, cyc_norm, cyc_beta, steps = [], [], [], []
    restarts = 0
    for i in range(10**9):
        r = (bb - Aout @ x).astype(X)
        w = r.astype(T)
        r_norm = float(np.linalg.norm(w)) if mode == "mixed" else float(X(np.linalg.norm(r)))
        w = apply_m(w)
        beta = float(T(np.linalg.norm(w)))
        x_norm = float(np.linalg.norm(x))
        normal = float(X(b_norm + X(a_norm) * X(x_norm))) if mode != "mixed" else b_norm + a_norm * x_norm
        cyc_r.append(r_norm)
        cyc_norm.append(normal)
        cyc_beta.append(beta)
        restarts += 1
        if restarts > max_restarts:
            status = "aborted"
            break
        if r_norm / normal <= tol:
            status = "converged"
            break
        y, V = _cycle(lambda v: (Ain @ v).astype(T), apply_m, w, m, orth, T, minvb, steps)
        inc = (V[:, :m] @ y).astype(T)
        x = (x + inc.astype(X)).astype(X)
    return dict(status=status, restarts=i, total_iters=len(steps), cyc_r_norm=np.array(cyc_r),
                cyc_normalization=np.array(cyc_norm), cyc_beta=np.array(cyc_beta), step_res=np.array(steps),
                x=x.astype(np.float64), minvb_norm=minvb)
