"""Parity rules between a GMRES run and the oracle / golden record.

Stated tolerances (the north-star's "within a stated fp tolerance"):

fp64 Arnoldi with an fp64 preconditioner (mode baseline):
  * same final status, same restart index i and total iteration count;
  * per-step Arnoldi residual |s(k+1)|, cycle 0:
        |Δ| <= 1e-8 |s_ref| + 1e-12 ||M^-1 b||
    later cycles: |Δ| <= 1e-5 |s_ref| + 1e-10 ||M^-1 b||;
  * per-restart backward error r/(||b|| + ||A||_F ||x||):
        |Δ| <= 1e-5 be_ref + 1e-15.
fp32 Arnoldi, or fp64 Arnoldi whose vectors pass through an fp32
preconditioner every step (modes mixed, single, mixed-half, single-prec):
  * same final status; restart index within ±1;
  * cycle-0 history |Δ| <= 1e-3 |s_ref| + 1e-5 ||M^-1 b||;
  * when converged, the final backward error is <= tol.
"""
import numpy as np


def _arr(x):
    return np.asarray(x, dtype=np.float64)


def compare(ref: dict, got, mode: str, tol: float, rlen: int, label: str = ""):
    fp64 = mode == "baseline"
    assert got.status == ref["status"], f"{label}: status {got.status} vs {ref['status']}"
    minvb = float(ref["minvb_norm"])
    s_ref, s_got = _arr(ref["step_res"]), _arr(got.step_res)
    cyc = np.asarray(got.step_cycle)
    be_ref = _arr(ref["cyc_r_norm"]) / _arr(ref["cyc_normalization"])
    be_got = _arr(got.cyc_r_norm) / _arr(got.cyc_normalization)
    if fp64:
        assert got.restarts == ref["restarts"], f"{label}: restarts {got.restarts} vs {ref['restarts']}"
        assert got.total_iters == ref["total_iters"], f"{label}: iters {got.total_iters} vs {ref['total_iters']}"
        assert len(s_got) == len(s_ref)
        c0 = cyc == 0
        d = np.abs(s_got - s_ref)
        assert np.all(d[c0] <= 1e-8 * s_ref[c0] + 1e-12 * minvb), f"{label}: cycle-0 history {d[c0].max():.3e}"
        assert np.all(d[~c0] <= 1e-5 * s_ref[~c0] + 1e-10 * minvb), f"{label}: history {d[~c0].max():.3e}"
        assert np.all(np.abs(be_got - be_ref) <= 1e-5 * be_ref + 1e-15), f"{label}: backward errors"
    else:
        assert abs(got.restarts - ref["restarts"]) <= 1, f"{label}: restarts {got.restarts} vs {ref['restarts']}"
        k = min(rlen, len(s_ref), len(s_got))
        d = np.abs(s_got[:k] - s_ref[:k])
        assert np.all(d <= 1e-3 * s_ref[:k] + 1e-5 * minvb), f"{label}: cycle-0 history {d.max():.3e}"
        if got.status == "converged":
            assert be_got[-1] <= tol, f"{label}: final backward error {be_got[-1]:.3e} > {tol}"


def as_ref(result) -> dict:
    """Turn a live oracle Result into the golden-record shape."""
    return dict(status=result.status, restarts=result.restarts, total_iters=result.total_iters,
                minvb_norm=result.minvb_norm, step_res=result.step_res, step_cycle=result.step_cycle,
                cyc_r_norm=result.cyc_r_norm, cyc_normalization=result.cyc_normalization,
                res_norm=result.res_norm, err_norm=result.err_norm)
