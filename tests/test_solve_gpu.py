"""End-to-end parity of GMRES on the MI355X against the golden records of the
CPU oracle (tests/golden/gmres_golden.json) and against the oracle run live
on the same inputs. Tolerances: tests/parity.py."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import inputs
from tests.parity import as_ref, compare

pytestmark = pytest.mark.gpu

GOLDEN = json.loads((Path(__file__).parent / "golden" / "gmres_golden.json").read_text())


@pytest.fixture(scope="module")
def mats(mpg):
    return inputs(mpg)


def _case_id(c):
    k = c["case"]
    return f"{k['matrix']}-{k['mode']}-{k['orth']}-{k['prec']}-m{k['rlen']}"


@pytest.mark.parametrize("engine", ["surface", "fused"])
@pytest.mark.parametrize("rec", GOLDEN["cases"], ids=_case_id)
def test_golden(mpg, mats, rec, engine):
    case = dict(rec["case"])
    A = mats[case.pop("matrix")]
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = mpg.solve(A, b, xt, engine=engine, **case)
    compare(rec, got, case["mode"], case["tol"], case["rlen"], _case_id(rec) + "/" + engine)


@pytest.mark.parametrize("engine", ["surface", "fused"])
@pytest.mark.parametrize("mode", ["mixed", "baseline"])
def test_live_oracle_band(mpg, oracle, engine, mode):
    """Larger input than the fixtures: BAND n=200k, GMRES(30), live oracle."""
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=1e-9, max_restarts=40)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    got = mpg.solve(A, b, xt, engine=engine, **opts)
    compare(as_ref(ref), got, mode, opts["tol"], 30, f"band200k-{mode}-{engine}")
    if mode == "baseline":  # same restart count -> comparable final residuals
        assert abs(got.res_norm - ref.res_norm) <= 0.5 * ref.res_norm + 1e-12 * np.linalg.norm(b)


@pytest.mark.parametrize("prec", ["identity", "jacobi"])
def test_mixed_half_values_converge(mpg, prec):
    """Low-precision cast path (BASELINE config 5): fp16 matrix values in the
    Arnoldi SpMV, fp32 vectors, fp64 residual/update. The reference has no
    fp16 mode, so parity is the final backward error <= tol."""
    A = mpg.gen_band(300_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = mpg.solve(A, b, xt, engine="fused", mode="mixed-half", orth="cgs", prec=prec, rlen=30, tol=1e-10,
                    max_restarts=100)
    assert got.status == "converged"
    assert got.backward_error[-1] <= 1e-10
    assert got.err_norm <= 1e-6 * np.linalg.norm(xt)


@pytest.mark.parametrize("engine", ["surface", "fused"])
def test_aborts_at_max_restarts(mpg, engine):
    """tol = 0 never converges: exactly max_restarts cycles of m steps, then abort
    at check_initial of the next cycle (IterUtil.hpp:43-45)."""
    A = mpg.gen_laplace3d(12)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = mpg.solve(A, b, xt, engine=engine, mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0,
                    max_restarts=3)
    assert got.status == "aborted"
    assert got.total_iters == 90 and len(got.step_res) == 90 and len(got.cyc_r_norm) == 4
