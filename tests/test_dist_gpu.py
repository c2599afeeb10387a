"""The row-partitioned engine on one GPU: P ranks as threads with the
loopback communicator (device-to-device halo copies, rank-ordered fp64
all-reduce) must reproduce the single-GPU solve and the golden records
within the stated parity tolerances (tests/parity.py). The RCCL transport
differs only in how the same bytes move (exercised by bench.py at N > 1)."""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import inputs
from tests.parity import compare

pytestmark = pytest.mark.gpu

GOLDEN = json.loads((Path(__file__).parent / "golden" / "gmres_golden.json").read_text())
# (ILU factors the whole matrix: single-GPU only, tests/test_ilu_gpu.py)
PICK = [c for c in GOLDEN["cases"] if c["case"]["rlen"] == 30 and c["case"]["orth"] in ("cgs", "mgs", "cgsr")
        and c["case"]["prec"] in ("identity", "jacobi")]


@pytest.fixture(scope="module")
def mats(mpg):
    return inputs(mpg)


@pytest.mark.parametrize("fold", ["0", "1"], ids=["givens", "fold"])
@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("rec", PICK, ids=lambda c: "-".join(str(c["case"][k]) for k in ("matrix", "mode", "orth", "prec")))
def test_loopback_golden(mpg, mats, rec, nranks, fold, monkeypatch):
    monkeypatch.setenv("MPG_FOLD_GIVENS", fold)
    case = dict(rec["case"])
    A = mats[case.pop("matrix")]
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = mpg.solve_loopback(A, b, xt, nranks=nranks, **case)
    compare(rec, got, case["mode"], case["tol"], case["rlen"], f"loopback{nranks}")


def test_rccl_single_rank_engine(mpg):
    """The RCCL engine path (communicator init, captured all-reduces, empty
    halo) on one rank reproduces the single-GPU engine."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=4)
    plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
    eng = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, **opts)
    ran, done = eng.run(10)
    assert ran == 4 and done and eng.total_iters == 120
    eng.close()
    one = mpg.Engine(A, b, xt, **opts)
    ran1, done1 = one.run(10)
    assert ran1 == 4 and done1 and one.total_iters == 120
    one.close()


@pytest.mark.parametrize("nranks", [2, 4])
def test_loopback_matches_single_gpu_band(mpg, nranks):
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    one = mpg.solve(A, b, xt, engine="fused", **opts)
    many = mpg.solve_loopback(A, b, xt, nranks=nranks, **opts)
    assert many.status == one.status == "aborted" and many.total_iters == one.total_iters == 90
    # fp32 Arnoldi: partial sums combine in a different order across ranks
    assert np.allclose(many.step_res[:30], one.step_res[:30], rtol=1e-3, atol=1e-6 * one.minvb_norm)
    assert np.allclose(many.x, one.x, rtol=1e-3, atol=1e-5)
    assert abs(many.res_norm - one.res_norm) <= 1e-2 * one.res_norm
