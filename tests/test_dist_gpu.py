"""The row-partitioned engine on one GPU: P ranks as threads with the
loopback communicator (device-to-device halo copies, rank-ordered fp64
all-reduce) must reproduce the single-GPU solve and the golden records
within the stated parity tolerances (tests/parity.py). The RCCL transport
differs only in how the same bytes move (exercised by bench.py at N > 1)."""
import json
import os
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import inputs
from tests.parity import as_ref, compare

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


@pytest.mark.parametrize("orth", ["cgs", "mgs"])
def test_rccl_single_rank_engine(mpg, orth):
    """The RCCL engine path (communicator init, captured all-reduces, empty
    halo) on one rank: the same history, solution and norms as the
    single-GPU engine (the rank's step program closes every step with its own
    Givens launch and all-reduces its partials in place, so the two run
    different kernel sequences on the same arithmetic)."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=4)
    plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
    eng = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, **opts)
    ran, done = eng.run(10)
    assert ran == 4 and done and eng.total_iters == 120
    dist_res = eng.report()
    eng.close()
    one = mpg.Engine(A, b, xt, **opts)
    ran1, done1 = one.run(10)
    assert ran1 == 4 and done1 and one.total_iters == 120
    one_res = one.report()
    one.close()
    ref = mpg.solve(A, b, xt, engine="fused", **opts)
    # the stepped engine reports what mpg_solve reports
    assert np.array_equal(one_res.step_res, ref.step_res) and np.array_equal(one_res.x, ref.x)
    assert one_res.res_norm == ref.res_norm and one_res.status == ref.status == "aborted"
    assert dist_res.status == "aborted" and dist_res.total_iters == 120 and len(dist_res.step_res) == 120
    assert np.allclose(dist_res.step_res, one_res.step_res, rtol=1e-5, atol=1e-9 * one_res.minvb_norm)
    assert np.allclose(dist_res.cyc_r_norm, one_res.cyc_r_norm, rtol=1e-5)
    assert np.allclose(dist_res.x, one_res.x, rtol=1e-5, atol=1e-9)
    assert abs(dist_res.res_norm - one_res.res_norm) <= 1e-4 * one_res.res_norm


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("mode,orth,prec", [("mixed", "cgs", "jacobi"), ("baseline", "mgs", "identity"),
                                            ("mixed", "cgsr", "identity")])
def test_host_transport_processes_match_loopback(mpg, oracle, tmp_path, nranks, mode, orth, prec):
    """The product's distributed engine as separate processes (one per rank,
    all on device 0, torch.distributed over gloo through the host transport
    of mpg_engine_create_dist_host). The transport sums the partials in rank
    order like the in-process loopback communicator, and the halo moves exact
    copies, so the multi-process solve must give the loopback solve's bits;
    both are checked against the oracle at the parity tolerances."""
    import subprocess
    import sys

    n, max_restarts, tol = 60_000, 40, 1e-9
    out = tmp_path / "rank0.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).parent / "dist_host_worker.py"),
           str(out), str(n), mode, orth, prec, str(max_restarts), str(tol)]
    run = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert run.returncode == 0, run.stdout[-3000:] + run.stderr[-3000:]
    got = np.load(out)
    assert str(got["transport_error"]) == ""
    A = mpg.gen_band(n, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec=prec, rlen=30, tol=tol, max_restarts=max_restarts)
    loop = mpg.solve_loopback(A, b, xt, nranks=nranks, **opts)
    assert np.array_equal(got["starts"], mpg.nnz_balanced_starts(A, nranks))
    assert list(got["counts"]) == [loop.restarts, loop.inner_k, loop.total_iters]
    assert str(got["status"]) == loop.status
    assert np.array_equal(got["step_res"], loop.step_res)
    assert np.array_equal(got["cyc_r_norm"], loop.cyc_r_norm)
    assert np.array_equal(got["x"], loop.x)
    assert got["norms"][0] == loop.res_norm and got["norms"][1] == loop.err_norm
    ref = oracle.solve(mpg, A, b, xt, **opts)
    compare(as_ref(ref), loop, mode, tol, 30, f"host-transport{nranks}")


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
