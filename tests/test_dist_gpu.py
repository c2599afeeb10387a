"""The row-partitioned engine on one GPU: P ranks as threads with the
loopback communicator (device-to-device halo copies, rank-ordered fp64
all-reduce) must reproduce the single-GPU solve and the golden records
within the stated parity tolerances (tests/parity.py). The RCCL transport
differs only in how the same bytes move (exercised by bench.py at N > 1).

The 8-GPU configs (BASELINE C4, C5) are rehearsed at P = 8: the C4
stand-in's structure in the stepped-int16 layout against the oracle, BAND
with fp16 values against the oracle's fp32-value solve, and a BAND split at
1.25M rows per rank (C5's per-GPU share) through size-independent
properties. Each asserts per rank the SpMV layout and the front-halo
numbering it actually ran (mpg_solve_loopback_ex)."""
import json
import os
import re
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


def _assert_rank_layouts(lays, nranks, forms):
    assert len(lays) == nranks
    for q, L in enumerate(lays):
        assert L["format"] == "sell" and L["col_form"] in forms, (q, L)
        # the lower halo numbered in front of row 0 (dist.h): rank 0 has none
        assert (L["n_front"] == 0) == (q == 0), (q, L)
        assert L["n_ext"] > L["n_local"] or q == nranks - 1, (q, L)
    assert [L["row0"] for L in lays] == sorted(L["row0"] for L in lays)


@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("baseline", "mgs")])
def test_p8_stencil27_stepped_live_oracle(mpg, oracle, mode, orth):
    """BASELINE C4's structure (27-point, 3 dof, planes of 33,075 rows) split
    over P = 8 ranks: each rank's SELL copy keeps 2-byte columns (stepped
    int16, or int16 where a rank's span fits), against the oracle at the parity tolerances (Orthogonalization.hpp:82-88
    is where the dots become all-reduces)."""
    A = mpg.gen_stencil27(105, 3, ny=105, nz=8)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=100)
    lays = []
    # (SELL forced: auto may take the node-block copy on a rank whose rows
    # start on a node boundary, test_p8_stencil27_auto_node_ranks)
    got = mpg.solve_loopback(A, b, xt, nranks=8, layouts=lays, spmv_format="sell", **opts)
    # nnz-balanced ranks hold ~30k rows, under a plane (33,075): where the
    # compacted halo numbering brings a rank's neighbour offsets within
    # +-32767 its copy takes int16 columns, the others the stepped form
    _assert_rank_layouts(lays, 8, ("stepped", "int16"))
    assert any(L["col_form"] == "stepped" for L in lays), lays
    ref = oracle.solve(mpg, A, b, xt, **opts)
    assert ref.status == "converged"
    compare(as_ref(ref), got, mode, opts["tol"], 30, f"p8-stencil27-{mode}-{orth}")


def test_p8_stencil27_auto_node_ranks(mpg, oracle):
    """The same split on auto: each rank keeps whichever copy streams fewer
    bytes -- its stepped / int16 SELL copy, or the node-block copy where its
    rows start on a node boundary (3-dof nodes, halo triples kept whole by
    the compacted numbering) -- and the solve stays at oracle parity."""
    A = mpg.gen_stencil27(105, 3, ny=105, nz=8)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=1e-10, max_restarts=100)
    lays = []
    got = mpg.solve_loopback(A, b, xt, nranks=8, layouts=lays, **opts)
    for q, L in enumerate(lays):
        assert L["format"] in ("sell", "node"), (q, L)
        if L["format"] == "node":
            assert L["row0"] % 3 == 0 and L["n_local"] % 3 == 0, (q, L)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    compare(as_ref(ref), got, "mixed", opts["tol"], 30, "p8-stencil27-auto")


def test_p8_band_half_values_vs_oracle(mpg, oracle):
    """BASELINE C5's cast path (fp16 Arnoldi values, fp32 vectors, fp64 outer
    refinement) row-partitioned over P = 8: converges to tol like the oracle's
    fp32-value mixed solve (the reference has no fp16 mode), within one
    restart of it, with the forward error the fp64 refinement reaches."""
    n = 400_000
    A = mpg.gen_band(n, 5, 4, seed=7)
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(orth="cgs", prec="identity", rlen=30, tol=1e-10, max_restarts=60)
    lays = []
    half = mpg.solve_loopback(A, b, xt, nranks=8, layouts=lays, mode="mixed-half", **opts)
    _assert_rank_layouts(lays, 8, ("int16",))
    assert all(L["window"] and L["implicit_slices"] > 0 and L["half_rows_scaled"] == 0 for L in lays), lays
    ref = oracle.solve(mpg, A, b, xt, mode="mixed", **opts)
    assert ref.status == half.status == "converged"
    assert half.backward_error[-1] <= opts["tol"]
    assert abs(half.restarts - ref.restarts) <= 1, (half.restarts, ref.restarts)
    assert half.err_norm <= 1e-6 * np.linalg.norm(xt)
    one = mpg.solve(A, b, xt, engine="fused", mode="mixed-half", **opts)
    assert one.status == "converged" and abs(one.restarts - half.restarts) <= 1


def test_p8_band_c5_share_properties(mpg):
    """P = 8 ranks of 1.25M rows each (BAND-100M split as on 8 GPUs; every
    rank holds C5's per-GPU share): mixed CGS GMRES(30), 3 cycles at tol = 0.
    Cycle 0 matches the single-GPU solve to fp32 rounding, the restart
    properties hold, and the returned x's true residual recomputed on the
    host is the reported resNorm."""
    from tests.test_configs_gpu import _restart_properties

    n = 10_000_000
    A = mpg.gen_band(n, 5, 4, seed=7)
    assert A.nnz == 99_999_975
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    lays = []
    many = mpg.solve_loopback(A, b, xt, nranks=8, layouts=lays, **opts)
    _assert_rank_layouts(lays, 8, ("int16",))
    assert all(abs(L["n_local"] - n // 8) <= 64 for L in lays), [L["n_local"] for L in lays]
    assert many.status == "aborted" and many.total_iters == 90
    one = mpg.solve(A, b, xt, engine="fused", **opts)
    assert np.allclose(many.step_res[:30], one.step_res[:30], rtol=1e-3, atol=1e-6 * one.minvb_norm)
    _restart_properties(many, 30, 1e-5)
    r = b - mpg.host_spmv(A, many.x)
    assert abs(np.linalg.norm(r) - many.res_norm) <= 1e-6 * np.linalg.norm(b)


@pytest.mark.parametrize("fmt", ["sell", "auto"])
def test_host_transport_processes_stencil27(mpg, oracle, tmp_path, fmt):
    """The C4 structure as 2 separate processes over the host transport: the
    same bits as the 2-rank loopback solve, every rank on the stepped int16
    layout (sell) or on auto's choice (the ranks start on node boundaries, so
    the node-block copy is a candidate) with its lower halo numbered in
    front, and the oracle's result at the parity tolerances."""
    import subprocess
    import sys

    spec, mode, orth, prec, max_restarts, tol = "stencil27:105:105:8", "mixed", "cgs", "jacobi", 100, 1e-10
    out = tmp_path / "rank0.npz"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).parent / "dist_host_worker.py"),
           str(out), spec, mode, orth, prec, str(max_restarts), str(tol), fmt]
    run = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert run.returncode == 0, run.stdout[-3000:] + run.stderr[-3000:]
    got = np.load(out)
    assert str(got["transport_error"]) == ""
    lay = got["layouts"]  # per rank: [format (1 sell, 2 node), column form (2 stepped), CSR-summed slices, n_front]
    if fmt == "sell":
        assert list(lay[:, 0]) == [1, 1] and list(lay[:, 1]) == [2, 2], lay
    else:  # whichever copy streams fewer bytes (each rank's x fits an L2: strictly fewer)
        assert set(lay[:, 0]) <= {1, 2}, lay
    assert lay[0, 3] == 0 and lay[1, 3] > 0, lay
    A = mpg.gen_stencil27(105, 3, ny=105, nz=8)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec=prec, rlen=30, tol=tol, max_restarts=max_restarts)
    loop = mpg.solve_loopback(A, b, xt, nranks=2, spmv_format=fmt, **opts)
    assert list(got["counts"]) == [loop.restarts, loop.inner_k, loop.total_iters]
    assert np.array_equal(got["step_res"], loop.step_res) and np.array_equal(got["x"], loop.x)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    compare(as_ref(ref), loop, mode, tol, 30, "host-transport-stencil27")


def _two_width_band(mpg, n):
    """Rows [0, n/2) hold offsets -1..+1, rows [n/2, n) offsets -5..+4
    (diagonally dominant, the BAND value rule): nnz-balanced ranks then get
    very different row counts and SELL forms (rank 0 mixed widths, one slice
    per wave; rank 1 uniform, two slices per wave)."""
    rng = np.random.default_rng(5)
    rows, cols, vals = [], [], []
    for lo, hi, r0, r1 in ((1, 1, 0, n // 2), (5, 4, n // 2, n)):
        r = np.arange(r0, r1)
        for o in range(-lo, hi + 1):
            c = r + o
            ok = (c >= 0) & (c < n) & (o != 0)
            rows.append(r[ok]), cols.append(c[ok]), vals.append(-rng.random(ok.sum()))
    rr, cc, vv = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    diag = 1.0 + np.bincount(rr, weights=np.abs(vv), minlength=n)
    rr = np.concatenate([rr, np.arange(n)])
    cc = np.concatenate([cc, np.arange(n)])
    vv = np.concatenate([vv, diag])
    order = np.lexsort((cc, rr))
    rp = np.zeros(n + 1, np.int32)
    np.cumsum(np.bincount(rr, minlength=n), out=rp[1:])
    return mpg.Csr(n, n, rp, cc[order].astype(np.int32), vv[order].astype(np.float64))


@pytest.mark.parametrize("limit,folded", [("600", 0), ("4096", 1)], ids=["straddle", "both-pay"])
def test_fold_decision_is_collective(mpg, oracle, monkeypatch, limit, folded):
    """each rank used to decide the Givens fold from its own SpMV
    workgroup count, so ranks near the limit could run different collective
    sequences. With the limit between the two ranks' counts (~1,055 and ~254
    workgroups) and MPG_FOLD_GIVENS unset, every rank must take the same
    decision (the fold only where it pays on every rank) and the solve must
    match the oracle."""
    monkeypatch.delenv("MPG_FOLD_GIVENS", raising=False)
    monkeypatch.setenv("MPG_FOLD_MAX_GROUPS", limit)
    A = _two_width_band(mpg, 400_000)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    # fp64 Arnoldi: the strict rules (same counts, history to 1e-8). In mode
    # mixed this matrix's cycle-1 backward error is 45x smaller on the GPU than
    # on MKL, whose fp32 sgemv rounds every term, past the 3x rule
    opts = dict(mode="baseline", orth="cgs", prec="jacobi", rlen=30, tol=1e-12, max_restarts=60)
    lays = []
    got = mpg.solve_loopback(A, b, xt, nranks=2, layouts=lays, **opts)
    assert lays[0]["n_local"] > 1.8 * lays[1]["n_local"], lays
    assert [L["givens_folded"] for L in lays] == [folded, folded], lays
    ref = oracle.solve(mpg, A, b, xt, **opts)
    compare(as_ref(ref), got, "baseline", opts["tol"], 30, f"fold-collective-{limit}")


def _rccl_one_rank(mpg, A, b, xt, opts, cycles=10):
    plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
    eng = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, **opts)
    try:
        eng.run(cycles)
        return eng.report()
    finally:
        eng.close()


@pytest.mark.parametrize("orth", ["cgs", "mgs"])
def test_rccl_single_rank_bits(mpg, orth, monkeypatch):
    """at P = 1 the RCCL engine runs the single-GPU
    engine's kernels in the same order (the all-reduces and the empty halo are
    identities); the one difference is the panel kernels' partial count (256
    on ranks, so every rank all-reduces equal-length arrays, against
    ceil(n / 4096) on one GPU), which regroups the fp64 partial sums. With
    MPG_UNIFORM_GROUPS=1 the single-GPU engine takes the ranks' count, and
    the two solves are bit-identical."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=4)
    dist_res = _rccl_one_rank(mpg, A, b, xt, opts)
    monkeypatch.setenv("MPG_UNIFORM_GROUPS", "1")
    one = mpg.Engine(A, b, xt, **opts)
    one.run(10)
    one_res = one.report()
    one.close()
    assert dist_res.total_iters == one_res.total_iters == 120
    assert np.array_equal(dist_res.step_res, one_res.step_res)
    assert np.array_equal(dist_res.cyc_r_norm, one_res.cyc_r_norm)
    assert np.array_equal(dist_res.x, one_res.x)
    assert dist_res.res_norm == one_res.res_norm


def test_rccl_eager_matches_captured(mpg, monkeypatch):
    """The uncaptured RCCL path (MPG_NO_GRAPH=1: the same collectives issued
    eagerly, the fallback when capture is refused) gives the captured
    cycle's bits."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    cap = _rccl_one_rank(mpg, A, b, xt, opts)
    monkeypatch.setenv("MPG_NO_GRAPH", "1")
    eager = _rccl_one_rank(mpg, A, b, xt, opts)
    assert cap.total_iters == eager.total_iters == 90
    assert np.array_equal(cap.step_res, eager.step_res) and np.array_equal(cap.x, eager.x)
    assert cap.res_norm == eager.res_norm


def test_rccl_watchdog_names_rank_and_cycle(mpg, monkeypatch, capfd):
    """The RCCL wait is bounded: past MPG_COMM_TIMEOUT_S without completion
    (and a 5 s grace period) the communicator is aborted and mpg_engine_run
    fails (MPG_ERR_RCCL) naming the rank and the cycle. Work that completes
    within the grace period was slow, not hung: with the limit
    at 0 every cycle's wait expires at once, completes in the grace period,
    and the solve goes on with a warning naming the rank and the cycle --
    the same bits as an unwatched solve."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=3)
    plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
    ref = _rccl_one_rank(mpg, A, b, xt, opts)
    eng = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, **opts)
    try:
        monkeypatch.setenv("MPG_COMM_TIMEOUT_S", "0")
        ran, done = eng.run(10)
        got = eng.report()
    finally:
        eng.close()
    err = capfd.readouterr().err
    assert re.search(r"warning: rank 0 of 1: restart cycle \d+, waiting for .*no progress.*continuing", err), err
    assert done and got.total_iters == ref.total_iters == 90
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)


# ---- one process, one host thread per GPU, an RCCL clique (mpg_solve_multi_gpu; the CLI's --ngpus)


@pytest.mark.parametrize("orth", ["cgs", "mgs"])
def test_multi_gpu_one_rank_bits(mpg, orth, monkeypatch):
    """mpg_solve_multi_gpu at one GPU (ncclCommInitAll over one device, the
    rank on its own host thread) is the P = 1 RCCL engine, so with the
    ranks' partial count it is bit-identical to the single-GPU solve; the
    rank reports the communicator's own count (ncclCommCount = 1)."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    lay = []
    multi = mpg.solve_multi_gpu(A, b, xt, ngpus=1, layouts=lay, **opts)
    assert lay[0]["transport_ranks"] == 1 and lay[0]["device"] == 0 and lay[0]["n_local"] == A.nrows
    monkeypatch.setenv("MPG_UNIFORM_GROUPS", "1")
    one = mpg.solve(A, b, xt, engine="fused", **opts)
    assert multi.total_iters == one.total_iters == 90
    assert np.array_equal(multi.step_res, one.step_res) and np.array_equal(multi.x, one.x)
    assert multi.res_norm == one.res_norm and multi.gmres_seconds > 0


def test_multi_gpu_refuses_missing_or_repeated_devices(mpg):
    A = mpg.gen_band(20_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    have = mpg.device_count()
    with pytest.raises(RuntimeError, match=r"requested but %d visible" % have):
        mpg.solve_multi_gpu(A, b, xt, ngpus=have + 1, rlen=10, tol=0.0, max_restarts=1)
    with pytest.raises(RuntimeError, match="named twice"):
        mpg.solve_multi_gpu(A, b, xt, ngpus=2, devices=[0, 0], rlen=10, tol=0.0, max_restarts=1)


def test_engine_reports_rccl_ranks(mpg):
    """Engine.comm_ranks(): 1 on one GPU; the RCCL rank's ncclCommCount."""
    A = mpg.gen_band(50_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    e = mpg.Engine(A, b, xt, rlen=10, tol=0.0, max_restarts=2)
    try:
        assert e.comm_ranks() == 1
    finally:
        e.close()
    plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
    e = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, rlen=10, tol=0.0, max_restarts=2)
    try:
        assert e.comm_ranks() == 1
    finally:
        e.close()
