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


# (engine, storage, environment): the fused engine on both Arnoldi SpMV
# storages (CSR row blocks, SELL-64);: MPG_SELL_WINDOW=0 gathers v_k from memory
# instead of the LDS window; the others are launch-count experiments
FLAGS = ("MPG_SURFACE_GRAPH", "MPG_SURFACE_BATCH", "MPG_SURFACE_FUSE", "MPG_COMBINE", "MPG_FOLD_GIVENS", "MPG_CGS_PARTIALS", "MPG_SELL_WINDOW", "MPG_SURFACE_SELL", "MPG_FUSE_DOTS")
ON_BY_DEFAULT = ("MPG_SELL_WINDOW", "MPG_SURFACE_SELL")
ENGINES = {"surface": ("surface", "auto", {}), "surface-eager": ("surface", "auto", {"MPG_SURFACE_GRAPH": "0", "MPG_SURFACE_BATCH": "0",
                                                 "MPG_SURFACE_FUSE": "0"}),
           "surface-csr": ("surface", "auto", {"MPG_SURFACE_SELL": "0"}),
           "fused-csr": ("fused", "csr", {}),
           "fused-sell": ("fused", "sell", {}), "fused-gather": ("fused", "sell", {"MPG_SELL_WINDOW": "0"}),
           "fused-fold": ("fused", "auto", {"MPG_FOLD_GIVENS": "1"}),
           "fused-combine": ("fused", "auto", {"MPG_COMBINE": "1"}),
           "fused-cgspart": ("fused", "auto", {"MPG_CGS_PARTIALS": "1"}),
           "fused-dots": ("fused", "sell", {"MPG_CGS_PARTIALS": "1", "MPG_FUSE_DOTS": "1"}),
           "fused-dots-fold": ("fused", "sell", {"MPG_CGS_PARTIALS": "1", "MPG_FUSE_DOTS": "1",
                                                 "MPG_FOLD_GIVENS": "1"})}


def _engine(monkeypatch, engine):
    eng, fmt, env = ENGINES[engine]
    for f in FLAGS:
        monkeypatch.setenv(f, env.get(f, "1" if f in ON_BY_DEFAULT else "0"))
    return dict(engine=eng, spmv_format=fmt)


@pytest.mark.parametrize("engine", list(ENGINES))
@pytest.mark.parametrize("rec", GOLDEN["cases"], ids=_case_id)
def test_golden(mpg, mats, rec, engine, monkeypatch):
    case = dict(rec["case"])
    A = mats[case.pop("matrix")]
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = mpg.solve(A, b, xt, **_engine(monkeypatch, engine), **case)
    compare(rec, got, case["mode"], case["tol"], case["rlen"], _case_id(rec) + "/" + engine)


def _arrow(mpg, n):
    """Diagonally dominant arrow matrix: a dense first row and column, so
    one slice would pad every row to n (auto keeps CSR)."""
    rows = [[(0, float(n + 1))] + [(j, 0.5) for j in range(1, n)]]
    for i in range(1, n):
        rows.append([(0, 0.25), (i, 4.0)] + ([(i + 1, -1.0)] if i + 1 < n else []))
    rowptr = np.zeros(n + 1, dtype=np.int32)
    cols, vals = [], []
    for i, r in enumerate(rows):
        rowptr[i + 1] = rowptr[i] + len(r)
        cols += [c for c, _ in r]
        vals += [v for _, v in r]
    return mpg.Csr(n, n, rowptr, np.array(cols, dtype=np.int32), np.array(vals))


def test_spmv_layout_choice(mpg):
    """Auto picks SELL-64 with int16 offsets and 2-wide loads for the band,
    CSR for the arrow matrix; forcing either storage gives the same solve."""
    A = mpg.gen_band(20_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    e = mpg.Engine(A, b, xt, mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=2)
    try:  # 10 entries per row, 64-row slices, the last one half full
        assert e.spmv_layout() == {"format": "sell", "vec_width": 2, "col_bytes": 2,
                                   "stored": -(-A.nrows // 64) * 64 * 10, "window": True,
                                   "slices_per_wave": 2,  # uniform int16 slices: k_step_sell2
                                   "givens_folded": True, "accum": "f64", "prologue": "sell"}
    finally:
        e.close()
    B = _arrow(mpg, 3000)
    xb = mpg.rand_vect(B.nrows, 42)
    bb = mpg.host_spmv(B, xb)
    e = mpg.Engine(B, bb, xb, mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=2)
    try:
        assert e.spmv_layout()["format"] == "csr"
    finally:
        e.close()
    res = {}
    for fmt in ("csr", "sell"):
        got = mpg.solve(B, bb, xb, engine="fused", spmv_format=fmt, mode="mixed", orth="cgs", prec="jacobi",
                        rlen=30, tol=1e-10, max_restarts=50)
        assert got.status == "converged"
        res[fmt] = got
    assert res["csr"].total_iters == res["sell"].total_iters
    np.testing.assert_allclose(res["csr"].step_res, res["sell"].step_res, rtol=1e-4)


@pytest.mark.parametrize("engine", list(ENGINES))
@pytest.mark.parametrize("mode", ["mixed", "baseline"])
def test_live_oracle_band(mpg, oracle, engine, mode, monkeypatch):
    """Larger input than the fixtures: BAND n=200k, GMRES(30), live oracle."""
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=1e-9, max_restarts=40)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    got = mpg.solve(A, b, xt, **_engine(monkeypatch, engine), **opts)
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


@pytest.mark.parametrize("engine", ["surface", "fused"])
@pytest.mark.parametrize("n", [1, 2, 3, 65])
def test_tiny_systems_match_oracle(mpg, oracle, engine, n):
    """Restart length above n: the Krylov space is exhausted, h_{k+1,k}
    collapses to (near) zero and, with no breakdown guard in the reference,
    the cycle can turn non-finite. The GPU path must take the same restart
    decisions as the oracle on the same inputs."""
    A = mpg.gen_band(n, 1, 1, seed=5)
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="baseline", orth="cgs", prec="identity", rlen=30, tol=1e-12, max_restarts=5)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    got = mpg.solve(A, b, xt, engine=engine, **opts)
    assert got.status == ref.status
    assert got.restarts == ref.restarts and got.total_iters == ref.total_iters
    assert np.array_equal(np.isfinite(got.step_res), np.isfinite(ref.step_res))


@pytest.mark.parametrize("engine", ["surface", "fused"])
@pytest.mark.parametrize("mode", ["baseline", "mixed"])
@pytest.mark.parametrize("n", [1, 3])
def test_breakdown_report_and_stop(mpg, oracle, engine, mode, n):
    """the solve keeps the reference's unguarded
    normalisation (Orthogonalization.hpp:56-59), but reports what happened:
    at n = 1 the Krylov space is exhausted after one step and every later
    |s(k+1)| of the cycle is NaN (the oracle: 29 steps from step 1, one
    restart with a non-finite residual); n = 3 stays finite. The counts
    match the oracle's, and --stop-on-breakdown ends the solve with
    MPG_ERR_BREAKDOWN at the first one instead."""
    A = mpg.gen_band(n, 1, 1, seed=5)
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="identity", rlen=30, tol=1e-12, max_restarts=5)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    got = mpg.solve(A, b, xt, engine=engine, **opts)
    assert (got.nonfinite_steps, got.nonfinite_cycles, got.first_nonfinite_step) == \
        (ref.nonfinite_steps, ref.nonfinite_cycles, ref.first_nonfinite_step)
    assert (ref.nonfinite_steps > 0) == (n == 1), ref.nonfinite_steps
    if n == 1:
        with pytest.raises(RuntimeError, match=r"\(-6\).*non-finite"):
            mpg.solve(A, b, xt, engine=engine, stop_on_breakdown=True, **opts)
    else:
        ok = mpg.solve(A, b, xt, engine=engine, stop_on_breakdown=True, **opts)
        assert ok.status == got.status and np.array_equal(ok.step_res, got.step_res)


@pytest.mark.parametrize("engine", ["fused", "fused-cgspart", "surface"])
@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
@pytest.mark.parametrize("mode", ["mixed", "baseline"])
@pytest.mark.parametrize("rlen", [32, 33, 40, 70])
def test_long_restart_matches_oracle(mpg, oracle, engine, orth, mode, rlen, monkeypatch):
    """Restart lengths around and past the one-panel kernels' 32 columns:
    m = 32 is the last compile-time column count, m > 32 runs the multi-panel
    dots and the runtime-count CGS update / solution update, m > 64 also the
    separate trsv and an unfolded Givens launch. Live oracle, same inputs."""
    A = mpg.gen_band(3000, 5, 4, seed=11)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=rlen, tol=1e-10, max_restarts=30)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    env = {"fused": {}, "fused-cgspart": {"MPG_CGS_PARTIALS": "1"}, "surface": {}}[engine]
    for f in FLAGS:
        monkeypatch.setenv(f, env.get(f, "1" if f in ON_BY_DEFAULT + ("MPG_FOLD_GIVENS",) else "0"))
    got = mpg.solve(A, b, xt, engine="surface" if engine == "surface" else "fused", **opts)
    compare(as_ref(ref), got, mode, opts["tol"], rlen, f"band3000-{mode}-{orth}-m{rlen}-{engine}")


@pytest.mark.parametrize("mode", ["mixed", "baseline"])
@pytest.mark.parametrize("stop", ["converged", "aborted"])
def test_pipelined_cycles_match_serial(mpg, mode, stop, monkeypatch):
    """The pipelined cycle loop (the next cycle's graph is launched before
    this cycle's report is read; a cycle launched past the stop decision is
    undone by restoring x) gives bit-identical results to the serial loop,
    for a solve that converges and one that aborts at max_restarts."""
    A = mpg.gen_band(50_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="fused", mode=mode, orth="cgs", prec="jacobi", rlen=30,
                tol=1e-9 if stop == "converged" else 0.0, max_restarts=40 if stop == "converged" else 3)
    got = {}
    for pipe in ("1", "0"):
        monkeypatch.setenv("MPG_PIPELINE", pipe)
        got[pipe] = mpg.solve(A, b, xt, **opts)
    p, s = got["1"], got["0"]
    assert p.status == s.status == stop
    assert p.total_iters == s.total_iters and p.restarts == s.restarts
    assert np.array_equal(p.step_res, s.step_res)
    assert p.res_norm == s.res_norm and p.err_norm == s.err_norm


def test_engine_sequence_in_one_process(mpg, oracle):
    """CGS surface -> CGS fused -> MGS surface -> MGS fused in one process
    (each solve creates and destroys its own context, engine, graphs and
    pinned report buffers). Round 1 saw a SIGSEGV on the first MGS fused
    solve of this sequence under rocprofv3 --kernel-trace; its PC lies in
    librocprofiler-sdk's queue intercept while HIP submits the packet-captured
    graph, and the same sequence passes under the profiler with
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (profiles/r02_engine_sequence_*).
    Every solve here is checked against the oracle."""
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    for orth in ("cgs", "mgs"):
        opts = dict(mode="mixed", orth=orth, prec="identity", rlen=30, tol=1e-9, max_restarts=40)
        ref = oracle.solve(mpg, A, b, xt, **opts)
        for engine in ("surface", "fused"):
            got = mpg.solve(A, b, xt, engine=engine, **opts)
            compare(as_ref(ref), got, "mixed", opts["tol"], 30, f"sequence-{orth}-{engine}")


@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "single"])
@pytest.mark.parametrize("prec", ["identity", "jacobi", "ilu"])
def test_surface_cycle_program_matches_eager(mpg, orth, mode, prec, monkeypatch):
    """The operator-surface driver records its Arnoldi steps once per solve
    (CycleProgram<Hip>: first cycle eager, second recorded, later replayed)
    when the strategy makes no decision inside a cycle. Replays must give the
    same bits as issuing every call on its own (MPG_SURFACE_GRAPH=0,
    MPG_SURFACE_BATCH=0, MPG_SURFACE_FUSE=0: no recording, no scalar-op
    batching, every reduction's stage 2 its own launch); an ILU apply,
    which reads its fault word, voids the recording and runs eagerly."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="surface", mode=mode, orth=orth, prec=prec, rlen=30, tol=1e-9, max_restarts=6)
    got = {}
    for g in ("1", "0"):
        monkeypatch.setenv("MPG_SURFACE_GRAPH", g)
        monkeypatch.setenv("MPG_SURFACE_BATCH", g)
        monkeypatch.setenv("MPG_SURFACE_FUSE", g)
        before = mpg.cycle_program_counts()
        got[g] = mpg.solve(A, b, xt, **opts)
        after = mpg.cycle_program_counts()
        delta = {k: after[k] - before[k] for k in after}
        if g == "0":
            assert delta == {"recorded": 0, "replayed": 0, "voided": 0}
        elif got[g].total_iters // 30 >= 2:
            if prec == "ilu":
                assert delta == {"recorded": 0, "replayed": 0, "voided": 1}, delta
            else:
                assert delta["recorded"] == 1 and delta["voided"] == 0, delta
                assert delta["replayed"] == got[g].total_iters // 30 - 2, delta
    p, e = got["1"], got["0"]
    assert p.status == e.status and p.total_iters == e.total_iters and p.restarts == e.restarts
    assert np.array_equal(p.step_res, e.step_res)
    assert p.res_norm == e.res_norm and p.err_norm == e.err_norm


@pytest.mark.parametrize("mode", ["mixed", "baseline"])
@pytest.mark.parametrize("prec", ["identity", "jacobi"])
def test_surface_host_norm_memo(mpg, mode, prec, monkeypatch):
    """Round 6 (MPG_SURFACE_FUSE bit 32): a host-value nrm2 of a vector that
    nothing has written since its last host read returns that read (the
    reference's restart section reads ||w|| as r_norm, beta and in
    first_vector). With the identity preconditioner beta and first_vector's
    read are answered from it, with Jacobi only first_vector's (gdmv writes
    w between r_norm and beta); the solve keeps the bits of the surface
    without the memo."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="surface", mode=mode, orth="cgs", prec=prec, rlen=30, tol=0.0, max_restarts=3)
    monkeypatch.delenv("MPG_SURFACE_FUSE", raising=False)
    h0 = mpg.surface_host_norm_hits()
    on = mpg.solve(A, b, xt, **opts)
    hits = mpg.surface_host_norm_hits() - h0
    monkeypatch.setenv("MPG_SURFACE_FUSE", str(1 | 4 | 8 | 16))
    h1 = mpg.surface_host_norm_hits()
    off = mpg.solve(A, b, xt, **opts)
    assert mpg.surface_host_norm_hits() == h1
    assert hits >= (2 * 3 if prec == "identity" else 3), hits
    assert on.total_iters == off.total_iters == 90
    assert np.array_equal(on.step_res, off.step_res) and np.array_equal(on.x, off.x)
    assert on.res_norm == off.res_norm


@pytest.mark.parametrize("mode", ["mixed", "baseline", "single"])
@pytest.mark.parametrize("prec", ["identity", "jacobi"])
def test_surface_host_norm_pair(mpg, mode, prec, monkeypatch):
    """Round 6 (MPG_SURFACE_FUSE bit 64): the restart section's r_norm read
    also reads ||x|| of the residual SpMV's input in the same launch
    (mpg_nrm2_pair_host), and x_norm is then a memo hit when nothing wrote
    in between (identity; with Jacobi gdmv writes w first, so x_norm reads
    again). The solve keeps the bits of the surface without the pairing and
    of the surface without any memo."""
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="surface", mode=mode, orth="cgs", prec=prec, rlen=30, tol=0.0, max_restarts=3)
    monkeypatch.delenv("MPG_SURFACE_FUSE", raising=False)
    p0, h0 = mpg.surface_host_norm_pairs(), mpg.surface_host_norm_hits()
    on = mpg.solve(A, b, xt, **opts)
    pairs, hits = mpg.surface_host_norm_pairs() - p0, mpg.surface_host_norm_hits() - h0
    monkeypatch.setenv("MPG_SURFACE_FUSE", str(1 | 4 | 8 | 16 | 32))
    p1, h1 = mpg.surface_host_norm_pairs(), mpg.surface_host_norm_hits()
    mid = mpg.solve(A, b, xt, **opts)
    assert mpg.surface_host_norm_pairs() == p1
    hits_memo_only = mpg.surface_host_norm_hits() - h1
    monkeypatch.setenv("MPG_SURFACE_FUSE", str(1 | 4 | 8 | 16))
    off = mpg.solve(A, b, xt, **opts)
    assert pairs >= 3, pairs  # one per restart section (3 cycles + the final residual)
    if prec == "identity":
        assert hits >= hits_memo_only + 3, (hits, hits_memo_only)  # x_norm answered by the pair
    for r in (mid, off):
        assert on.total_iters == r.total_iters == 90
        assert np.array_equal(on.step_res, r.step_res) and np.array_equal(on.x, r.x)
        assert on.res_norm == r.res_norm


def test_nrm2_pair_host_same_bits(hip):
    """mpg_nrm2_pair_host: each norm with the bits of its own
    mpg_nrm2_*_host, for every type pair, tails (n not a multiple of 4) and
    one workgroup up to the full stage-1 grid."""
    import ctypes as C

    F64, F32 = 0, 1
    g = np.random.default_rng(5)
    for n in (1, 7, 4099, 1_000_003, 4_000_000):
        for ta, tb in ((F32, F64), (F64, F64), (F32, F32), (F64, F32)):
            dta = np.float64 if ta == F64 else np.float32
            dtb = np.float64 if tb == F64 else np.float32
            a = (g.standard_normal(n) * 3).astype(dta)
            bvec = g.standard_normal(n).astype(dtb)
            da, db = hip.buf(a), hip.buf(bvec)
            ra, rb = C.c_double(), C.c_double()
            hip.check(hip.lib.mpg_nrm2_pair_host(hip.ctx, n, ta, da.p, tb, db.p, C.byref(ra), C.byref(rb)), "pair")
            ref = []
            for t, d in ((ta, da), (tb, db)):
                if t == F64:
                    r = C.c_double()
                    hip.check(hip.lib.mpg_nrm2_f64_host(hip.ctx, n, d.p, C.byref(r)), "nrm2")
                else:
                    r = C.c_float()
                    hip.check(hip.lib.mpg_nrm2_f32_host(hip.ctx, n, d.p, C.byref(r)), "nrm2")
                ref.append(float(r.value))
            assert ra.value == ref[0] and rb.value == ref[1], (n, ta, tb, ra.value, rb.value, ref)
            assert np.isclose(ra.value, np.linalg.norm(a.astype(np.float64)), rtol=1e-6)
            da.free()
            db.free()


@pytest.mark.parametrize("matrix", ["band", "lap", "stencil27"])
@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "single"])
@pytest.mark.parametrize("prec", ["identity", "jacobi"])
def test_surface_normalisation_ride_same_bits(mpg, matrix, orth, mode, prec, monkeypatch):
    """Round 5: add_vector's scal_recip rides the next SELL
    SpMV on the operator surface (MPG_SURFACE_FUSE bit 16, default on): the
    CGS gemv writes w's new value to a scratch copy, the SpMV forms h(k+1,k),
    V(:,k+1) and A V(:,k+1) -> w in one launch. The solve must give the bits
    of the same surface without the ride (bits 1|4|8) and of every call on
    its own (0), on the two-slice window kernel (BAND), the two-slice gather
    kernel (7-point Laplacian) and the stepped kernel with CSR-summed slices
    (27-point, 3 dof, planes past 32767 rows); CGS must actually ride, and
    the cycles still record and replay."""
    monkeypatch.setenv("MPG_SURFACE_NODE", "0")  # (the SELL kernels' rides; node blocks: the next test)
    A = {"band": lambda: mpg.gen_band(100_000, 5, 4, seed=7), "lap": lambda: mpg.gen_laplace3d(40),
         "stencil27": lambda: mpg.gen_stencil27(105, 3, ny=105, nz=3)}[matrix]()
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="surface", mode=mode, orth=orth, prec=prec, rlen=30, tol=0.0, max_restarts=3)
    got = {}
    for fuse in ("", "13", "0"):
        if fuse:
            monkeypatch.setenv("MPG_SURFACE_FUSE", fuse)
        else:
            monkeypatch.delenv("MPG_SURFACE_FUSE", raising=False)
        before = mpg.surface_ride_counts()
        got[fuse] = mpg.solve(A, b, xt, **opts)
        after = mpg.surface_ride_counts()
        delta = {k: after[k] - before[k] for k in after}
        if fuse:
            assert delta["redirects"] == 0 and delta["rides"] == 0, delta
        elif orth == "cgs":
            # every step but the last of a cycle rides, counted on the host in
            # the eager cycle and the recording one (the third cycle replays
            # the recorded graph, rides included, with no host calls)
            assert delta["rides"] >= 2 * 27 and delta["flushed"] <= 2, delta
        elif orth == "mgs":
            assert delta == {"redirects": 0, "rides": 0, "flushed": 0}, delta
    ref = got["0"]
    for fuse in ("", "13"):
        g = got[fuse]
        assert g.total_iters == ref.total_iters == 90, (fuse, g.total_iters)
        assert np.array_equal(g.step_res, ref.step_res), fuse
        assert np.array_equal(g.x, ref.x) and g.res_norm == ref.res_norm, fuse


@pytest.mark.parametrize("prec", ["identity", "jacobi"])
@pytest.mark.parametrize("mode", ["mixed", "baseline", "single"])
@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
@pytest.mark.parametrize("matrix", ["fem27", "stencil27p"])
def test_surface_node_ride_same_bits(mpg, matrix, orth, mode, prec, monkeypatch):
    """Round 6: the same rides on the node-block copy
    (mpg_node_spmv_norm_* / _prog_*): the surface's SpMV runs on node blocks,
    CGS rides every step but a cycle's last, and the solve has the bits of the
    surface without the ride (MPG_SURFACE_FUSE=13) and of every call on its own
    (0)."""
    monkeypatch.delenv("MPG_SURFACE_NODE", raising=False)
    A = {"fem27": lambda: mpg.gen_fem27(24, 3, keep_pct=70, seed=13),
         "stencil27p": lambda: mpg.gen_stencil27p(40, 3, ny=40, nz=8, block=64, perm_seed=5)}[matrix]()
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="surface", mode=mode, orth=orth, prec=prec, rlen=30, tol=0.0, max_restarts=3)
    got = {}
    for fuse in ("", "13", "0"):
        if fuse:
            monkeypatch.setenv("MPG_SURFACE_FUSE", fuse)
        else:
            monkeypatch.delenv("MPG_SURFACE_FUSE", raising=False)
        before, sp0 = mpg.surface_ride_counts(), mpg.surface_spmv_counts()
        got[fuse] = mpg.solve(A, b, xt, **opts)
        after, sp1 = mpg.surface_ride_counts(), mpg.surface_spmv_counts()
        delta = {k: after[k] - before[k] for k in after}
        assert sp1["node"] > sp0["node"] and sp1["sell"] == sp0["sell"], (sp0, sp1)
        if fuse:
            assert delta["redirects"] == 0 and delta["rides"] == 0, delta
        elif orth == "cgs":
            assert delta["rides"] >= 2 * 27 and delta["flushed"] <= 2, delta
    ref = got["0"]
    for fuse in ("", "13"):
        g = got[fuse]
        assert g.total_iters == ref.total_iters == 90, (fuse, g.total_iters)
        assert np.array_equal(g.step_res, ref.step_res), fuse
        assert np.array_equal(g.x, ref.x) and g.res_norm == ref.res_norm, fuse


@pytest.mark.parametrize("mode", ["mixed", "single"])
@pytest.mark.parametrize("orth", ["cgs", "cgsr"])
def test_fused_dots_strict(mpg, oracle, mode, orth, monkeypatch):
    """MPG_FUSE_DOTS=2 makes an unsupported fused SpMV + dots launch an
    error instead of a silent fallback, so this case proves k_step_sell's
    SellDots form ran (fp32 basis and values, int16 columns, LDS window:
    BAND) and matches the oracle. The golden-suite engines use =1, which
    falls back wherever the form does not apply."""
    monkeypatch.setenv("MPG_CGS_PARTIALS", "1")
    monkeypatch.setenv("MPG_FUSE_DOTS", "2")
    A = mpg.gen_band(150_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=1e-9, max_restarts=40)
    eng = mpg.Engine(A, b, xt, spmv_format="sell", **opts)
    assert eng.spmv_layout()["col_bytes"] == 2 and eng.spmv_layout()["window"]
    eng.close()
    got = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
    ref = oracle.solve(mpg, A, b, xt, **opts)
    compare(as_ref(ref), got, mode, opts["tol"], 30, f"fused-dots-strict-{mode}-{orth}")


@pytest.mark.parametrize("orth", ["cgs", "cgsr"])
@pytest.mark.parametrize("mode", ["mixed", "baseline"])
def test_surface_gemv_emits_nrm2_partials_same_bits(mpg, orth, mode, monkeypatch):
    """Operator surface, MPG_SURFACE_FUSE bit 8: the CGS update's gemv emits
    the ||w||^2 stage-1 partials in the quad nrm2 layout, and add_vector's
    nrm2(w) takes them instead of launching its stage 1 (CGSR: across the
    axpy into h). The partials are the ones k_nrm2_quad computes, so the
    solve bits are those of the unfused surface (bit 8 off), on a size with
    tail rows and on one with several row quads per lane."""
    for A in (mpg.gen_laplace3d(23), mpg.gen_band(1_200_003, 5, 4, seed=5)):
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=2)
        got = {}
        for fuse in ("13", "5"):
            monkeypatch.setenv("MPG_SURFACE_FUSE", fuse)
            got[fuse] = mpg.solve(A, b, xt, engine="surface", **opts)
        p, q = got["13"], got["5"]
        assert p.total_iters == q.total_iters == 60
        assert np.array_equal(p.step_res, q.step_res) and np.array_equal(p.x, q.x), A.nrows


@pytest.mark.parametrize("flag,engine,accum", [("MPG_CGS_PREFETCH", "fused", "f64"), ("MPG_CGS_PREFETCH", "fused", "f32"),
                                               ("MPG_SURFACE_PAIR", "surface", "f64")])
@pytest.mark.parametrize("mode", ["mixed", "baseline"])
def test_round4_kernel_variants_same_bits(mpg, flag, engine, accum, mode, monkeypatch):
    """Round-4 kernel forms that must not change a bit: the CGS update that
    issues its first row group under the coefficient sums (MPG_CGS_PREFETCH;
    on by default in the fp32 accumulation class since round 6) and the
    operator surface's two-slice-per-wave SELL SpMV (MPG_SURFACE_PAIR, on by
    default) -- the same operands summed in the same order."""
    res = {}
    for mpg_case in ("band", "lap"):
        A = mpg.gen_band(120_000, 5, 4, seed=7) if mpg_case == "band" else mpg.gen_laplace3d(40)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
        if accum == "f32":
            opts["accum"] = "f32"
        for v in ("0", "1"):
            monkeypatch.setenv(flag, v)
            res[(mpg_case, v)] = mpg.solve(A, b, xt, engine=engine, **opts)
        a, c = res[(mpg_case, "0")], res[(mpg_case, "1")]
        assert a.total_iters == c.total_iters == 90
        assert np.array_equal(a.step_res, c.step_res) and np.array_equal(a.x, c.x), (flag, mpg_case)
