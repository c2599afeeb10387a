"""CPU checks of bench.py's bookkeeping (no GPU): the committed profiles it
reads beside its live measurement belong to the kernels it names."""
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_rocprof_summary_names_the_bench_kernels():
    """profiles/bench_kernel_stats.rocprof (the rocprofv3 --stats CSV of
    `bench.py --steps 10`) holds every kernel the roofline reports, with a
    plausible mean launch time."""
    prof = REPO / "profiles"
    for k in ("k_step_sell2", "k_dots_nc", "k_cgs_update_nc"):
        ms = bench.rocprof_avg_ms(prof, k)
        assert ms is not None and 0.001 < ms < 0.1, (k, ms)


def test_rocprof_summary_absent_is_none(tmp_path):
    assert bench.rocprof_avg_ms(tmp_path, "k_step_sell2") is None


def test_pmc_traffic_has_the_bench_kernels():
    t = bench.pmc_traffic(REPO / "profiles")
    for k in ("k_step_sell2:fold", "k_dots_nc", "k_cgs_update_nc"):
        assert t.get(k) and t[k] > 1e7, (k, t.get(k))
    # the FETCH_SIZE x2 correction is recorded with the numbers
    d = json.loads((REPO / "profiles" / "pmc_traffic.json").read_text())
    assert "x2" in d["_fetch_correction"]


# ---- the N-rank launcher: no GPU work in --dry-run


def _bench(args, env_extra=None, timeout=300):
    import os
    import subprocess

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(REPO / "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env)


def test_launcher_starts_n_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes with
    the torch.distributed.run environment; rank 0's line is relayed on
    stdout, rank 1's goes to stderr."""
    p = _bench(["--gpus", "2", "--dry-run"])
    assert p.returncode == 0, p.stderr
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and lines[0]["rank"] == 0 and lines[0]["world"] == 2, p.stdout
    assert lines[0]["master"].startswith("127.0.0.1:")
    other = [json.loads(ln.split("] ", 1)[1]) for ln in p.stderr.splitlines() if ln.startswith("[rank 1 stdout]")]
    assert len(other) == 1 and other[0]["world"] == 2 and other[0]["local_rank"] == 1, p.stderr
    assert other[0]["master"] == lines[0]["master"]


def test_launcher_world8_rehearses_the_setup_over_gloo():
    """The N = 8 run's CPU-side set-up, pre-flighted: eight
    rank processes, one gloo process group (the only torch group a rank
    makes; the data path's RCCL communicator is the engine's own), each
    rank's BAND block analysed and the halo lists swapped: rank q receives
    5 rows from q-1 and 4 from q+1 (offsets -5..+4) and sends the mirror;
    rank 0's 128-byte unique-id stand-in reaches every rank."""
    p = _bench(["--gpus", "8", "--dry-run", "--n-local", "2000"], timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    others = [json.loads(ln.split("] ", 1)[1]) for ln in p.stderr.splitlines()
              if ln.startswith("[rank ") and ln.split("] ", 1)[1].startswith("{")]
    ranks = sorted(lines + others, key=lambda d: d["rank"])
    assert [d["rank"] for d in ranks] == list(range(8)), p.stderr[-2000:]
    for d in ranks:
        q = d["rank"]
        assert d["world"] == 8 and d["process_group"] == "gloo" and d["uid_bytes"] == 128
        want_recv = {**({str(q - 1): 5} if q > 0 else {}), **({str(q + 1): 4} if q < 7 else {})}
        want_send = {**({str(q - 1): 4} if q > 0 else {}), **({str(q + 1): 5} if q < 7 else {})}
        assert d["halo_recv"] == want_recv and d["halo_send"] == want_send, d
        assert d["n_ext"] == 2000 + (4 if q < 7 else 0)
        assert any("ncclAllReduce" in c for c in d["step_collectives"])


class _Res:
    def __init__(self, iters, secs):
        self.total_iters, self.gmres_seconds = iters, secs


def test_cpu_baseline_respects_its_budget_and_reports_best():
    """A CPU leg stops its timed solves when the next would overrun the leg's
    budget (the N = 8 legs on 80M / 100M-nnz matrices stay bounded), keeps at
    least one per orthogonalisation, and reports the faster one as `best`."""
    import argparse
    import time

    def slow_solve(mpg, A, b, xt, orth, max_restarts, threads, **o):
        t = 0.3 if orth == "cgs" else 0.1  # MGS the faster, as MKL's is
        time.sleep(t)
        return _Res(30 * max_restarts, t)

    args = argparse.Namespace(orth="cgs", cpu_cycles=2, cpu_runs=50, cpu_budget_s=2.0, rlen=30, mode="mixed")
    opts = dict(mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=10, device=0)
    t0 = time.perf_counter()
    cpu = bench.cpu_baseline(None, None, None, None, opts, args, solve=slow_solve)
    wall = time.perf_counter() - t0
    assert wall < 2.0 + 0.3 + 0.3 + 0.5, wall  # the budget, one overrunning solve and the warm-ups
    assert 1 <= len(cpu["by_orth"]["cgs"]["runs"]) < 50 and 1 <= len(cpu["by_orth"]["mgs"]["runs"]) < 50
    assert cpu["value"] == cpu["by_orth"]["cgs"]["median"] and cpu["best_orth"] == "mgs"
    assert cpu["best"] == cpu["by_orth"]["mgs"]["median"] > cpu["value"]
    bench.vs_gpu(cpu, 26000.0)
    assert cpu["vs_gpu_best"] == round(26000.0 / cpu["best"], 2) < cpu["vs_gpu"]


def test_launcher_fails_when_a_rank_fails():
    p = _bench(["--gpus", "3", "--dry-run"], {"MPG_BENCH_DRY_FAIL_RANK": "1"})
    assert p.returncode != 0
    assert "rank 1 exited" in p.stderr


def test_launcher_refuses_missing_gpus():
    """Fewer visible GPUs than --gpus is an error, never a silent N = 1
    (this container has none)."""
    p = _bench(["--gpus", "2"])
    assert p.returncode == 2 and "needs 2 visible GPU(s), found 0" in p.stderr, (p.returncode, p.stderr[-500:])
    assert not p.stdout.strip()


def test_launcher_flag_and_world_must_agree():
    p = _bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "4", "RANK": "0"})
    assert p.returncode == 0  # dry-run reports before any check
    p = _bench(["--gpus", "2"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2 and "disagree" in p.stderr


# ---- degenerate timings: bench never divides by a non-positive time


class _FakeEngine:
    def __init__(self, dup_ms, stamps_ms):
        self.dup_ms, self.stamps_ms = dup_ms, stamps_ms

    def spmv_layout(self):
        return {"format": "sell", "slices_per_wave": 2, "givens_folded": True}

    def time_phase_dup(self, phase, reps):
        return self.dup_ms, 30 * reps

    def time_phase_graph(self, phase, reps):
        return 0.012, [0.012] * (30 * reps)

    def time_phase_stamps(self, phase, reps):
        return self.stamps_ms, [self.stamps_ms or 0.0] * (30 * reps)

    def time_spmv_incycle(self, cycles):
        return 0.0125, [0.0125] * (30 * cycles)

    def phase_bytes(self, phase):
        return 5.2e7


def test_phase_roofline_degenerate_clock_is_null():
    for dup, st in ((0.0, 0.011), (-0.002, 0.011), (0.011, 0.0)):
        out = bench.phase_roofline(_FakeEngine(dup, st), 30, 3, {})
        assert out == {"k_dots_nc": None, "k_cgs_update_nc": None}, (dup, st, out)
    out = bench.phase_roofline(_FakeEngine(0.012, 0.011), 30, 3, {})
    assert out["k_dots_nc"]["avg_launch_ms"] == 0.012


def test_phase_roofline_empty_timings_are_null():
    class Empty(_FakeEngine):
        def time_phase_stamps(self, phase, reps):
            return 0.011, []

    out = bench.phase_roofline(Empty(0.012, 0.011), 30, 3, {})
    assert out == {"k_dots_nc": None, "k_cgs_update_nc": None}


def test_spmv_roofline_falls_back_on_a_degenerate_difference():
    for dup in (0.0, -0.001):
        sp = bench.spmv_roofline(_FakeEngine(dup, 0.011), 3)
        assert sp["timing"] == "eager" and sp["avg_launch_ms"] == 0.0125
    sp = bench.spmv_roofline(_FakeEngine(0.011, 0.011), 3)
    assert sp["timing"] == "dup" and sp["avg_launch_ms"] == 0.011
