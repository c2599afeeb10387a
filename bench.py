#!/usr/bin/env python3
"""GMRES iterations/s on MI355X for the BASELINE.json metric.

Workload (BASELINE.json metric "GMRES iterations/sec + SpMV achieved HBM GB/s,
10M-nnz CSR, 1/2/4/8 GPUs"): the synthetic banded CSR "BAND-10M" (n = 1e6
rows per GPU, column offsets -5..+4, 9,999,975 nnz at one GPU; values from
the counter-based generator of include/mpgmres/problems.h), x_true =
rand_vect(n, 42), b = A x_true, restarted GMRES(30), mixed precision
(fp32 Arnoldi + fp64 residual/update: gmres_singleUpdate), CGS, identity
preconditioner, tol = 0 so the solve never stops early. The fp32 Arnoldi runs
in the reference's fp32 accumulation class by default (--accum f32: every
dot / norm / gemv / SpMV partial sum in fp32, as cblas_s* / mkl_sparse_s_mv
sum); --accum f64 sums the fp32 products in fp64 instead. The line's
"accum" names the one it timed.

One step = one restart cycle = check_initial on the host + 30 Arnoldi
iterations + solution update + the next true-residual prologue (the fused
engine's graph replay).

Scaling modes (one row-partitioned solve over all ranks either way; value
is that one solve's GMRES iterations per second at every N):
  weak (default)       each rank owns a 1e6-row BAND block of an N*1e6-row
                       matrix (10M nnz per GPU); the aggregate over row
                       blocks (iterations x N per second) is reported
                       separately as "aggregate";
  strong               --global-rows R: one R-row BAND matrix split over the
                       N ranks (R = 1e7 is the north star's 100M-nnz matrix).

Also reported, at every N from rank 0: the roofline of the dominant kernel --
the Arnoldi SpMV as the cycle runs it (Givens folded on one GPU), each launch
timed by its own kernel events -- on the bytes its storage moves, against the
8 TB/s spec and the GPU's measured streaming peak (mpg_bw_probe, 2 GiB), with
every rank's mean launch time; the whole-iteration fraction; at N = 1 the
same SpMV on BAND-100M (past the 256 MB Infinity Cache) as the HBM figure;
and the CPU oracle (MKL restatement of kernels_mkl.cpp) on the same global
matrix on the host cores -- the box's share at N = 1, the N GPUs' share of
the node's physical cores at N > 1 (all of them at N = 8) -- 1 warm-up +
the median of the timed runs per orthogonalisation.
"""
import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "GMRES iterations/sec + SpMV achieved HBM GB/s, 10M-nnz CSR, 1/2/4/8 GPUs"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_CPU_INFO = None


def cpu_info() -> dict:
    """CPU model, physical cores of the machine (lscpu), and the cores this
    process may run on (its affinity mask: the box's share of the host)."""
    info = {"model": "unknown", "physical_cores": None, "affinity_cpus": len(os.sched_getaffinity(0))}
    try:
        import subprocess

        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {k.strip(): v.strip() for k, v in (ln.split(":", 1) for ln in out.splitlines() if ":" in ln)}
        info["model"] = kv.get("Model name", "unknown")
        info["physical_cores"] = int(kv.get("Core(s) per socket", "0")) * int(kv.get("Socket(s)", "1"))
    except Exception:
        pass
    return info


def cpu_threads(world: int = 1, shared_gpu: bool = False) -> int:
    """Threads for the CPU baseline. N = 1: the box's CPU share
    (OMP_NUM_THREADS, set to 16 per GPU on the pool). N > 1: the N GPUs'
    share of the node's physical cores (N/8 of them; all at N = 8), as the
    north star's ">= 6x vs MKL at 8 GPUs" compares against the whole host.
    Never more than the affinity mask or the physical cores."""
    info = _CPU_INFO or cpu_info()
    cores = min(info["affinity_cpus"], info["physical_cores"] or info["affinity_cpus"])
    if world > 1 and not shared_gpu:
        n = max(cores * min(world, 8) // 8, 1)
    else:
        n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or info["affinity_cpus"]
    return max(min(n, cores), 1)


def load_pkg():
    from __graft_entry__ import _load

    return _load()


ROCPROF_STATS = "bench_kernel_stats.rocprof"


def rocprof_avg_ms(profile_dir: Path, kernel: str):
    """Mean duration (ms) over all launches of `kernel` (every template
    instance) in the committed rocprofv3 --kernel-trace --stats summary of
    `bench.py --steps 10 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0`
    (profiles/bench_kernel_stats.rocprof: the CSV, renamed so it travels with the tree), None when absent:
    the CP's timestamps of each dispatch, which rocprof reports, set beside
    the live wave-stamp time."""
    f = profile_dir / ROCPROF_STATS
    if not f.exists():
        return None
    import csv

    calls, total = 0, 0.0
    try:
        for r in csv.DictReader(f.open()):
            name = r["Name"]
            if f"::{kernel}<" in name or name.startswith(f"{kernel}<") or f" {kernel}<" in name:
                calls += int(r["Calls"])
                total += float(r["TotalDurationNs"])
    except (KeyError, ValueError, OSError):
        return None
    return round(total / calls * 1e-6, 5) if calls else None


def pmc_traffic(profile_dir: Path) -> dict:
    """HBM bytes per launch of each kernel of the bench command from the
    committed rocprofv3 PMC summary (profiles/pmc_traffic.json written by
    tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE in separate passes,
    gfx950 correction), {} when absent."""
    f = profile_dir / "pmc_traffic.json"
    if not f.exists():
        return {}
    try:
        d = json.loads(f.read_text())
        return {k: v.get("hbm_bytes_per_launch") for k, v in d.items() if isinstance(v, dict)}
    except Exception:
        return {}


def spmv_roofline(eng, cycles: int) -> dict:
    """The Arnoldi SpMV in its place in the cycle (k = 0 plain, k >= 1 with
    the Givens step folded): what one launch adds to a graph replay of the
    cycle -- the timed region's form -- measured with HIP events around
    whole replays of the cycle as run and of the cycle with every SpMV
    launched twice in a row (mpg_engine_time_phase_dup: the kernel plus its
    dispatch and release, the figure rocprofv3's kernel trace reports); the
    same launches between event-record nodes (which add two marker packets)
    beside it; eager cycles with each launch's own kernel events when the
    engine does not capture its cycle. Bytes: what the storage moves, and
    SURVEY 8(d)'s CSR bytes."""
    layout = eng.spmv_layout()
    event_ms = None
    try:
        avg_ms, n_added = eng.time_phase_dup("spmv", max(5, 2 * cycles))
        per = [avg_ms] * n_added
        timing = "dup"
        try:  # the same launches between event-record nodes, for comparison
            event_ms = eng.time_phase_graph("spmv", cycles)[0]
        except RuntimeError as ex:
            log(f"[bench] graph-event timing unavailable ({ex})")
    except RuntimeError as ex:
        log(f"[bench] duplicate-launch timing unavailable ({ex}); timing eager cycles")
        avg_ms, per, timing = None, None, "eager"
    if avg_ms is None or not avg_ms > 0:  # unavailable, or a degenerate difference of replay times
        if timing == "dup":
            log(f"[bench] duplicate-launch difference {avg_ms} ms is not a launch time; timing eager cycles")
        avg_ms, per = eng.time_spmv_incycle(cycles)
        timing = "eager"
    actual = eng.phase_bytes("spmv_storage")
    csr = eng.phase_bytes("spmv")
    kernel = ("k_step_sell2" if layout.get("slices_per_wave") == 2 else "k_step_sell") if layout["format"] == "sell" \
        else "k_step_spmv"
    return {"kernel": kernel, "layout": layout, "timing": timing, "event_graph_ms": event_ms,
            "avg_launch_ms": avg_ms, "launches": len(per), "min_launch_ms": min(per), "max_launch_ms": max(per),
            "storage_bytes": actual, "csr_bytes": csr,
            "achieved_gbs": actual / (avg_ms * 1e-3) / 1e9, "csr_equiv_gbs": csr / (avg_ms * 1e-3) / 1e9}


def phase_roofline(eng, rlen: int, reps: int, traffic: dict) -> dict:
    """The CGS step's other two kernels, timed like the SpMV (wave stamps in
    graph replays of the cycle): per kernel the mean launch time over the
    cycle's steps, the fit t(k) = a + b k (a = the fixed cost of a launch, b
    = one more basis column), the bytes it moves at the cycle's mean k
    (basis columns 0..k, w read, and for the update w written) and their
    fraction of 8 TB/s; PMC bytes from the committed profile when present."""
    out = {}
    for ph, kname in (("dots", "k_dots_nc"), ("cgs_update", "k_cgs_update_nc")):
        try:
            ms, n_added = eng.time_phase_dup(ph, max(5, 2 * reps))
        except RuntimeError:  # the phase has no launch of its own (e.g. dots fused into the SpMV)
            out[kname] = None
            continue
        timing = "HIP events around graph replays of the cycle as run and with the phase's launches doubled"
        try:  # the kernel alone: its waves' wall-clock stamps, per k for the fit
            k_ms, per = eng.time_phase_stamps(ph, reps)
        except RuntimeError:
            k_ms, per = eng.time_phase_graph(ph, reps)
        if n_added < rlen or len(per) < rlen:
            out[kname] = None
            continue
        if not ms or ms <= 0 or not k_ms or k_ms <= 0:  # a degenerate clock (noise larger than the launch)
            out[kname] = None
            continue
        byk = np.asarray(per[:len(per) // rlen * rlen]).reshape(-1, rlen).mean(axis=0) * 1e3
        b, a = np.polyfit(np.arange(rlen), byk, 1)
        mb = eng.phase_bytes(ph)
        ach = mb / (ms * 1e-3) / 1e9
        pmc = traffic.get(kname) if rlen <= 32 else None
        out[kname] = {"bytes_mean_k": int(mb), "avg_launch_ms": round(ms, 5), "achieved": round(ach, 1),
                      "timing": timing, "kernel_only_ms": round(k_ms, 5),
                      "fit_basis": "wave wall-clock stamps per launch (first wave start to last wave end)",
                      "rocprof_avg_launch_ms": rocprof_avg_ms(REPO / "profiles", kname),
                      "frac": round(ach / HBM_PEAK_GBS, 4), "fit_a_us": round(float(a), 3),
                      "fit_b_us_per_column": round(float(b), 4),
                      "traffic": pmc, "traffic_over_bytes": round(pmc / mb, 4) if pmc else None}
    return out


def pair_rate(mpg, A, b, xt, o, cycles: int):
    """(iterations/s, whole-solve iterations/s, the three pair rates) of
    mpg.solve with options o: two solves of 4 and 4 + `cycles` restart
    cycles, the difference of their GMRES iterations over the difference of
    their GMRES times (so the first cycle's lazy set-up cancels), median of
    three such pairs (one pair moved +-4 % between runs of one box), after a
    2-cycle warm-up solve (the process's first solve of an engine also pays
    one-time code-object loads)."""
    mpg.solve(A, b, xt, **dict(o, max_restarts=2))
    rates, wholes = [], []
    for _ in range(3):
        runs = []
        for r in (4, 4 + cycles):
            res = mpg.solve(A, b, xt, **dict(o, max_restarts=r))
            runs.append((res.total_iters, res.gmres_seconds))
        rates.append((runs[1][0] - runs[0][0]) / (runs[1][1] - runs[0][1]))
        wholes.append(runs[1][0] / runs[1][1])
    return sorted(rates)[1], sorted(wholes)[1], rates


def surface_rate(mpg, A, b, xt, opts, cycles: int, fused_rate: float) -> dict:
    """The same solve through the drop-in boundary north_star names: the
    reference's driver (gmres_singleUpdate / gmres_baseline, restated in
    host/gmres_impl.hpp) over the kernels.hpp operator surface of
    kernels_hip.cpp (mpg_solve, engine surface), timed by pair_rate.
    The surface's kernels sum in fp64 (accumulation class f64), so beside
    vs_fused (against the headline line, whose class is the bench's --accum)
    the fused engine is timed the same way in the f64 class: vs_fused_f64 is
    the surface against the fused engine doing the same arithmetic."""
    o = {k: v for k, v in opts.items() if k not in ("spmv_format", "accum")}
    rate, whole, rates = pair_rate(mpg, A, b, xt, dict(o, engine="surface"), cycles)
    f64, _, f64_rates = pair_rate(mpg, A, b, xt, dict(o, engine="fused", accum="f64"), cycles)
    log(f"[bench] operator surface: {rate:.0f} it/s ({rate / fused_rate:.3f} of the fused engine, "
        f"{rate / f64:.3f} of the fused engine in the f64 class, {f64:.0f} it/s); "
        f"{whole:.0f} it/s over the whole {4 + cycles}-cycle solve")
    return {"iters_per_s": round(rate, 2), "vs_fused": round(rate / fused_rate, 4),
            "fused_f64_iters_per_s": round(f64, 2), "vs_fused_f64": round(rate / f64, 4),
            "whole_solve_iters_per_s": round(whole, 2),
            "pairs_iters_per_s": [round(v, 2) for v in rates],
            "fused_f64_pairs_iters_per_s": [round(v, 2) for v in f64_rates],
            "how": f"mpg_solve engine=surface (gmres.cpp's driver over kernels_hip.cpp), after a 2-cycle warm-up "
                   f"solve: (iters, time) of a {4 + cycles}-cycle solve minus a 4-cycle solve, median of 3 pairs; "
                   f"vs_fused against the headline rate, vs_fused_f64 against the fused engine timed the same way "
                   f"in the surface's accumulation class (f64)"}


def cpu_baseline(mpg, A, b, xt, opts, args, world=1, workload="BAND-10M", solve=None):
    """The oracle (kernels_mkl.cpp restatement over the image's MKL) on the
    host cores: per orthogonalisation, a 1-cycle warm-up, then up to
    `cpu_runs` timed solves of `cpu_cycles` restart cycles each, as many as
    fit the leg's wall-time budget (`cpu_budget_s`, split over the
    orthogonalisations; at least one timed solve each), and their median.
    `value` is the bench's own orthogonalisation (CGS by default, like the
    GPU line); `best` is the faster of it and MGS (the reference CLI's
    default, gmres_perf_test.cpp:320), so the GPU is also compared with the
    strongest host figure. `solve` replaces the oracle call (CPU tests)."""
    if solve is None:
        from oracle import binding

        solve, backend = binding.solve, binding.backend()
    else:
        backend = "test stub"
    t_leg = time.perf_counter()
    # (the shared-GPU rehearsal runs on one GPU's box: its share only)
    threads = cpu_threads(world, os.environ.get("MPG_BENCH_SHARED_GPU") == "1")
    info = _CPU_INFO or cpu_info()
    orths = list(dict.fromkeys([args.orth, "mgs"]))
    budget = float(getattr(args, "cpu_budget_s", 0) or 0)
    by_orth = {}
    for i, orth in enumerate(orths):
        t_orth = time.perf_counter()
        o = dict(opts, orth=orth, max_restarts=args.cpu_cycles, threads=threads)
        o.pop("device")
        o.pop("spmv_format", None)
        o.pop("accum", None)  # (MKL's fp32 BLAS: the f32 class by construction)
        solve(mpg, A, b, xt, **dict(o, max_restarts=1))  # warm-up: one cycle
        rates = []
        for r in range(args.cpu_runs):
            t_run = time.perf_counter()
            res = solve(mpg, A, b, xt, **o)
            rates.append(res.total_iters / res.gmres_seconds)
            if budget:  # stop when another solve would overrun this orthogonalisation's share
                share = budget * (i + 1) / len(orths) - (time.perf_counter() - t_leg)
                if time.perf_counter() - t_run > share:
                    break
        by_orth[orth] = {"median": round(float(np.median(rates)), 2), "runs": [round(x, 2) for x in rates],
                         "iterations_per_run": int(res.total_iters),
                         "wall_s": round(time.perf_counter() - t_orth, 2)}
        log(f"[bench] CPU oracle {orth}: median {by_orth[orth]['median']} it/s over {len(rates)} runs "
            f"({threads} threads, {by_orth[orth]['wall_s']} s)")
    best = max(by_orth, key=lambda k: by_orth[k]["median"])
    return {"value": by_orth[args.orth]["median"], "unit": "GMRES it/s", "cores": threads, "kind": "port",
            "best": by_orth[best]["median"], "best_orth": best,
            "sample": f"{args.cpu_cycles} restart cycles ({args.cpu_cycles * args.rlen} iterations) of the same "
                      f"{workload} GMRES({args.rlen}) {args.mode}/{args.orth} solve; a 1-cycle warm-up + median of "
                      f"up to {args.cpu_runs} (within a {budget or 'unlimited'} s leg budget); `best` is the faster "
                      f"of {' and '.join(orths)}; oracle backend {backend} (MKL restatement of kernels_mkl.cpp, "
                      f"GNU OpenMP threading, OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, "
                      f"OMP_PLACES={os.environ.get('OMP_PLACES')})",
            "by_orth": by_orth, "cpu_model": info["model"], "physical_cores": info["physical_cores"],
            "affinity_cpus": info["affinity_cpus"], "wall_s": round(time.perf_counter() - t_leg, 2)}


def vs_gpu(cpu: dict, gpu_rate: float) -> None:
    """GPU / CPU ratios: against the bench's own orthogonalisation and
    against the faster host configuration."""
    cpu["vs_gpu"] = round(gpu_rate / cpu["value"], 2) if cpu["value"] else None
    cpu["vs_gpu_best"] = round(gpu_rate / cpu["best"], 2) if cpu.get("best") else None


def visible_gpus() -> int:
    """GPUs a child process will see, counted in a child so that this
    process never initialises the GPU (it starts the ranks; an exec or fork
    after a HIP call is unsafe). torch.cuda.device_count() does not create
    a HIP context on this image."""
    out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                         capture_output=True, text=True, timeout=600)
    try:
        return int(out.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        log(f"[bench] could not count GPUs: {out.stderr.strip()[-400:]}")
        return 0


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """`bench.py --gpus N` without a launcher (WORLD_SIZE unset): start N
    rank processes of this script, one per GPU, before anything here touches
    the GPU (this process imports neither torch nor the HIP library). Each
    child gets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE /
    MASTER_ADDR=127.0.0.1 / MASTER_PORT, as torch.distributed.run would set
    them. Rank 0's stdout (the JSON line) is relayed; the other ranks'
    stdout goes to stderr. A failing rank ends the others and the exit code
    is non-zero; fewer visible GPUs than N is an error, never a silent N=1."""
    n = args.gpus
    shared = os.environ.get("MPG_BENCH_SHARED_GPU") == "1"
    if not args.dry_run:
        have = visible_gpus()
        need = 1 if shared else n
        if have < need:
            log(f"bench.py: --gpus {n} needs {need} visible GPU(s), found {have}"
                + ("" if shared else " (MPG_BENCH_SHARED_GPU=1 rehearses N ranks on one GPU over gloo)"))
            return 2
    port = int(os.environ.get("MASTER_PORT", "0") or 0) or free_port()
    procs = []
    for q in range(n):
        env = dict(os.environ, RANK=str(q), LOCAL_RANK=str(q), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MPG_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, "-u", str(Path(__file__).resolve()), *argv], env=env,
                                      stdout=subprocess.PIPE, text=True, start_new_session=True))
    lines = [[] for _ in procs]

    def pump(q, p):
        for ln in p.stdout:
            lines[q].append(ln)
            if q != 0:
                sys.stderr.write(f"[rank {q} stdout] {ln}")
                sys.stderr.flush()

    pumps = [threading.Thread(target=pump, args=(q, p), daemon=True) for q, p in enumerate(procs)]
    for t in pumps:
        t.start()
    rc = 0
    failed = None
    while True:
        codes = [p.poll() for p in procs]
        bad = [(q, c) for q, c in enumerate(codes) if c not in (None, 0)]
        if bad and failed is None:
            failed = bad[0]
            log(f"bench.py: rank {failed[0]} exited with {failed[1]}; ending the other ranks")
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGTERM)
            deadline = time.time() + 20
            while time.time() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGKILL)
        if all(c is not None for c in (p.poll() for p in procs)):
            break
        time.sleep(0.2)
    for t in pumps:
        t.join(timeout=5)
    if failed is not None:
        rc = failed[1] if failed[1] > 0 else 1
    for ln in lines[0]:
        sys.stdout.write(ln)
    sys.stdout.flush()
    return rc


# The collectives one CGS step of the row-partitioned engine issues on each
# rank (host/dist.cpp), all on the engine's own RCCL
# communicator, none on the torch process group (gloo: set-up and timing only).
STEP_COLLECTIVES = [
    "k >= 1: ncclGroupStart; ncclAllReduce(sum, fp64, the previous CGS update's 256 ||w||^2 partials, in place); "
    "ncclSend/ncclRecv of w_prev's halo rows (fp32, unnormalised) to/from each neighbour rank; ncclGroupEnd "
    "(FusedEngine::step, fold; k = 0: the halo send/recv group alone)",
    "ncclAllReduce(sum, fp64, the panel dots' (k+1) x 256 partials, in place) -- the CGS update sums them itself "
    "(k+1 <= 32; wider panels: a reduce launch + ncclAllReduce of the k+1 sums)",
]
CYCLE_COLLECTIVES = [
    "x halo send/recv (fp64) before the residual SpMV (FusedEngine::prologue)",
    "ncclAllReduce(sum, fp64, 3 sums: ||r||^2, ||x||^2, ||M r||^2) after the prologue's reduce",
    "the last step's Givens: reduce + ncclAllReduce(sum, fp64, 1) of ||w||^2",
]


def dry_run_line(args) -> None:
    """--dry-run: what this rank would run, without touching a GPU. At N > 1
    it also rehearses the CPU side of the set-up over the gloo group the real
    run uses: each rank builds its BAND row block (--n-local rows), analyses
    its halo and swaps the "rows I need from you" lists, and rank 0
    broadcasts a 128-byte stand-in for the RCCL unique id."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    line = {"dry_run": True, "rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
            "world": world, "gpus": args.gpus,
            "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}",
            "shared_gpu": os.environ.get("MPG_BENCH_SHARED_GPU") == "1"}
    if os.environ.get("MPG_BENCH_DRY_FAIL_RANK") == os.environ.get("RANK"):  # (tests: a rank that fails)
        print(json.dumps(line), flush=True)
        sys.exit(3)
    if world > 1 and args.n_local <= 100_000:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        mpg = load_pkg()
        starts = [q * args.n_local for q in range(world + 1)]
        A = mpg.gen_band(args.n_local * world, 5, 4, seed=7, row_begin=starts[rank], row_end=starts[rank + 1])
        plan = mpg.HaloPlan(rank, world, starts, A)
        needs = {q: plan.recv_rows(q).tolist() for q in range(world) if q != rank}
        gathered = [None] * world
        dist.all_gather_object(gathered, needs)
        sends = {q: gathered[q].get(rank, []) for q in range(world) if q != rank}
        for q, rows in sends.items():
            plan.set_send(q, rows)
        uid = [bytes(range(128)) if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        line.update(process_group=dist.get_backend(), uid_bytes=len(uid[0]) if uid[0] == bytes(range(128)) else -1,
                    halo_recv={q: len(v) for q, v in needs.items() if v},
                    halo_send={q: len(v) for q, v in sends.items() if v},
                    n_front=plan.n_front, n_ext=plan.n_ext,
                    step_collectives=STEP_COLLECTIVES, cycle_collectives=CYCLE_COLLECTIVES)
        plan.close()
        dist.barrier()
        dist.destroy_process_group()
    print(json.dumps(line), flush=True)


def measure(mpg, torch, dist, args, world, rank, local_rank, n, strong, keep=False) -> dict:
    """One row-partitioned BAND solve of n global rows (strong: split evenly
    over the ranks; weak: args.n_local rows per rank): build this rank's row
    block and engine, run the warm-up cycles, then time exactly args.steps
    restart cycles between a barrier + device synchronise on both sides; the
    time is the max over ranks. keep=True returns the engine (open) and the
    local problem for the roofline / surface / CPU legs."""
    starts = [n * q // world for q in range(world + 1)] if strong else [q * args.n_local for q in range(world + 1)]
    r0, r1 = starts[rank], starts[rank + 1]
    t0 = time.time()
    A = mpg.gen_band(n, 5, 4, seed=7, row_begin=r0, row_end=r1)
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    log(f"[bench] rank {rank}: BAND rows {r0}..{r1} of {n}, local nnz={A.nnz}, built in {time.time() - t0:.1f}s")

    opts = dict(mode=args.mode, orth=args.orth, prec=args.prec, rlen=args.rlen, tol=0.0,
                max_restarts=args.warmup + args.steps + 10, device=local_rank, spmv_format=args.spmv_format,
                accum=args.accum)
    if world == 1:
        eng = mpg.Engine(A, b, xt, **opts)
    else:
        # halo plan: exchange "rows I need from you" with every rank, then RCCL
        plan = mpg.HaloPlan(rank, world, starts, A)
        needs = {q: plan.recv_rows(q).tolist() for q in range(world) if q != rank}
        gathered = [None] * world
        dist.all_gather_object(gathered, needs)
        for q in range(world):
            if q != rank:
                plan.set_send(q, gathered[q].get(rank, []))
        if os.environ.get("MPG_BENCH_SHARED_GPU") == "1":
            # rehearsal on one GPU: the same engine, collectives through host
            # memory over gloo (RCCL refuses two ranks on one device)
            from mpgmres_amd.transport import HostTransport

            eng = mpg.Engine.distributed_host(A, b, xt[r0:r1], plan, HostTransport(), world, rank, **opts)
        else:
            uid = [mpg.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            eng = mpg.Engine.distributed(A, b, xt[r0:r1], plan, uid[0], world, rank, **opts)
    comm_ranks = eng.comm_ranks()
    eng.run(args.warmup)
    eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    it0 = eng.total_iters
    t_start = time.perf_counter()
    ran, done = eng.run(args.steps)
    eng.sync()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        dev = "cpu" if dist.get_backend() == "gloo" else "cuda"
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    iters = eng.total_iters - it0
    assert ran == args.steps and iters == args.steps * args.rlen, (ran, iters)
    rate = iters / elapsed
    log(f"[bench] n={n} ({'strong' if strong else 'weak'}): {args.steps} cycles, {iters} iterations in "
        f"{elapsed:.4f}s -> {rate:.1f} it/s; communicator ranks {comm_ranks}")
    out = {"r0": r0, "r1": r1, "rate": rate, "elapsed": elapsed, "comm_ranks": comm_ranks, "opts": opts}
    if keep:
        out.update(engine=eng, A=A, b=b, xt=xt)
    else:
        out["spmv_ms"] = spmv_roofline(eng, args.roofline_cycles)["avg_launch_ms"]
        out["layout"] = eng.spmv_layout()
        eng.close()
    return out


def claim_stdout():
    """The bench prints exactly one JSON line on stdout: everything else --
    including native libraries writing to fd 1 (gloo's connection notes,
    RCCL, HIP) -- goes to stderr. Returns a writer for the real stdout."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    sys.stdout = os.fdopen(os.dup(2), "w", buffering=1)
    return os.fdopen(real, "w", buffering=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed restart cycles")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-local", type=int, default=1_000_000, help="rows per GPU (weak scaling)")
    ap.add_argument("--global-rows", type=int, default=0,
                    help="strong scaling: one BAND matrix of this many rows split over the ranks")
    ap.add_argument("--rlen", type=int, default=30)
    ap.add_argument("--mode", default="mixed")
    ap.add_argument("--orth", default="cgs")
    ap.add_argument("--prec", default="identity")
    ap.add_argument("--cpu-cycles", type=int, default=2, help="restart cycles per CPU-baseline solve")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU-baseline solves (after 1 warm-up)")
    ap.add_argument("--cpu-budget-s", type=float, default=45.0,
                    help="wall-time budget of each CPU-baseline leg (timed solves stop when the next would overrun)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-cycles", type=int, default=3)
    ap.add_argument("--hbm-rows", type=int, default=10_000_000,
                    help="rows of the BAND matrix of the HBM-scale SpMV figure (0: skip)")
    ap.add_argument("--surface-cycles", type=int, default=20,
                    help="N = 1: restart cycles of the same solve through the drop-in operator surface (0: skip)")
    ap.add_argument("--spmv-format", default="auto", choices=["auto", "csr", "sell", "node"],
                    help="Arnoldi SpMV storage (auto: by the bytes each copy moves; node: 3x3 node blocks, "
                         "for 3-dof matrices only)")
    ap.add_argument("--accum", default="f32", choices=["f64", "f32"],
                    help="fp32 Arnoldi's accumulation class: f32 (default: every partial sum in fp32, the "
                         "reference's cblas_sdot / sgemv / mkl_sparse_s_mv class) or f64 (fp32 products summed in "
                         "fp64, rounded once)")
    ap.add_argument("--strong-rows", type=int, default=10_000_000,
                    help="N > 1: also time one BAND matrix of this many rows split over the ranks (the north "
                         "star's 100M-nnz strong-scaling case; 0: skip)")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks and report what each would run; no GPU work")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if args.dry_run:
        dry_run_line(args)
        return
    out = claim_stdout()

    # the CPU facts before anything binds this thread (libgomp pins the
    # initial thread to one place under OMP_PROC_BIND)
    global _CPU_INFO
    _CPU_INFO = cpu_info()
    # the CPU baseline's OpenMP placement (automated.py:13-15); libgomp reads
    # these when it is first loaded, which importing torch does
    os.environ.setdefault("OMP_PROC_BIND", "spread")
    os.environ.setdefault("OMP_PLACES", "threads")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: the launcher and the flag disagree")
        sys.exit(2)
    import torch  # first: the engine then shares PyTorch's HIP runtime

    mpg = load_pkg()
    shared_gpu = os.environ.get("MPG_BENCH_SHARED_GPU") == "1"
    if world > 1 and not shared_gpu:
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        have = torch.cuda.device_count()
        if have < local_world or local_rank >= have:
            log(f"bench.py: rank {rank} (local rank {local_rank}) needs {local_world} visible GPUs, found {have}")
            sys.exit(2)

    dist = None
    if world > 1:
        import torch.distributed as dist

        # The torch process group is gloo (host sockets) in both modes: it only
        # carries the set-up exchanges (halo "rows I need" lists, the RCCL
        # unique id), the barriers around the timed region and the max of the
        # elapsed times. The data path's collectives are the engine's own
        # RCCL communicator, the only NCCL/RCCL communicator a rank creates
        # (VERDICT r5 #6). MPG_BENCH_SHARED_GPU=1 rehearses the multi-rank path
        # with every rank on device 0 (engine collectives over the host
        # transport); the default is one GPU per rank over RCCL.
        if os.environ.get("MPG_BENCH_SHARED_GPU") == "1":
            local_rank = 0
        torch.cuda.set_device(local_rank)
        dist.init_process_group("gloo")

    strong = args.global_rows > 0
    n = args.global_rows if strong else args.n_local * world
    m = measure(mpg, torch, dist, args, world, rank, local_rank, n, strong, keep=True)
    eng, A, b, xt, opts = m["engine"], m["A"], m["b"], m["xt"], m["opts"]
    r0, r1, solve_rate, elapsed = m["r0"], m["r1"], m["rate"], m["elapsed"]
    global_nnz = 10 * n - 25
    value = solve_rate  # the one solve's iterations per second, at every N
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline of the dominant kernel: the Arnoldi SpMV as the cycle runs it
    sp = spmv_roofline(eng, args.roofline_cycles)
    pmc = pmc_traffic(REPO / "profiles")
    phases = (phase_roofline(eng, args.rlen, args.roofline_cycles, pmc)
              if args.orth == "cgs" and world == 1 and sp["timing"] == "dup" else None)
    # the whole CGS Arnoldi iteration on the same footing: the SpMV's storage
    # bytes + the panel dots and the CGS update at the cycle's mean k (the
    # once-per-cycle prologue and solution update are left out, so this
    # undercounts the bytes the measured rate moves)
    iter_bytes = (eng.phase_bytes("spmv_storage") + eng.phase_bytes("dots") + eng.phase_bytes("cgs_update")
                  if args.orth == "cgs" else None)
    eng.close()
    log(f"[bench] rank {rank} {sp['kernel']} in-cycle {sp['avg_launch_ms'] * 1e3:.2f} us/launch over {sp['launches']} "
        f"launches: {sp['achieved_gbs']:.0f} GB/s on its storage bytes, {sp['csr_equiv_gbs']:.0f} GB/s "
        f"CSR-equivalent; {sp['layout']}")
    per_rank_ms = [sp["avg_launch_ms"]]
    if dist:
        per_rank_ms = [None] * world
        dist.all_gather_object(per_rank_ms, sp["avg_launch_ms"])
    # N > 1: the north star's 100M-nnz strong-scaling case beside the default
    # weak one (one 1e7-row BAND matrix split over the ranks)
    strong100 = None
    if world > 1 and args.strong_rows > 0 and not (strong and n == args.strong_rows):
        sm = measure(mpg, torch, dist, args, world, rank, local_rank, args.strong_rows, True)
        sp_ms = [None] * world
        dist.all_gather_object(sp_ms, sm["spmv_ms"])
        strong100 = {"value": round(sm["rate"], 2), "unit": "GMRES iterations/s", "scaling": "strong",
                     "ms_per_step": round(1e3 * sm["elapsed"] / args.steps, 4), "steps": args.steps,
                     "rccl_ranks": sm["comm_ranks"] if not shared_gpu else None, "comm_ranks": sm["comm_ranks"],
                     "workload": f"BAND banded CSR n={args.strong_rows}, offsets -5..+4, "
                                 f"nnz={10 * args.strong_rows - 25}, split over {world} GPUs; GMRES({args.rlen}) "
                                 f"{args.mode}, {args.orth}, {args.prec}, tol=0",
                     "rows_per_gpu": sm["r1"] - sm["r0"],
                     "spmv_per_rank_avg_launch_ms": [round(t, 5) for t in sp_ms], "spmv_layout_rank0": sm["layout"]}
    surface = None
    if rank == 0 and world == 1 and args.surface_cycles > 0:
        surface = surface_rate(mpg, A, b, xt, opts, args.surface_cycles, solve_rate)
    roofline = None
    cpu = None
    if rank == 0:
        peak_read = mpg.bw_probe("read", 2 << 30, 3, local_rank)
        peak_copy = mpg.bw_probe("copy", 1 << 30, 3, local_rank)
        measured = max(peak_read, peak_copy)
        log(f"[bench] measured streaming peak: read {peak_read:.0f} GB/s, copy {peak_copy:.0f} GB/s")
        hbm = None
        if args.hbm_rows > 0 and world == 1:
            t1 = time.time()
            Ah = mpg.gen_band(args.hbm_rows, 5, 4, seed=7)
            xh = mpg.rand_vect(args.hbm_rows, 42)
            bh = mpg.host_spmv(Ah, xh)
            eh = mpg.Engine(Ah, bh, xh, **dict(opts, max_restarts=4))
            eh.run(1)
            hs = spmv_roofline(eh, 2)
            eh.close()
            del Ah, bh, xh
            hbm = {"workload": f"BAND n={args.hbm_rows}, nnz={10 * args.hbm_rows - 25} (working set > 256 MB "
                               f"Infinity Cache), same solve", "kernel": hs["kernel"], "timing": hs["timing"],
                   "avg_launch_ms": round(hs["avg_launch_ms"], 5), "bytes_per_launch": int(hs["storage_bytes"]),
                   "bytes_basis": "storage",
                   "achieved": round(hs["achieved_gbs"], 1), "frac": round(hs["achieved_gbs"] / HBM_PEAK_GBS, 4),
                   "frac_of_measured": round(hs["achieved_gbs"] / measured, 4),
                   "csr_equiv_bytes_per_launch": int(hs["csr_bytes"]),
                   "csr_equiv_achieved": round(hs["csr_equiv_gbs"], 1),
                   "csr_equiv_frac": round(hs["csr_equiv_gbs"] / HBM_PEAK_GBS, 4), "layout": hs["layout"]}
            log(f"[bench] HBM scale ({time.time() - t1:.1f}s): {hs['avg_launch_ms'] * 1e3:.1f} us/launch, "
                f"{hs['achieved_gbs']:.0f} GB/s on storage bytes")
        # the PMC figure of the committed profile belongs to this workload's
        # kernel only (BAND-10M, one GPU, m <= 32: tools/pmc_summary.py)
        key = sp["kernel"] + (":fold" if sp["layout"]["givens_folded"] else "")
        traffic = pmc.get(key) if world == 1 and args.rlen <= 32 and args.n_local == 1_000_000 else None
        # achieved / frac: the bytes the kernel really moves (PMC HBM bytes of
        # the committed profile when they belong to this run's kernel, else
        # its storage bytes) over the in-cycle launch time -- a physical
        # fraction of 8 TB/s. SURVEY 8(d)'s algorithmic CSR bytes,
        # which count column indices the implicit slices never read, are
        # reported beside it as csr_equiv_*.
        moved = traffic if traffic else sp["storage_bytes"]
        ach = moved / (sp["avg_launch_ms"] * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "bytes_per_launch": int(moved), "bytes_basis": "pmc" if traffic else "storage",
                    "kernel": sp["kernel"] + (" (in-cycle, Givens folded for k >= 1)" if sp["layout"]["givens_folded"]
                                              else " (in-cycle; the Givens step has its own launch)"),
                    "avg_launch_ms": round(sp["avg_launch_ms"], 5), "launches_timed": sp["launches"],
                    "timing": ("HIP events around graph replays of the cycle as run and with every SpMV launched "
                               "twice in a row; median replay-time difference over the added launches (kernel + "
                               "dispatch + release, the timed region's form)" if sp["timing"] == "dup" else
                               "hipExtLaunchKernel start/stop events of each launch of eager cycles"),
                    "event_graph_ms": round(sp["event_graph_ms"], 5) if sp["event_graph_ms"] else None,
                    "rocprof_avg_launch_ms": rocprof_avg_ms(REPO / "profiles", sp["kernel"]),
                    "storage_bytes_per_launch": int(sp["storage_bytes"]),
                    "storage_achieved": round(sp["achieved_gbs"], 1),
                    "storage_frac": round(sp["achieved_gbs"] / HBM_PEAK_GBS, 4),
                    "storage_formula": "what the SELL copy moves: slots x value bytes + stored columns (implicit "
                                       "slices read none) + slice offsets/pattern indices + 3 n s_T (w_prev read, "
                                       "v_k and w written)",
                    "csr_equiv_bytes_per_launch": int(sp["csr_bytes"]),
                    "csr_equiv_achieved": round(sp["csr_equiv_gbs"], 1),
                    "csr_equiv_frac": round(sp["csr_equiv_gbs"] / HBM_PEAK_GBS, 4),
                    "csr_equiv_formula": "SURVEY 8(d) B_spmv = nnz*(s_v+4) + (n+1)*4 + 2*n*s_x (algorithmic: "
                                         "the reference's CSR SpMV; above the bytes the SELL copy moves)",
                    "measured_peak": round(measured, 1), "measured_peak_read": round(peak_read, 1),
                    "measured_peak_copy": round(peak_copy, 1),
                    "frac_of_measured": round(ach / measured, 4),
                    "storage_frac_of_measured": round(sp["achieved_gbs"] / measured, 4),
                    "phases": phases,
                    "cache_note": "the BAND-10M Arnoldi working set (~190 MB) fits the 256 MB Infinity Cache; "
                                  "hbm_scale is the same kernel past it",
                    "hbm_scale": hbm, "rank": 0,
                    "per_rank_avg_launch_ms": [round(t, 5) for t in per_rank_ms]}
        if world > 1:
            roofline["kernel"] = sp["kernel"] + (" (in-cycle, rank 0's row block; Givens folded for k >= 1, its "
                                                 "||w||^2 partials all-reduced with the halo)"
                                                 if sp["layout"]["givens_folded"]
                                                 else " (in-cycle, rank 0's row block; the Givens step has its own launch)")
            if shared_gpu:
                roofline["note"] = "rehearsal: all ranks share GPU 0, so each rank's launches overlap the others'"
        if iter_bytes:
            ach = iter_bytes * solve_rate / 1e9
            roofline["iteration"] = {
                "bytes": int(iter_bytes), "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "frac_of_measured": round(ach / measured, 4),
                "formula": "per CGS iteration at the cycle's mean k: SpMV storage bytes + panel dots (V(:,0..k), w "
                           "read) + CGS update (V(:,0..k) read, w read + written); x solve_iters_per_s; the "
                           "once-per-cycle residual prologue and solution update are not counted"}
            log(f"[bench] whole iteration: {iter_bytes / 1e6:.1f} MB x {solve_rate:.0f} it/s = {ach:.0f} GB/s "
                f"({ach / HBM_PEAK_GBS:.3f} of 8 TB/s, {ach / measured:.3f} of measured)")
        if not args.no_cpu_baseline:
            if world == 1:
                cpu = cpu_baseline(mpg, A, b, xt, opts, args)
            else:
                # the same global matrix on the host (the GPU ranks hold row
                # blocks of it), fewer timed runs at this size
                t2 = time.time()
                Ag = mpg.gen_band(n, 5, 4, seed=7)
                bg = mpg.host_spmv(Ag, xt)
                cargs = argparse.Namespace(**dict(vars(args), cpu_runs=min(args.cpu_runs, 3)))
                cpu = cpu_baseline(mpg, Ag, bg, xt, opts, cargs, world, f"BAND n={n} ({global_nnz} nnz)")
                log(f"[bench] CPU baseline on the global matrix took {time.time() - t2:.1f}s")
                del Ag, bg
            vs_gpu(cpu, value)
            if strong100 is not None:
                t3 = time.time()
                As = mpg.gen_band(args.strong_rows, 5, 4, seed=7)
                xs = mpg.rand_vect(args.strong_rows, 42)
                bs = mpg.host_spmv(As, xs)
                cargs = argparse.Namespace(**dict(vars(args), cpu_runs=min(args.cpu_runs, 3)))
                sc = cpu_baseline(mpg, As, bs, xs, opts, cargs, world,
                                  f"BAND n={args.strong_rows} ({10 * args.strong_rows - 25} nnz)")
                vs_gpu(sc, strong100["value"])
                strong100["cpu_baseline"] = sc
                log(f"[bench] strong case: {strong100['value']:.0f} it/s on {world} GPUs vs {sc['value']} it/s "
                    f"on {sc['cores']} host cores ({sc['vs_gpu']}x; best host {sc['best']} it/s, "
                    f"{sc['vs_gpu_best']}x); CPU leg took {time.time() - t3:.1f}s")
                del As, bs, xs

    if rank == 0:
        scaling = "strong" if strong else "weak"
        if strong100 is not None and "cpu_baseline" not in strong100:
            strong100["cpu_baseline"] = None
        transport = ("RCCL" if not shared_gpu else
                     "the gloo host transport, every rank on GPU 0 (rehearsal; RCCL refuses two ranks on one GPU)")
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GMRES iterations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "accum": {"f32": "f32: every dot / norm / gemv / SpMV partial sum of the fp32 Arnoldi in fp32 (the "
                             "reference's cblas_s* / mkl_sparse_s_mv class)",
                      "f64": "f64: the fp32 Arnoldi's products summed in fp64, rounded once"}[args.accum],
            "data": "synthetic", "roofline": roofline, "cpu_baseline": cpu,
            "solve_iters_per_s": round(solve_rate, 2), "surface": surface,
            "rccl_ranks": m["comm_ranks"] if world > 1 and not shared_gpu else None,
            "comm_ranks": m["comm_ranks"], "strong_100m": strong100,
            "surface_iters_per_s": surface["iters_per_s"] if surface else None,
            "aggregate": (None if strong or world == 1 else
                          {"value": round(solve_rate * world, 2),
                           "unit": "GMRES iterations x 10M-nnz row blocks (one per GPU) per second"}),
            "config": {"workload": f"BAND banded CSR n={n}, offsets -5..+4, nnz={global_nnz} "
                                   f"({'split over' if strong else '1e6 rows = 10M nnz per GPU,'} {world} GPU(s)); "
                                   f"GMRES({args.rlen}) {args.mode} (fp32 Arnoldi, {args.accum} accumulation, "
                                   f"fp64 residual/update), "
                                   f"{args.orth}, {args.prec} preconditioner, tol=0",
                       "step": f"one restart cycle = {args.rlen} iterations",
                       "value_counts": "GMRES iterations of the one (row-partitioned) solve per second",
                       "rows_per_gpu": (r1 - r0), "nnz": global_nnz, "spmv_storage": sp["layout"],
                       "parallelism": (f"row-partition x{world} (halo send/recv + fp64 all-reduce over {transport})"
                                       if world > 1 else "one GPU")},
        }
        out.write(json.dumps(line) + "\n")
        out.flush()
    if dist:
        dist.barrier()  # the other ranks wait for rank 0's measurements
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
