#!/usr/bin/env python3
"""GMRES iterations/s on MI355X for the BASELINE.json metric.

Workload (BASELINE.json metric "GMRES iterations/sec + SpMV achieved HBM GB/s,
10M-nnz CSR, 1/2/4/8 GPUs"): the synthetic banded CSR "BAND-10M" (n = 1e6
rows per GPU, column offsets -5..+4, 9,999,975 nnz at one GPU; values from
the counter-based generator of include/mpgmres/problems.h), x_true =
rand_vect(n, 42), b = A x_true, restarted GMRES(30), mixed precision
(fp32 Arnoldi + fp64 residual/update: gmres_singleUpdate), CGS, identity
preconditioner, tol = 0 so the solve never stops early.

One step = one restart cycle = check_initial on the host + 30 Arnoldi
iterations + solution update + the next true-residual prologue (the fused
engine's graph replay). value = iterations/s of the whole job; with N GPUs
each rank owns a 1e6-row slice of an N*1e6-row BAND matrix (weak scaling)
and value counts iterations x N shards.

Also reported: the roofline of the dominant kernel (the Arnoldi SpMV phase,
k_step_spmv) from HIP events on the engine's stream, and the CPU oracle
(MKL restatement of kernels_mkl.cpp) on a bounded sample of the same solve.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "GMRES iterations/sec + SpMV achieved HBM GB/s, 10M-nnz CSR, 1/2/4/8 GPUs"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def stream_copy_peak(torch, nbytes=1 << 30, reps=5):
    """Measured device-to-device copy rate (read + write bytes / s) of a
    1 GiB fp32 buffer — larger than the 256 MB Infinity Cache, so it is HBM."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device="cuda").fill_(1.0)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    e1.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return gbs


def load_pkg():
    from __graft_entry__ import _load

    return _load()


def pmc_traffic(profile_dir: Path, kernel_prefix: str):
    """HBM bytes per launch of the dominant kernel from a committed rocprofv3
    PMC summary (profiles/*pmc*.json written by tools/pmc_summary.py), or None."""
    f = profile_dir / "pmc_traffic.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        return d.get(kernel_prefix, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed restart cycles")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n-local", type=int, default=1_000_000, help="rows per GPU")
    ap.add_argument("--rlen", type=int, default=30)
    ap.add_argument("--mode", default="mixed")
    ap.add_argument("--orth", default="cgs")
    ap.add_argument("--prec", default="identity")
    ap.add_argument("--cpu-cycles", type=int, default=4, help="restart cycles in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-reps", type=int, default=10)
    ap.add_argument("--spmv-format", default="auto", choices=["auto", "csr", "sell"],
                    help="Arnoldi SpMV storage (auto: SELL-64 when its padding is small)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    mpg = load_pkg()
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        # MPG_BENCH_SHARED_GPU=1 rehearses the multi-rank path with every rank on
        # device 0 (torch side on gloo); the default is one GPU per rank over RCCL
        if os.environ.get("MPG_BENCH_SHARED_GPU") == "1":
            local_rank = 0
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    # global BAND matrix of world * n_local rows; this rank owns one row block
    n = args.n_local * world
    r0, r1 = rank * args.n_local, (rank + 1) * args.n_local
    t0 = time.time()
    A = mpg.gen_band(n, 5, 4, seed=7, row_begin=r0, row_end=r1)
    xt = mpg.rand_vect(n, 42)
    b = mpg.host_spmv(A, xt)
    global_nnz = 10 * n - 25
    log(f"[bench] rank {rank}: BAND rows {r0}..{r1} of {n}, local nnz={A.nnz}, built in {time.time() - t0:.1f}s")

    opts = dict(mode=args.mode, orth=args.orth, prec=args.prec, rlen=args.rlen, tol=0.0,
                max_restarts=args.warmup + args.steps + 10, device=local_rank, spmv_format=args.spmv_format)
    if world == 1:
        eng = mpg.Engine(A, b, xt, **opts)
    else:
        # halo plan: exchange "rows I need from you" with every rank, then RCCL
        starts = [q * args.n_local for q in range(world + 1)]
        plan = mpg.HaloPlan(rank, world, starts, A)
        needs = {q: plan.recv_rows(q).tolist() for q in range(world) if q != rank}
        gathered = [None] * world
        dist.all_gather_object(gathered, needs)
        for q in range(world):
            if q != rank:
                plan.set_send(q, gathered[q].get(rank, []))
        uid = [mpg.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng = mpg.Engine.distributed(A, b, xt[r0:r1], plan, uid[0], world, rank, **opts)
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
    value = iters * world / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    log(f"[bench] {args.steps} cycles, {iters} iterations in {elapsed:.4f}s -> {iters / elapsed:.1f} it/s")

    # roofline of the dominant kernel: the Arnoldi SpMV phase, mean over k
    layout = eng.spmv_layout()
    kernel = "k_step_sell" if layout["format"] == "sell" else "k_step_spmv"
    avg_ms = eng.time_phase("spmv", args.roofline_reps)
    bytes_per_launch = eng.phase_bytes("spmv")
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = pmc_traffic(REPO / "profiles", kernel)
    stream = stream_copy_peak(torch)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "kernel": kernel, "avg_launch_ms": round(avg_ms, 5),
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "bytes_formula": "SURVEY 8(d) B_spmv = nnz*(s_v+4) + (n+1)*4 + 2*n*s_x",
                "measured_copy_peak": round(stream, 1), "frac_of_measured": round(achieved / stream, 4)}
    log(f"[bench] {kernel} {avg_ms * 1e3:.1f} us/launch, {achieved:.0f} GB/s algorithmic, storage {layout}; "
        f"measured copy peak {stream:.0f} GB/s")
    eng.close()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import binding

        cpu_opts = dict(opts, max_restarts=args.cpu_cycles)
        cpu_opts.pop("device")
        r = binding.solve(mpg, A, b, xt, **cpu_opts)
        cpu_its = r.total_iters / r.gmres_seconds
        cpu = {"value": round(cpu_its, 2), "unit": "GMRES it/s", "cores": binding.lib().oracle_max_threads(),
               "kind": "port",
               "sample": f"{r.total_iters} iterations ({args.cpu_cycles} restart cycles) of the same BAND-10M "
                         f"GMRES({args.rlen}) {args.mode}/{args.orth} solve, oracle backend "
                         f"{binding.backend()} (MKL restatement of kernels_mkl.cpp)"}
        log(f"[bench] CPU oracle: {cpu_its:.2f} it/s on {cpu['cores']} threads")

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GMRES iterations/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic", "roofline": roofline, "cpu_baseline": cpu,
            "config": {"workload": f"BAND-10M per GPU: banded CSR n={n}, offsets -5..+4, nnz={global_nnz}; "
                                   f"GMRES({args.rlen}) {args.mode} (fp32 Arnoldi, fp64 residual/update), "
                                   f"{args.orth}, {args.prec} preconditioner, tol=0",
                       "step": f"one restart cycle = {args.rlen} iterations",
                       "value_counts": "GMRES iterations x 10M-nnz row blocks (one per GPU) per second",
                       "rows_per_gpu": args.n_local, "nnz": global_nnz,
                       "spmv_storage": layout,
                       "parallelism": f"row-partition x{world} (halo send/recv + fp64 all-reduce over RCCL)"},
        }
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
