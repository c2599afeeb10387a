#!/usr/bin/env python3
"""How long does the in-cycle Arnoldi SpMV take? Three clocks on one engine,
in this order, so a rocprofv3 --kernel-trace of this script can be split
by launch index and set beside each:
  1. `--warm` graph-replayed restart cycles (the bench's timed region;
     no timing of our own: rocprof alone),
  2. `--eager` eager cycles, every SpMV launch timed by its own
     hipExtLaunchKernel start/stop events (mpg_engine_time_spmv_incycle),
  3. `--graph` replays of the cycle captured with an event-record node on
     each side of every SpMV (mpg_engine_time_phase_graph),
  4. replays of the cycle as run and with every SpMV launched twice in a
     row, HIP events around whole replays (mpg_engine_time_phase_dup: what
     one launch adds to the cycle, no packet near the kernel).
Prints one JSON line: the mean of 2, 3 and 4, the launch counts of each
block (m per cycle) and the workload. With --torch, PyTorch's HIP runtime is
loaded first, as in bench.py.
usage: python tools/timing_probe.py [--rows 1000000] [--rlen 30]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--rlen", type=int, default=30)
    ap.add_argument("--orth", default="cgs")
    ap.add_argument("--warm", type=int, default=4)
    ap.add_argument("--eager", type=int, default=3)
    ap.add_argument("--graph", type=int, default=5)
    ap.add_argument("--torch", action="store_true")
    args = ap.parse_args()
    if args.torch:
        import torch

        torch.cuda.synchronize()
    from __graft_entry__ import _load

    mpg = _load()
    A = mpg.gen_band(args.rows, 5, 4, seed=7)
    xt = mpg.rand_vect(args.rows, 42)
    b = mpg.host_spmv(A, xt)
    eng = mpg.Engine(A, b, xt, mode="mixed", orth=args.orth, prec="identity", rlen=args.rlen, tol=0.0,
                     max_restarts=args.warm + 10)
    eng.run(args.warm)
    eng.sync()
    e_ms, e_per = eng.time_spmv_incycle(args.eager)
    g_ms, g_per = eng.time_phase_graph("spmv", args.graph)
    d_ms, d_added = eng.time_phase_dup("spmv", max(5, args.graph))
    phases = {}
    for ph in ("dots", "cgs_update"):
        d_ms_ph, _ = eng.time_phase_dup(ph, max(5, args.graph))
        phases[f"{ph}_dup_us"] = round(1e3 * d_ms_ph, 3)
        for clock, fn in (("graph_events", eng.time_phase_graph), ("stamps", eng.time_phase_stamps)):
            try:
                ms, per = fn(ph, args.graph)
            except RuntimeError as ex:  # (stamps: only the one-panel forms, k + 1 <= 32)
                phases[f"{ph}_{clock}"] = str(ex)
                continue
            m = args.rlen
            byk = np.asarray(per[:len(per) // m * m]).reshape(-1, m).mean(axis=0) * 1e3 if len(per) % m == 0 \
                else np.asarray(per) * 1e3
            b, a = np.polyfit(np.arange(len(byk)), byk, 1)
            phases[f"{ph}_{clock}"] = {"mean_us": round(1e3 * ms, 3), "launches": len(per), "fit_a_us": round(float(a), 3),
                                       "fit_b_us": round(float(b), 4)}
    lay = eng.spmv_layout()
    eng.close()
    m = args.rlen
    print(json.dumps({
        "workload": f"BAND n={args.rows} mixed {args.orth} GMRES({m})", "layout": lay,
        "blocks": {"warm_graph": args.warm * m, "eager_events": len(e_per), "graph_events": len(g_per),
                   "dup_added": d_added},
        "dup_us": round(1e3 * d_ms, 3),
        "eager_event_us": round(1e3 * e_ms, 3), "eager_event_median_us": round(1e3 * float(np.median(e_per)), 3),
        "graph_event_us": round(1e3 * g_ms, 3), "graph_event_median_us": round(1e3 * float(np.median(g_per)), 3),
        "phases": phases,
    }), flush=True)


if __name__ == "__main__":
    main()
