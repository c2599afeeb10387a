"""Single-GPU throughput on the BASELINE.json configs other than the
headline bench (one MI355X): GMRES iterations/s of the fused engine at
tol = 0 (fixed work), the Arnoldi SpMV's achieved algorithmic GB/s
(SURVEY §8(d) B_spmv), and the CPU oracle on a bounded sample of the same
solve. Synthetic inputs:
  C2  LAP-1M   7-point 3-D Laplacian 100^3, fp64 GMRES(30) (baseline mode)
  C3  LAP-1M   fp32 Arnoldi + fp64 residual/update (mixed mode)
  C4  Queen_4147 stand-in: 27-point 3-D stencil, 3 dof/node, 111^3 nodes
      (n = 4.1M, 3.26e8 nnz), fp32 Arnoldi (mixed mode)
  C5  BAND-100M at one GPU: n = 1e7, fp16 Arnoldi values (mixed-half)
      (BASELINE quotes it on 8 GPUs; here one GPU holds the whole matrix)
Prints one JSON line per case; `--out FILE` also writes them to FILE.

usage: python tools/bench_configs.py [--cycles 10] [--cpu-cycles 2] [--only C4] [--out profiles/r01_configs.jsonl]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

CASES = [
    dict(name="C2 LAP-1M fp64 CGS", matrix=("laplace", 100), mode="baseline", orth="cgs"),
    dict(name="C2 LAP-1M fp64 MGS", matrix=("laplace", 100), mode="baseline", orth="mgs"),
    dict(name="C3 LAP-1M mixed CGS", matrix=("laplace", 100), mode="mixed", orth="cgs"),
    dict(name="C3 LAP-1M mixed MGS", matrix=("laplace", 100), mode="mixed", orth="mgs"),
    dict(name="C3 LAP-1M mixed CGSR", matrix=("laplace", 100), mode="mixed", orth="cgsr"),
    dict(name="C4 Queen-stand-in mixed CGS", matrix=("stencil27", 111), mode="mixed", orth="cgs"),
    dict(name="C5 BAND-100M mixed-half CGS (1 GPU)", matrix=("band", 10_000_000), mode="mixed-half", orth="cgs"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--cpu-cycles", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated case prefixes, e.g. C4,C5")
    args = ap.parse_args()
    from __graft_entry__ import _load

    mpg = _load()
    from oracle import binding

    lines = []
    only = tuple(args.only.split(",")) if args.only else None
    gens = {"laplace": mpg.gen_laplace3d, "stencil27": lambda s: mpg.gen_stencil27(s, 3),
            "band": lambda s: mpg.gen_band(s, 5, 4, seed=7)}
    for case in CASES:
        if only and not case["name"].startswith(only):
            continue
        kind, size = case["matrix"]
        t0 = time.time()
        A = gens[kind](size)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode=case["mode"], orth=case["orth"], prec="identity", rlen=30, tol=0.0,
                    max_restarts=args.cycles + 10)
        eng = mpg.Engine(A, b, xt, **opts)
        eng.run(2)
        eng.sync()
        it0 = eng.total_iters
        t = time.perf_counter()
        eng.run(args.cycles)
        eng.sync()
        dt = time.perf_counter() - t
        its = (eng.total_iters - it0) / dt
        # the Arnoldi SpMV as the cycle runs it, each launch timed by its own
        # kernel events (bench.py's roofline measurement), on the bytes its
        # storage moves and on SURVEY 8(d)'s CSR bytes
        spmv_ms, per = eng.time_spmv_incycle(2)
        gbs = eng.phase_bytes("spmv") / (spmv_ms * 1e-3) / 1e9
        gbs_storage = eng.phase_bytes("spmv_storage") / (spmv_ms * 1e-3) / 1e9
        layout = eng.spmv_layout()
        eng.close()
        cpu = None
        if args.cpu_cycles > 0:
            # the 1e8-nnz-scale matrices: one restart cycle; the oracle has no
            # fp16 mode, so mixed-half is timed as its fp32-value mixed solve
            cyc = args.cpu_cycles if kind == "laplace" else 1
            cmode = "mixed" if case["mode"] == "mixed-half" else case["mode"]
            r = binding.solve(mpg, A, b, xt, **dict(opts, mode=cmode, max_restarts=cyc))
            cpu = {"it_s": round(r.total_iters / r.gmres_seconds, 2), "iterations": int(r.total_iters),
                   "mode": cmode, "threads": binding.lib().oracle_max_threads(), "backend": binding.backend()}
        line = {"case": case["name"], "n": A.nrows, "nnz": A.nnz, "mode": case["mode"], "orth": case["orth"],
                "gmres_it_s": round(its, 1), "spmv_us": round(spmv_ms * 1e3, 2), "spmv_gbs": round(gbs, 1),
                "spmv_frac_8tbs": round(gbs / 8000, 3), "spmv_storage_gbs": round(gbs_storage, 1),
                "spmv_storage_frac_8tbs": round(gbs_storage / 8000, 3), "spmv_timing": "in-cycle kernel events",
                "spmv_storage": layout, "cpu_oracle": cpu,
                "gpu_over_cpu": round(its / cpu["it_s"], 1) if cpu else None,
                "setup_s": round(time.time() - t0 - dt, 1)}
        print(json.dumps(line), flush=True)
        lines.append(line)
    if args.out:
        Path(args.out).write_text("".join(json.dumps(x) + "\n" for x in lines))


if __name__ == "__main__":
    main()
