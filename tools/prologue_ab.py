"""Interleaved A/B of the residual prologue's storage on node-block matrices:
MPG_NODE_PROLOGUE=1 (row sums on the fp64 node copy + the CSR prologue's
epilogue) against 0 (the CSR prologue), fused engine, GMRES(30) mixed CGS at
tol = 0, each engine timed over `--cycles` restart cycles after 2 warm-up
cycles, `--reps` interleaved rounds; prints one JSON line per spec.

usage: python tools/prologue_ab.py [--spec stencil27:111 --spec fem27:111] [--cycles 6] [--reps 3]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", action="append")
    ap.add_argument("--cycles", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    from __graft_entry__ import _load

    mpg = _load()
    for spec in args.spec or ["stencil27:111", "fem27:111"]:
        A = mpg.gen_spec(spec)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=10 ** 6,
                    accum="f32")
        engs = {}
        for v in ("0", "1"):
            os.environ["MPG_NODE_PROLOGUE"] = v
            engs[v] = mpg.Engine(A, b, xt, **opts)
            engs[v].run(2)
            engs[v].sync()
        os.environ.pop("MPG_NODE_PROLOGUE")
        rates = {v: [] for v in engs}
        for _ in range(args.reps):
            for v, e in engs.items():
                it0 = e.total_iters
                t = time.perf_counter()
                e.run(args.cycles)
                e.sync()
                rates[v].append((e.total_iters - it0) / (time.perf_counter() - t))
        line = {"spec": spec, "prologue": {v: engs[v].spmv_layout()["prologue"] for v in engs},
                "it_s": {v: round(float(np.median(r)), 1) for v, r in rates.items()},
                "runs": {v: [round(x, 1) for x in r] for v, r in rates.items()}}
        for e in engs.values():
            e.close()
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
