"""The row-partitioned (multi-GPU) engine path on ONE rank over RCCL, against
the single-GPU engine, on BAND-10M: what the distributed step structure
costs before any interconnect latency (the one-rank collectives are local).
Mixed CGS / MGS GMRES(30), tol = 0.

usage: python tools/dist1_bench.py [--cycles 20]"""
import argparse
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from __graft_entry__ import _load


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=20)
    args = ap.parse_args()
    mpg = _load()
    A = mpg.gen_band(1_000_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    for orth in ("cgs", "mgs"):
        opts = dict(mode="mixed", orth=orth, prec="identity", rlen=30, tol=0.0, max_restarts=args.cycles + 10)
        for kind in ("single", "dist1"):
            if kind == "single":
                eng = mpg.Engine(A, b, xt, **opts)
            else:
                plan = mpg.HaloPlan(0, 1, [0, A.nrows], A)
                eng = mpg.Engine.distributed(A, b, xt, plan, mpg.rccl_unique_id(), 1, 0, **opts)
            eng.run(2)
            eng.sync()
            it0 = eng.total_iters
            t = time.perf_counter()
            eng.run(args.cycles)
            eng.sync()
            dt = time.perf_counter() - t
            its = (eng.total_iters - it0) / dt
            eng.close()
            print(f"{orth} {kind}: {its:.1f} it/s", flush=True)


if __name__ == "__main__":
    main()
