"""GMRES it/s with each preconditioner on one MI355X (fused engine, mixed
CGS GMRES(30), tol = 0, fixed work): identity, Jacobi, ILU(0) (sync-free
triangular solves) and ILU-Jacobi (5 sweeps), on LAP-1M (the 100^3 7-point
Laplacian, triangular-solve depth ~ 300) and a BAND matrix (depth = n).

usage: python tools/prec_bench.py [--cycles 3]"""
import argparse
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from __graft_entry__ import _load


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=3)
    args = ap.parse_args()
    mpg = _load()
    mats = {"LAP-1M": lambda: mpg.gen_laplace3d(100), "BAND-100k": lambda: mpg.gen_band(100_000, 5, 4, seed=7)}
    for name, gen in mats.items():
        A = gen()
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        for prec in ("identity", "jacobi", "ilu", "ilu_jacobi"):
            opts = dict(mode="mixed", orth="cgs", prec=prec, rlen=30, tol=0.0)
            t0 = time.time()
            eng = mpg.Engine(A, b, xt, max_restarts=args.cycles + 3, **opts)
            setup = time.time() - t0
            eng.run(1)
            eng.sync()
            it0 = eng.total_iters
            t = time.perf_counter()
            eng.run(args.cycles)
            eng.sync()
            dt = time.perf_counter() - t
            its = eng.total_iters - it0
            eng.close()
            print(json.dumps({"matrix": name, "prec": prec, "it_s": round(its / dt, 1),
                              "setup_s": round(setup, 3)}), flush=True)


if __name__ == "__main__":
    main()
