"""Interleaved A/B of Arnoldi SpMV variants selected by environment flags
read at launch time (e.g. MPG_SELL_UNIFORM), on one engine per matrix: the
in-cycle SpMV (Givens folded) timed by its own kernel events
(mpg_engine_time_spmv_incycle), median over `--reps` interleaved rounds.

usage: python tools/spmv_ab.py --case band100m-half --var MPG_SELL_UNIFORM=0 --var MPG_SELL_UNIFORM=1
cases: band10m, band100m, band100m-half, lap1m, lap1m-f64, c4, c4p, fem27, fem27p"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

CASES = {
    "band10m": ("band:1000000", "mixed"),
    "band100m": ("band:10000000", "mixed"),
    "band100m-half": ("band:10000000", "mixed-half"),
    "lap1m": ("laplace:100", "mixed"),
    "lap1m-f64": ("laplace:100", "baseline"),
    "c4": ("stencil27:111", "mixed"),
    # irregular stand-ins (mpg_gen_spec): C4 under a node-block permutation,
    # the thinned 27-point coupling in natural and permuted order
    "c4p": ("stencil27p:111", "mixed"),
    "fem27": ("fem27:111", "mixed"),
    "fem27p": ("fem27:111:3:70:13:64", "mixed"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", action="append", required=True)
    ap.add_argument("--var", action="append", required=True, help="NAME=VALUE[,NAME=VALUE] per variant")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cycles", type=int, default=2)
    ap.add_argument("--accum", default="f32", help="accumulation class of the fp32 Arnoldi (f32 | f64)")
    args = ap.parse_args()
    from __graft_entry__ import _load

    mpg = _load()
    variants = [dict(kv.split("=", 1) for kv in v.split(",")) for v in args.var]
    for case in args.case:
        spec, mode = CASES[case]
        A = mpg.gen_spec(spec)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        def with_env(v, fn):
            saved = {k: os.environ.get(k) for k in v}
            os.environ.update(v)
            try:
                return fn()
            finally:
                for k, old in saved.items():
                    if old is None:
                        os.environ.pop(k)
                    else:
                        os.environ[k] = old

        # one engine per variant, created and timed under its flags (flags
        # read at engine creation, e.g. MPG_FOLD_GIVENS, and at launch)
        engs = []
        for v in variants:
            # (a variant's spmv_format=auto|csr|sell picks the storage; the rest are environment flags)
            fmt = v.pop("spmv_format", "auto")
            e = with_env(v, lambda: mpg.Engine(A, b, xt, mode=mode, orth="cgs", prec="identity", rlen=30, tol=0.0,
                                              max_restarts=1000, spmv_format=fmt,
                                              accum=args.accum))
            v["spmv_format"] = fmt
            with_env(v, lambda: e.run(1))
            engs.append(e)
        times = [[] for _ in variants]
        for _ in range(args.reps):
            for i, v in enumerate(variants):
                env = {k: x for k, x in v.items() if k != "spmv_format"}
                ms, _ = with_env(env, lambda: engs[i].time_spmv_incycle(args.cycles))
                times[i].append(ms * 1e3)
        for v, t, e in zip(variants, times, engs):
            med = float(np.median(t))
            storage = e.phase_bytes("spmv_storage")
            print(json.dumps({"case": case, "variant": v, "us_median": round(med, 2), "us": [round(x, 2) for x in t],
                              "storage_mb": round(storage / 1e6, 2),
                              "storage_tbs": round(storage / (med * 1e-6) / 1e12, 3),
                              "layout": dict(e.spmv_layout(), **e.sell_columns())}), flush=True)
            e.close()
        del A, b, xt


if __name__ == "__main__":
    main()
