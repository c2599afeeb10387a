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

  M100 GMRES(100) on BAND-10M / LAP-1M (CGS, CGSR, MGS)
  IRR  irregular stand-ins: stencil27p (C4 under a node-block permutation),
       fem27 (thinned 27-point coupling, variable rows), natural / permuted
Inputs by their CLI spec (mpg_gen_spec).

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
    dict(name="C2 LAP-1M fp64 CGS", spec="laplace:100", mode="baseline", orth="cgs"),
    dict(name="C2 LAP-1M fp64 MGS", spec="laplace:100", mode="baseline", orth="mgs"),
    dict(name="C3 LAP-1M mixed CGS", spec="laplace:100", mode="mixed", orth="cgs"),
    dict(name="C3 LAP-1M mixed MGS", spec="laplace:100", mode="mixed", orth="mgs"),
    dict(name="C3 LAP-1M mixed CGSR", spec="laplace:100", mode="mixed", orth="cgsr"),
    dict(name="C4 Queen-stand-in mixed CGS", spec="stencil27:111", mode="mixed", orth="cgs"),
    dict(name="C5 BAND-100M mixed-half CGS (1 GPU)", spec="band:10000000", mode="mixed-half", orth="cgs"),
    # GMRES(100), the reference's published restart length (automated.py:41):
    # the 404 MB fp32 basis of BAND-10M no longer fits the 256 MB Infinity
    # Cache, so the panel kernels run from HBM
    dict(name="M100 BAND-10M mixed CGS", spec="band:1000000", mode="mixed", orth="cgs", rlen=100),
    dict(name="M100 BAND-10M mixed CGSR", spec="band:1000000", mode="mixed", orth="cgsr", rlen=100),
    dict(name="M100 BAND-10M mixed MGS", spec="band:1000000", mode="mixed", orth="mgs", rlen=100, cycles=3),
    dict(name="M100 LAP-1M mixed CGS", spec="laplace:100", mode="mixed", orth="cgs", rlen=100),
    dict(name="M100 LAP-1M fp64 CGS", spec="laplace:100", mode="baseline", orth="cgs", rlen=100),
    # irregular stand-ins (VERDICT r3 missing #2): the C4 stencil under a
    # symmetric node-block permutation (Queen-like scatter, same spectrum) and
    # a FEM-like randomly thinned 27-point coupling with variable rows
    dict(name="IRR Queen-like permuted stencil27 mixed CGS", spec="stencil27p:111", mode="mixed", orth="cgs"),
    dict(name="IRR FEM-like fem27 natural order mixed CGS", spec="fem27:111", mode="mixed", orth="cgs"),
    dict(name="IRR FEM-like fem27 permuted mixed CGS", spec="fem27:111:3:70:13:64", mode="mixed", orth="cgs"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--cpu-cycles", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="comma-separated case prefixes, e.g. C4,C5")
    ap.add_argument("--accum", default="f32", choices=["f64", "f32"],
                    help="accumulation class of the fp32 Arnoldi (bench.py's default: f32, the reference's)")
    args = ap.parse_args()
    from __graft_entry__ import _load

    mpg = _load()
    from oracle import binding

    lines = []
    only = tuple(args.only.split(",")) if args.only else None
    for case in CASES:
        if only and not case["name"].startswith(only):
            continue
        kind = case["spec"].split(":")[0]
        rlen = case.get("rlen", 30)
        cycles = min(args.cycles, case.get("cycles", args.cycles))
        t0 = time.time()
        A = mpg.gen_spec(case["spec"])
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode=case["mode"], orth=case["orth"], prec="identity", rlen=rlen, tol=0.0,
                    max_restarts=cycles + 10)
        eng = mpg.Engine(A, b, xt, accum=args.accum, **opts)
        accum = eng.spmv_layout()["accum"]
        eng.run(2)
        eng.sync()
        it0 = eng.total_iters
        t = time.perf_counter()
        eng.run(cycles)
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
        layout.update(eng.sell_columns())
        # the CGS phase kernels inside graph replays (event nodes around each
        # launch): mean over the cycle's steps and the fit t(k) = a + b k
        phases = {}
        if case["orth"] == "cgs":
            for ph, key in (("dots", "dots"), ("cgs_update", "cgs_update")):
                ms, per = eng.time_phase_graph(ph, 2)
                byk = np.asarray(per[:len(per) // rlen * rlen]).reshape(-1, rlen).mean(axis=0) * 1e3
                bfit, afit = np.polyfit(np.arange(rlen), byk, 1)
                mb = eng.phase_bytes(key)
                phases[ph] = {"mean_us": round(ms * 1e3, 2), "fit_a_us": round(float(afit), 2),
                              "fit_b_us": round(float(bfit), 4), "bytes_mean_k": int(mb),
                              "gbs": round(mb / (ms * 1e-3) / 1e9, 1), "frac_8tbs": round(mb / (ms * 1e-3) / 8e12, 3)}
        eng.close()
        cpu = None
        if args.cpu_cycles > 0:
            # the 1e8-nnz-scale matrices: one restart cycle; the oracle has no
            # fp16 mode, so mixed-half is timed as its fp32-value mixed solve
            cyc = args.cpu_cycles if kind == "laplace" and rlen <= 30 else 1
            cmode = "mixed" if case["mode"] == "mixed-half" else case["mode"]
            r = binding.solve(mpg, A, b, xt, **dict(opts, mode=cmode, max_restarts=cyc))
            cpu = {"it_s": round(r.total_iters / r.gmres_seconds, 2), "iterations": int(r.total_iters),
                   "mode": cmode, "threads": binding.lib().oracle_max_threads(), "backend": binding.backend()}
        line = {"case": case["name"], "spec": case["spec"], "rlen": rlen, "n": A.nrows, "nnz": A.nnz,
                "mode": case["mode"], "orth": case["orth"], "accum": accum, "phases_graph": phases,
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
