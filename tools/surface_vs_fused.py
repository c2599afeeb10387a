"""GMRES it/s of the operator-surface driver (the reference gmres.cpp control
flow over kernels_hip.cpp) against the fused engine on BAND-1M (or --spec, a
generator spec as the CLI's, e.g. fem27:111), mixed GMRES(30), --cycles
restart cycles per solve (default 20) after a 1-cycle warm-up solve;
gmres_seconds times the whole solve (set-up of the cycle program included);
"steady" is bench.py's form: the difference of a (2 + cycles)- and a
2-cycle solve, median of three pairs, so one-time set-up cancels.

usage: python tools/surface_vs_fused.py [orth ...] [--engines=surface,fused] [--cycles=N] [--pairs=N] [--spec=SPEC]"""
import sys
from pathlib import Path

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from __graft_entry__ import _load


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    engines = ["surface", "fused"]
    cycles = 20
    npairs = 3
    spec = None
    for a in sys.argv[1:]:
        if a.startswith("--spec="):
            spec = a.split("=", 1)[1]
        if a.startswith("--engines="):
            engines = a.split("=", 1)[1].split(",")
        if a.startswith("--cycles="):
            cycles = int(a.split("=", 1)[1])
        if a.startswith("--pairs="):
            npairs = int(a.split("=", 1)[1])
    orths = args or ["cgs", "mgs"]
    mpg = _load()
    A = mpg.gen_spec(spec) if spec else mpg.gen_band(1_000_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    import os
    maps = os.environ.get("MPG_DUMP_MAPS")  # crash triage: library map of this process
    for orth in orths:
        for eng in engines:
            if maps:
                Path(maps).write_text(Path("/proc/self/maps").read_text())
            opts = dict(engine=eng, mode="mixed", orth=orth, prec="identity", rlen=30, tol=0.0)
            mpg.solve(A, b, xt, max_restarts=1, **opts)
            r = mpg.solve(A, b, xt, max_restarts=cycles, **opts)
            # steady state as bench.py's surface figure: (iters, time) of a
            # (2 + cycles)-cycle solve minus a 2-cycle solve, median of --pairs (3)
            pairs, secs = [], []
            for _ in range(npairs):
                r2 = mpg.solve(A, b, xt, max_restarts=2, **opts)
                rn = mpg.solve(A, b, xt, max_restarts=2 + cycles, **opts)
                pairs.append((rn.total_iters - r2.total_iters) / (rn.gmres_seconds - r2.gmres_seconds))
                secs.append((round(r2.gmres_seconds * 1e3, 1), round(rn.gmres_seconds * 1e3, 1)))
            print(spec or "band1m", orth, eng, r.total_iters, "iters", round(r.gmres_seconds, 4), "s",
                  round(r.total_iters / r.gmres_seconds, 1), "it/s whole solve;", round(sorted(pairs)[len(pairs) // 2], 1),
                  "it/s steady (pairs", [round(v, 1) for v in pairs], ") ms per pair", secs, flush=True)


if __name__ == "__main__":
    main()
