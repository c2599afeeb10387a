"""Accumulation class vs order on the CPU oracle: the same
GMRES solve through the oracle's MKL backend (1 thread, pinned COMPATIBLE
branch) and its loop kernels in three summation modes for fp32 operands --
"loops" (fp64 sums), "seq32" (one sequential fp32 chain), "pair32" (fp32,
long reductions in pairwise order: a GPU reduction's shape). Prints one JSON
line per (case, backend) with the per-cycle backward errors.

    python tools/accum_order.py [band|stencil27p|convdiff32 ...] > profiles/r06_accum/order.jsonl
"""
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))

from oracle import binding  # noqa: E402
from tests.conftest import load_package  # noqa: E402


def cases(mpg, which):
    if which == "band":
        return "band300k-cgs-m100", mpg.gen_band(300_000, 5, 4, seed=7), dict(
            mode="mixed", orth="cgs", prec="jacobi", rlen=100, tol=0.0, max_restarts=2)
    if which == "stencil27p":
        return "stencil27p-cgs", mpg.gen_stencil27p(105, 3, ny=105, nz=8, block=64, perm_seed=5), dict(
            mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=1e-10, max_restarts=200)
    if which == "convdiff32":
        from tests.golden.make_golden import inputs

        return "convdiff32-cgs-m100", inputs(mpg)["convdiff32"], dict(
            mode="mixed", orth="cgs", prec="jacobi", rlen=100, tol=1e-12, max_restarts=200)
    raise SystemExit(f"unknown case {which}")


def main():
    mpg = load_package()
    binding.lib()
    for which in sys.argv[1:] or ["band", "stencil27p", "convdiff32"]:
        name, A, opts = cases(mpg, which)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        for be in ("mkl", "loops", "seq32", "pair32"):
            t = time.time()
            r = binding.solve(mpg, A, b, xt, backend=be, threads=1 if be == "mkl" else 8, **opts)
            print(json.dumps({"case": name, "backend": be, "status": r.status, "restarts": int(r.restarts),
                              "backward_error": [float(v) for v in r.backward_error],
                              "seconds": round(time.time() - t, 2)}), flush=True)


if __name__ == "__main__":
    main()
