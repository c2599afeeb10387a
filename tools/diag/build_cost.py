"""Set-up cost of the Arnoldi SpMV copies: wall time of creating (and
closing) a fused engine with each spmv_format on one matrix spec.
  python tools/diag/build_cost.py stencil27:111 [fem27:111 ...]"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from __graft_entry__ import _load  # noqa: E402


def main():
    mpg = _load()
    for spec in sys.argv[1:] or ["stencil27:111"]:
        A = mpg.gen_spec(spec)
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=1)
        for fmt in ("csr", "csr", "sell", "node", "auto"):
            t0 = time.perf_counter()
            eng = mpg.Engine(A, b, xt, spmv_format=fmt, **opts)
            t1 = time.perf_counter()
            lay = eng.spmv_layout()["format"]
            eng.close()
            print(f"{spec} {fmt:5s} -> {lay:5s} create {1e3 * (t1 - t0):8.1f} ms", flush=True)


if __name__ == "__main__":
    main()
