"""Which set-up makes mpg_engine_time_phase_graph fail: torch initialised
first, the engine having run cycles, eager timing first. Measurement aid."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    variant = sys.argv[1]
    if "torch" in variant:
        import torch

        torch.cuda.synchronize()
    from __graft_entry__ import _load

    mpg = _load()
    A = mpg.gen_band(1_000_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=40)
    if "dev" in variant:
        opts["device"] = 0
    eng = mpg.Engine(A, b, xt, **opts)
    if "run" in variant:
        eng.run(5)
        eng.sync()
    if "eager" in variant:
        eng.time_spmv_incycle(2)
    try:
        ms, per = eng.time_phase_graph("spmv", 3)
        print(variant, "ok", round(ms * 1e3, 3), "us")
    except RuntimeError as ex:
        print(variant, "FAIL", ex)
    eng.close()


if __name__ == "__main__":
    main()
