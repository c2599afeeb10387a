"""Per-cycle backward error of the oracle on its two backends (MKL, loop
kernels) for the large fp32-Arnoldi live-oracle cases of tests/test_m100_gpu.py
and tests/test_irregular_gpu.py, with the host's CPU model and MKL thread
count: shows how far MKL's fp32-summing sgemv moves cycle 1 between hosts
(tests/parity.py). Test infrastructure (imports the oracle).
  python tools/oracle_backends.py [--gpu]   (--gpu adds the HIP fused engine)"""
import argparse
import os
import platform
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oracle import binding  # noqa: E402
from tests.conftest import load_package  # noqa: E402


def cases(mpg):
    yield "band300k m100", mpg.gen_band(300_000, 5, 4, seed=7), dict(rlen=100, tol=0.0, max_restarts=2)
    yield "stencil27p", mpg.gen_stencil27p(105, 3, ny=105, nz=8, block=64, perm_seed=5), \
        dict(rlen=30, tol=1e-10, max_restarts=200)
    yield "fem27p", mpg.gen_spec("fem27:30:3:70:13:32:5"), dict(rlen=30, tol=1e-10, max_restarts=200)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    a = ap.parse_args()
    mpg = load_package()
    print(f"host cpu: {cpu_model()}; oracle default backend {binding.backend()}, "
          f"{binding.lib().oracle_max_threads()} threads; OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}")
    for name, A, o in cases(mpg):
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = dict(mode="mixed", orth="cgs", prec="jacobi", **o)
        runs = {be: binding.solve(mpg, A, b, xt, backend=be, **opts) for be in ("mkl", "loops")}
        if a.gpu:
            runs["gpu fused"] = mpg.solve(A, b, xt, engine="fused", **opts)
        for k, r in runs.items():
            be = np.asarray(r.cyc_r_norm) / np.asarray(r.cyc_normalization)
            print(f"{name:14s} n={A.nrows:7d} {k:9s} restarts {r.restarts:3d} cycle be "
                  + " ".join(f"{v:.4e}" for v in be[:4]) + f"  errNorm {r.err_norm:.3e}")


if __name__ == "__main__":
    main()
