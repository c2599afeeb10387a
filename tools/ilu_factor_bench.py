"""ILU(0) set-up time on one MI355X: mpg_ilu0_create (diagonal search, host
level schedules, the sync-free factorisation, rounding) and one L + U solve,
median of 3 creates, on LAP-1M and banded matrices (depth n).

usage: python tools/ilu_factor_bench.py"""
import ctypes as C
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from __graft_entry__ import _load  # noqa: E402
from tests.devbuf import Hip  # noqa: E402

mpg = _load()
hip = Hip(mpg.hip_lib())
lib = hip.lib


def bench(A, dt, reps=3):
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
    csr = C.c_void_p()
    hip.check(lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    create, solve = [], []
    x = hip.buf(np.ones(A.nrows, dt))
    for _ in range(reps):
        h = C.c_void_p()
        hip.sync()
        t = time.perf_counter()
        hip.check(lib.mpg_ilu0_create(hip.ctx, csr, dv.p, 0 if dt == np.float64 else 1, C.byref(h)), "ilu0_create")
        hip.sync()
        create.append(time.perf_counter() - t)
        t = time.perf_counter()
        hip.check(lib.mpg_ilu_solve(hip.ctx, h, x.p))
        hip.sync()
        solve.append(time.perf_counter() - t)
        assert lib.mpg_ilu_fault(h) == 0
        lib.mpg_ilu_destroy(h)
    lib.mpg_csr_destroy(csr)
    return float(np.median(create)), float(np.median(solve))


def main():
    mats = {"LAP-1M": lambda: mpg.gen_laplace3d(100), "BAND-100k": lambda: mpg.gen_band(100_000, 5, 4, seed=7),
            "band-9000-w60": lambda: mpg.gen_band(9000, 31, 29, seed=5)}
    for name, gen in mats.items():
        A = gen()
        for dt in (np.float64, np.float32):
            c, s = bench(A, dt)
            print(json.dumps({"matrix": name, "dtype": np.dtype(dt).name, "create_ms": round(1e3 * c, 2),
                              "solve_ms": round(1e3 * s, 3)}), flush=True)


if __name__ == "__main__":
    main()
