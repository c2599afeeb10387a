"""Small-step GPU check of the ILU kernels (debug aid): factor + solve on
growing 3-D Laplacians and a band, printing times and fault words as it
goes (run it under `timeout`).

usage: python tools/ilu_debug.py [nx ...]"""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from __graft_entry__ import _load  # noqa: E402
from tests.devbuf import Hip  # noqa: E402

mpg = _load()
hip = Hip(mpg.hip_lib())
lib = hip.lib


def run(A, dt, reps=3):
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
    csr, h = C.c_void_p(), C.c_void_p()
    hip.check(lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    t = time.time()
    st = lib.mpg_ilu0_create(hip.ctx, csr, dv.p, 0 if dt == np.float64 else 1, C.byref(h))
    print(f"  create n={A.nrows} st={st} {time.time() - t:.3f}s", flush=True)
    if st == 0:
        x = hip.buf(np.ones(A.nrows, dt))
        for _ in range(reps):
            t = time.time()
            st = lib.mpg_ilu_solve(hip.ctx, h, x.p)
            hip.sync()
            print(f"  solve st={st} fault={lib.mpg_ilu_fault(h)} mode={lib.mpg_ilu_solve_mode(h)} {1e3 * (time.time() - t):.3f} ms", flush=True)
        lib.mpg_ilu_destroy(h)
    lib.mpg_csr_destroy(csr)


sizes = [int(a) for a in sys.argv[1:]] or [8, 20, 40, 60, 80, 100]
for nx in sizes:
    print(f"lap3d-{nx}", flush=True)
    run(mpg.gen_laplace3d(nx), np.float64)
print("band20000", flush=True)
run(mpg.gen_band(20000, 5, 4, seed=3), np.float64, reps=2)
print("band1M", flush=True)
run(mpg.gen_band(1000000, 5, 4, seed=7), np.float64, reps=3)
print("done", flush=True)
