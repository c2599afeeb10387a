"""Small-step GPU check of the ILU kernels (debug aid): factor + solve on
tiny matrices, printing as it goes."""
import ctypes as C
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from __graft_entry__ import _load  # noqa: E402
from tests.devbuf import Hip  # noqa: E402

mpg = _load()
hip = Hip(mpg.hip_lib())
lib = hip.lib
lib.mpg_ilu_values_dev.restype = C.c_void_p


def run(A, dt):
    drp, dci, dv = hip.buf(A.rowptr), hip.buf(A.col), hip.buf(A.val)
    csr, h = C.c_void_p(), C.c_void_p()
    hip.check(lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
    t = time.time()
    st = lib.mpg_ilu0_create(hip.ctx, csr, dv.p, 0 if dt == np.float64 else 1, C.byref(h))
    print(f"  create n={A.nrows} st={st} {time.time() - t:.3f}s", flush=True)
    if st == 0:
        x = hip.buf(np.ones(A.nrows, dt))
        t = time.time()
        st = lib.mpg_ilu_solve(hip.ctx, h, x.p)
        hip.sync()
        print(f"  solve st={st} fault={lib.mpg_ilu_fault(h)} {time.time() - t:.3f}s x[:4]={x.get()[:4]}", flush=True)
        lib.mpg_ilu_destroy(h)
    lib.mpg_csr_destroy(csr)


n = 8
rp = np.arange(0, 3 * n - 1, 3, dtype=np.int32)
for i, nm in enumerate(["tridiag8"]):
    rows = []
    for r in range(n):
        rows.append([c for c in (r - 1, r, r + 1) if 0 <= c < n])
    rp = np.cumsum([0] + [len(r) for r in rows]).astype(np.int32)
    ci = np.array([c for r in rows for c in r], np.int32)
    va = np.array([4.0 if c == r else -1.0 for r, row in enumerate(rows) for c in row])
    A = mpg.Csr(n, n, rp, ci, va)
    print(nm, flush=True)
    run(A, np.float64)
print("band100", flush=True)
run(mpg.gen_band(100, 5, 4, seed=3), np.float64)
print("lap3d-8", flush=True)
run(mpg.gen_laplace3d(8), np.float64)
print("done", flush=True)
