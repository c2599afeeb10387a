"""Diagnostic: where mpg_csr_half_values and mpg_copy_f64f16 differ."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))
from tests.conftest import load_package  # noqa: E402
from tests.devbuf import Hip  # noqa: E402

mpg = load_package()
hip = Hip(mpg.hip_lib())
A = mpg.gen_band(100_000, 5, 4, seed=7)
drp, dci = hip.buf(A.rowptr), hip.buf(A.col)
csr = C.c_void_p()
hip.check(hip.lib.mpg_csr_create(hip.ctx, A.nrows, A.nrows, A.nnz, A.rowptr.ctypes.data, drp.p, dci.p, C.byref(csr)))
dv = hip.buf(A.val)
dh, de = hip.buf(A.nnz, np.uint16), hip.buf(A.nrows + 64, np.int8)
stats = (C.c_int64 * 4)()
print("st", hip.lib.mpg_csr_half_values(hip.ctx, csr, dv.p, 1, dh.p, de.p, stats), list(stats))
plain = hip.buf(A.nnz, np.uint16)
hip.call("mpg_copy_f64f16", A.nnz, dv.p, plain.p)
a, b = dh.get(), plain.get()
npy = A.val.astype(np.float32).astype(np.float16).view(np.uint16)
d = np.flatnonzero(a != b)
print("differ", len(d), "of", A.nnz, "mine!=numpy", int((a != npy).sum()), "plain!=numpy", int((b != npy).sum()))
for i in d[:12]:
    print(i, repr(A.val[i]), hex(a[i]), hex(b[i]), hex(npy[i]), np.float16(A.val[i]))
