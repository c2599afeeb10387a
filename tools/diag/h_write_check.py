"""Diagnostic: where mpg_scal_recip_nrm2_* / mpg_sell_spmv_norm_* store h."""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, "/root/repo")
from tests.conftest import load_package  # noqa: E402
from tests.devbuf import Hip  # noqa: E402

mpg = load_package()
hip = Hip(mpg.hip_lib())
n = 20000
w = np.random.default_rng(23).uniform(-1, 1, n).astype(np.float32)
dw = hip.buf(w)
np_ = C.c_int32()
hip.call("mpg_nrm2_partials_f32", C.c_int64(n), dw.p, C.byref(np_))
h_sep = hip.buf(np.zeros(1, np.float32))
col = hip.buf(np.arange(10, dtype=np.float32))
o = hip.buf(n, np.float32)
hip.call("mpg_scal_recip_nrm2_f32", np_, h_sep.p, C.c_int64(n), dw.p, o.p)
print("separate h:", h_sep.get(), "nparts", np_.value)
hip.call("mpg_nrm2_partials_f32", C.c_int64(n), dw.p, C.byref(np_))
print("col.dtype", col.dtype, "at(8)-p", col.at(8).value - col.p.value)
hip.call("mpg_scal_recip_nrm2_f32", np_, col.at(8), C.c_int64(n), dw.p, o.p)
print("col after:", col.get())
