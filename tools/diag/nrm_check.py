import sys, ctypes as C
sys.path.insert(0, '/root/repo')
import numpy as np
from tests.conftest import load_package
from tests.devbuf import Hip
mpg = load_package()
hip = Hip(mpg.hip_lib())
for n in (20000, 20001, 4096, 100000, 1000000):
    w = np.random.default_rng(23).uniform(-1, 1, n).astype(np.float32)
    dw = hip.buf(w); h = hip.buf(1, np.float32)
    hip.call("mpg_nrm2_f32", C.c_int64(n), dw.p, h.p)
    np_ = C.c_int32(); hip.call("mpg_nrm2_partials_f32", C.c_int64(n), dw.p, C.byref(np_))
    h2 = hip.buf(1, np.float32); o = hip.buf(n, np.float32)
    hip.call("mpg_scal_recip_nrm2_f32", np_, h2.p, C.c_int64(n), dw.p, o.p)
    print(n, np_.value, h.get()[0], h2.get()[0], np.sqrt(np.sum(w.astype(np.float64)**2)), np.array_equal(dw.get(), w))
