"""Launch-time probe of the small triangular solve: 200 back-to-back
mpg_trsv_f32 launches per form (MPG_TRSV_WAVE=1 one-wave LDS form, 0 the
workgroup form) at n = 30 and 64; run under rocprofv3 --kernel-trace --stats."""
import os, sys, numpy as np
sys.path.insert(0, "/root/repo")
from tests.conftest import load_package
from tests.devbuf import Hip
mpg = load_package()
h = Hip(mpg.hip_lib())
for n in (30, 64):
    ld = n + 1
    g = np.random.default_rng(n)
    M = np.zeros((ld, n), np.float32, order="F")
    M[:n] = np.triu(g.uniform(-1, 1, (n, n))) + np.diag(g.uniform(2, 3, n))
    dM = h.buf(M.ravel(order="F"))
    y = g.uniform(-1, 1, n).astype(np.float32)
    dy = h.buf(y)
    for w in ("1", "0"):
        os.environ["MPG_TRSV_WAVE"] = w
        for _ in range(200):
            h.call("mpg_trsv_f32", 1, 0, n, dM.p, ld, dy.p)
        h.sync()
print("ok")
h.close()
