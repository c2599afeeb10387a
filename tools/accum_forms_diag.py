"""Diagnostic: the fp32-accumulation class across the Arnoldi SpMV's storage
forms (CSR row blocks, SELL-64, node blocks): the first step at which each
form's |s(k+1)| history leaves CSR's, per accumulation class and Givens-fold
setting. Prints one JSON line per run."""
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from tests.conftest import load_package  # noqa: E402

mpg = load_package()
for which in ("stencil27p", "fem27", "band"):
    if which == "stencil27p":
        A = mpg.gen_stencil27p(40, 3, ny=40, nz=8, block=64, perm_seed=5)
    elif which == "fem27":
        A = mpg.gen_fem27(24, 3, keep_pct=70, seed=13)
    else:
        A = mpg.gen_band(60_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    for fold in ("", "0", "1"):
        if fold:
            os.environ["MPG_FOLD_GIVENS"] = fold
        else:
            os.environ.pop("MPG_FOLD_GIVENS", None)
        for accum in ("f64", "f32"):
            fmts = ("csr", "sell") + (("node",) if which != "band" else ())
            got = {f: mpg.solve(A, b, xt, engine="fused", spmv_format=f, accum=accum, **opts) for f in fmts}
            ref = got["csr"].step_res
            first = {f: int(np.argmax(got[f].step_res != ref)) if np.any(got[f].step_res != ref) else -1
                     for f in fmts[1:]}
            print(json.dumps({"matrix": which, "fold": fold or "auto", "accum": accum, "first_diff_step": first}),
                  flush=True)
