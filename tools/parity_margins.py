"""Measure how far the GPU solves sit from the golden records on the
quantities tests/parity.py checks beyond cycle 0 (every cycle's backward
error, x_head / x_sum, res_norm / err_norm), so the stated tolerances are
set from data with margin. One JSON line per (record, engine).

usage: python tools/parity_margins.py [engine ...]   (default: fused surface)"""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from tests.conftest import load_package  # noqa: E402
from tests.golden.make_golden import inputs  # noqa: E402


def main():
    engines = sys.argv[1:] or ["fused", "surface"]
    mpg = load_package()
    gold = json.loads((REPO / "tests/golden/gmres_golden.json").read_text())
    mats = inputs(mpg)
    for rec in gold["cases"]:
        case = dict(rec["case"])
        A = mats[case.pop("matrix")]
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        for eng in engines:
            g = mpg.solve(A, b, xt, engine=eng, **case)
            be_r = np.array(rec["cyc_r_norm"]) / np.array(rec["cyc_normalization"])
            be_g = g.backward_error
            c = min(len(be_r), len(be_g))
            lg = np.abs(np.log10(be_g[:c]) - np.log10(be_r[:c]))
            rel = np.abs(be_g[:c] - be_r[:c]) / be_r[:c]
            xh = np.array(rec["x_head"])
            print(json.dumps(dict(
                id=f"{rec['case']['matrix']}-{case['mode']}-{case['orth']}-{case['prec']}-m{case['rlen']}",
                engine=eng, status=(g.status, rec["status"]), restarts=(int(g.restarts), rec["restarts"]),
                iters=(int(g.total_iters), rec["total_iters"]),
                be_rel=[float(v) for v in rel], be_log=float(lg.max()),
                be_final=(float(be_g[-1]), float(be_r[-1])),
                xhead_rel=float(np.max(np.abs(g.x[:16] - xh)) / np.max(np.abs(xh))),
                xsum_rel=float(abs(g.x.sum() - rec["x_sum"]) / abs(rec["x_sum"])),
                res=(g.res_norm, rec["res_norm"]), err=(g.err_norm, rec["err_norm"]))), flush=True)


if __name__ == "__main__":
    main()
