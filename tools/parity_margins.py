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
                # the x differences against the reference's own errNorm
                # (tests/parity.py bounds them by e_ref alone)
                xhead_eref=float(np.max(np.abs(g.x[:16] - xh)) / rec["err_norm"]) if rec["err_norm"] else None,
                xsum_eref=float(abs(g.x.sum() - rec["x_sum"]) / (np.sqrt(len(g.x)) * rec["err_norm"]))
                if rec["err_norm"] else None,
                res=(g.res_norm, rec["res_norm"]), err=(g.err_norm, rec["err_norm"]))), flush=True)




def summary(path):
    """Per-mode maxima of a parity_margins.jsonl (profiles/r02_parity_margins.txt)."""
    gold = {}
    for rec in json.loads((REPO / "tests/golden/gmres_golden.json").read_text())["cases"]:
        c = rec["case"]
        gold[f"{c['matrix']}-{c['mode']}-{c['orth']}-{c['prec']}-m{c['rlen']}"] = rec
    per = {}
    for line in open(path):
        r = json.loads(line)
        rec = gold[r["id"]]
        mode = rec["case"]["mode"]
        be = np.array(rec["cyc_r_norm"]) / np.array(rec["cyc_normalization"])
        rel = np.array(r["be_rel"])
        floor = 1e-6 if mode == "single" else 1e-14
        above = be[:len(rel)] > floor
        d = per.setdefault(mode, dict(runs=0, same_restarts=0, same_status=0, be_rel_above_floor=0.0,
                                      xhead_rel=0.0, xsum_rel=0.0, xhead_eref=0.0, xsum_eref=0.0,
                                      res_factor=1.0, err_factor=1.0))
        d["runs"] += 1
        d["same_restarts"] += r["restarts"][0] == r["restarts"][1]
        d["same_status"] += r["status"][0] == r["status"][1]
        if above.any():
            d["be_rel_above_floor"] = max(d["be_rel_above_floor"], float(rel[above].max()))
        d["xhead_rel"] = max(d["xhead_rel"], r["xhead_rel"])
        d["xsum_rel"] = max(d["xsum_rel"], r["xsum_rel"])
        if r.get("xhead_eref") is not None and r["restarts"][0] == r["restarts"][1]:
            d["xhead_eref"] = max(d["xhead_eref"], r["xhead_eref"])
            d["xsum_eref"] = max(d["xsum_eref"], r["xsum_eref"])
        for k, key in (("res", "res_factor"), ("err", "err_factor")):
            a, b = r[k]
            if a > 0 and b > 0:
                d[key] = max(d[key], a / b, b / a)
    for mode, d in per.items():
        print(mode, json.dumps({k: (float(f"{v:.3g}") if isinstance(v, float) else v) for k, v in d.items()}))


if __name__ == "__main__":
    if len(sys.argv) == 3 and sys.argv[1] == "--summary":
        summary(sys.argv[2])
    else:
        main()
