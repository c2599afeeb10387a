"""Per-launch HBM traffic and L2 hit rate of the Arnoldi SpMV kernels from
rocprofv3 --pmc passes run as separate processes (FETCH_SIZE, WRITE_SIZE,
TCC_HIT_sum + TCC_MISS_sum; tools/battery.sh irrpmc / lappmc / ranks):
FETCH_SIZE x 2 (MI355X_MICROARCH.md §HBM; calibrated at 0.500 of the bytes
for every access width the SpMVs use, tools/pmc_calib.hip) + WRITE_SIZE, in
KB per launch, averaged over the launches of each SpMV kernel (grid size
kept apart, so rank blocks of different sizes stay separate).

usage: python tools/spmv_pmc_table.py CASE=DIR [CASE=DIR ...]
  DIR holds fetch/, write/ and optionally hit/ subdirectories (or
  DIR_fetch, DIR_write, DIR_hit siblings), each with a *counter_collection.csv
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SPMV = re.compile(r"(k_step_node|k_step_sell2?|k_step_spmv|k_node_spmv|k_sell_spmv2?|k_csr_adaptive)")


def collect(d):
    """{(kernel, grid): {counter: [values per dispatch]}}"""
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)  # (dispatch, kernel, grid, counter) -> sum over dimensions
        for r in csv.DictReader(open(f)):
            m = SPMV.search(r["Kernel_Name"])
            if not m:
                continue
            per[(r["Dispatch_Id"], m.group(1), int(r["Grid_Size"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, k, g, c), v in per.items():
            out[(k, g)][c].append(v)
    return out


def subdirs(d):
    for part in ("fetch", "write", "hit"):
        for cand in (os.path.join(d, part), f"{d}_{part}"):
            if os.path.isdir(cand):
                yield part, cand
                break


def main():
    rows = []
    for arg in sys.argv[1:]:
        case, d = arg.split("=", 1)
        merged = defaultdict(dict)
        for part, sd in subdirs(d):
            for key, cs in collect(sd).items():
                for c, vals in cs.items():
                    merged[key][c] = sum(vals) / len(vals)
                merged[key]["launches_" + part] = max(len(v) for v in cs.values())
        for (k, g), cs in sorted(merged.items()):
            fetch = cs.get("FETCH_SIZE")
            write = cs.get("WRITE_SIZE")
            hit, miss = cs.get("TCC_HIT_sum"), cs.get("TCC_MISS_sum")
            row = {"case": case, "kernel": k, "grid": g,
                   "fetch_mb_x2": round(2 * fetch / 1e3, 2) if fetch is not None else None,
                   "write_mb": round(write / 1e3, 2) if write is not None else None,
                   "hbm_mb": round((2 * fetch + write) / 1e3, 2) if fetch is not None and write is not None else None,
                   "l2_hit": round(hit / (hit + miss), 3) if hit is not None and miss else None,
                   "launches": {p: cs.get("launches_" + p) for p in ("fetch", "write", "hit")}}
            rows.append(row)
            print(json.dumps(row))


if __name__ == "__main__":
    main()
