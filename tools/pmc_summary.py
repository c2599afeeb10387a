"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE and
WRITE_SIZE cannot share a pass on gfx950), with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of a coalesced
streaming read, so the read side is calibrated on tools/stream_bench's
k_calib kernels (known byte counts at 4/8/16 B per lane) when that run is
given, else doubled. Writes profiles/pmc_traffic.json, which bench.py reads
for roofline.traffic.

usage: python tools/pmc_summary.py FETCH_DIR WRITE_DIR OUT.json [CALIB_DIR]
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            m = re.search(r"(k_\w+)(<[^(]*>)?", r["Kernel_Name"])
            name = m.group(1) if m else r["Kernel_Name"][:40]
            # the Arnoldi SpMVs come in a plain and a Givens-folded
            # instantiation: keep them apart (FOLD is template argument 7 of
            # k_step_sell<T, P, VI, CI, W, WIN, FOLD, DN> and 4 of
            # k_step_spmv<T, P, VI, FOLD>)
            if m and name in ("k_step_sell", "k_step_sell2", "k_step_spmv") and m.group(2):
                # (k_step_sell2<T, P, VI, W, WIN, FOLD, BE, BS>: FOLD is argument 6)
                args = [a.strip() for a in m.group(2)[1:-1].split(",")]
                at = {"k_step_sell": 6, "k_step_sell2": 5, "k_step_spmv": 3}[name]
                if len(args) > at and args[at] == "true":
                    name += ":fold"
            vals[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    factor, how = 2.0, "x2 (MI355X_MICROARCH.md §HBM)"
    if len(sys.argv) > 4:
        cal = per_kernel(sys.argv[4], "FETCH_SIZE")
        known = 512 * 1024 * 1024
        facs = {k: known / (v * 1024) for k, v in cal.items() if k.startswith("k_calib") and v > 0}
        if facs:
            factor = sum(facs.values()) / len(facs)
            how = "calibrated on k_calib (512 MiB reads): " + ", ".join(f"{k} x{v:.3f}" for k, v in facs.items())
    out = {"_fetch_correction": how}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        out[k] = {"fetch_kb": round(f, 1), "write_kb": round(w, 1),
                  "hbm_bytes_per_launch": int(factor * f * 1024 + w * 1024)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
