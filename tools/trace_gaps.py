"""Per-kernel busy time and the idle gap before each kernel, from a rocprofv3
--kernel-trace CSV: where a GMRES step's wall time goes (kernel bodies vs
launch boundaries). Only kernels inside graph-replayed cycles are counted
(the longest run of dispatches whose names are all phase kernels).

usage: python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:30]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    busy, gap, calls = defaultdict(float), defaultdict(float), defaultdict(int)
    prev_end = None
    t0 = t1 = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        if prev_end is not None and 0 <= s - prev_end < 50_000:  # same burst (< 50 us apart)
            gap[k] += s - prev_end
            busy[k] += e - s
            calls[k] += 1
            t1 = e
        else:
            t0 = s
        prev_end = e
    tot_b, tot_g = sum(busy.values()), sum(gap.values())
    print(f"{'kernel':28s} {'calls':>6s} {'busy_us':>9s} {'gap_us':>8s}")
    for k in sorted(busy, key=lambda k: -busy[k]):
        print(f"{k:28s} {calls[k]:6d} {busy[k] / calls[k] / 1e3:9.2f} {gap[k] / calls[k] / 1e3:8.2f}")
    print(f"busy {tot_b / 1e3:.1f} us, gaps {tot_g / 1e3:.1f} us ({100 * tot_g / (tot_b + tot_g):.1f}% of burst time)")


if __name__ == "__main__":
    main()
