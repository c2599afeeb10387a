"""Kernel statistics from a rocprofv3 results database (rocpd SQLite, the
default output format of this ROCm's rocprofv3) or a `--output-format csv`
kernel_trace.csv, in the layout of
`rocprofv3 --stats` kernel_stats.csv, plus a per-(kernel, grid) split that
separates the same kernel run on two problem sizes in one process (bench.py
times BAND-10M and the BAND-100M HBM-scale figure).

usage: python tools/rocpd_summary.py RESULTS.db|KERNEL_TRACE.csv OUT_PREFIX
  writes OUT_PREFIX_kernel_stats.csv and OUT_PREFIX_kernel_grid.csv
"""
import csv
import re
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    prefix = sys.argv[2]
    if sys.argv[1].endswith(".csv"):
        with open(sys.argv[1], newline="") as f:
            rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]),
                     int(r["Workgroup_Size_X"])) for r in csv.DictReader(f)]
        rows.sort(key=lambda r: r[1])
    else:
        db = sqlite3.connect(sys.argv[1])
        rows = db.execute("select name, start, end, grid_x, workgroup_x from kernels order by start").fetchall()
    by_name = defaultdict(list)
    by_grid = defaultdict(list)
    for name, s, e, g, w in rows:
        d = e - s
        by_name[name].append(d)
        by_grid[(short(name), name, g, w)].append(d)
    total = sum(sum(v) for v in by_name.values())
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, v in sorted(by_name.items(), key=lambda kv: -sum(kv[1])):
            wr.writerow([name, len(v), sum(v), round(sum(v) / len(v), 1), round(100 * sum(v) / total, 3), min(v), max(v)])
    with open(prefix + "_kernel_grid.csv", "w", newline="") as f:
        wr = csv.writer(f)
        wr.writerow(["Kernel", "GridX", "WorkgroupX", "Calls", "AverageNs", "MinNs", "MaxNs", "Name"])
        for (k, name, g, w), v in sorted(by_grid.items(), key=lambda kv: -sum(kv[1])):
            wr.writerow([k, g, w, len(v), round(sum(v) / len(v), 1), min(v), max(v), name])
    for (k, name, g, w), v in sorted(by_grid.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"{k:22s} grid={g:>9} wg={w:>5} calls={len(v):>5} avg_us={sum(v) / len(v) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
