"""One restart cycle's kernel timeline from a rocprofv3 --kernel-trace CSV:
every dispatch between two consecutive launches of the cycle's marker kernel
(`--marker=NAME`, by default the kernel with the largest gap before it), with its duration and
the idle gap before it. Shows where a cycle's wall time goes outside the
kernel bodies (host round trips of the operator surface's restart section).

usage: python tools/cycle_timeline.py trace.csv [--cycle=N] [--min-gap-us=X]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    path = sys.argv[1]
    opt = dict(a[2:].split("=", 1) for a in sys.argv[2:] if a.startswith("--"))
    which = int(opt.get("cycle", "5"))
    min_gap = float(opt.get("min-gap-us", "0"))
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows]
    # the cycle's boundary: the kernel name whose launches carry the largest total gap
    gaps = defaultdict(list)
    for (s0, e0, _), (s1, e1, k1) in zip(ev, ev[1:]):
        gaps[k1].append(s1 - e0)
    marker = opt.get("marker") or max(gaps, key=lambda k: max(gaps[k]))
    idx = [i for i, e in enumerate(ev) if e[2] == marker]
    if len(idx) < which + 2:
        which = max(0, len(idx) - 2)
    a, b = idx[which], idx[which + 1]
    print(f"marker {marker}: {len(idx)} launches; cycle {which}: dispatches {a}..{b - 1}")
    t0 = ev[a][0]
    busy = gap = 0
    for i in range(a, b):
        s, e, k = ev[i]
        g = s - ev[i - 1][1] if i else 0
        busy += e - s
        gap += g
        if g / 1e3 >= min_gap or i == a:
            print(f"{(s - t0) / 1e3:9.1f} us  gap {g / 1e3:7.1f}  dur {(e - s) / 1e3:7.1f}  {k}")
    tot = ev[b][0] - t0
    print(f"cycle wall {tot / 1e3:.1f} us: kernels {busy / 1e3:.1f} us, gaps {gap / 1e3:.1f} us")


if __name__ == "__main__":
    main()
