"""Per-step kernel durations inside graph-replayed restart cycles, from a
rocprofv3 --kernel-trace CSV: for every phase kernel, the mean duration at
each Arnoldi step k (its occurrence index within a cycle), and a least-squares
fit t(k) = a + b*k, which separates a launch's fixed cost (a) from the cost of
each added basis column (b).

A cycle starts at k_prologue / k_prologue_sell (or k_update_x closes one); k counts the
occurrences of each kernel name since the cycle started.

usage: python tools/per_step.py gpurun_out/prof/.../kernel_trace.csv [col_bytes]
  col_bytes: bytes of one basis column (n * s_T), to print the marginal GB/s.
"""
import csv
import re
import sys
from collections import Counter, defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    return m.group(1) if m else name[:30]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    col_bytes = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cycles, cur = [], None
    for r in rows:
        k = short(r["Kernel_Name"])
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if k in ("k_prologue", "k_prologue_sell"):
            cur = []
            continue
        if cur is None:
            continue
        cur.append((k, d))
        if k.startswith("k_update_x"):
            cycles.append(cur)
            cur = None
    # keep the cycles of the most common shape (drops eagerly timed cycles
    # whose extra replays would shift k)
    shape = lambda c: tuple(sorted(Counter(k for k, _ in c).items()))
    common = Counter(shape(c) for c in cycles).most_common(1)
    per = defaultdict(lambda: defaultdict(list))  # kernel -> k -> [us]
    for c in cycles:
        if not common or shape(c) != common[0][0]:
            continue
        count = defaultdict(int)
        for k, d in c:
            per[k][count[k]].append(d)
            count[k] += 1
    print(f"{len(cycles)} cycles, {common[0][1] if common else 0} of the common shape")
    for k, byk in sorted(per.items()):
        ks = sorted(byk)
        means = [sum(byk[i]) / len(byk[i]) for i in ks]
        line = " ".join(f"{m:5.1f}" for m in means)
        n = len(ks)
        fit = ""
        if n >= 3:
            mx = sum(ks) / n
            my = sum(means) / n
            sxx = sum((x - mx) ** 2 for x in ks)
            b = sum((x - mx) * (y - my) for x, y in zip(ks, means)) / sxx if sxx else 0.0
            a = my - b * mx
            fit = f"  fit a={a:.2f} us b={b:.3f} us/k"
            if col_bytes and b > 0:
                fit += f" ({col_bytes / (b * 1e3):.0f} GB/s per added column)"
        print(f"{k:22s} n={n:3d} mean={sum(means) / n:6.2f}{fit}\n    {line}")


if __name__ == "__main__":
    main()
