"""Print the top kernels of a rocprofv3 --stats kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{r['Name'][:64]:64s} calls={r['Calls']:>6} avg_us={float(r['AverageNs'])/1e3:9.2f} "
          f"pct={100*float(r['TotalDurationNs'])/tot:5.1f}")
