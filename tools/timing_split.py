#!/usr/bin/env python3
"""Split the Arnoldi SpMV launches of a rocprofv3 kernel trace of
tools/timing_probe.py into its three blocks (graph replays without timing,
eager event-timed cycles, graph replays with event nodes) and print the
rocprof mean / median duration of each, beside the probe's own clocks.
usage: python tools/timing_split.py TRACE.csv PROBE.json"""
import csv
import json
import re
import statistics as st
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    probe = json.loads([ln for ln in open(sys.argv[2]) if ln.startswith("{")][-1])
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sp = [r for r in rows if re.search(r"k_step_(sell2?|spmv)\b", r["Kernel_Name"])]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sp]
    out = {"spmv_launches_in_trace": len(d)}
    i = 0
    for name in ("warm_graph", "eager_events", "graph_events"):
        c = probe["blocks"][name]
        seg = d[i:i + c]
        i += c
        out[name] = {"launches": len(seg), "rocprof_mean_us": round(st.mean(seg), 3) if seg else None,
                     "rocprof_median_us": round(st.median(seg), 3) if seg else None}
    out["eager_event_us"] = probe["eager_event_us"]
    out["graph_event_us"] = probe["graph_event_us"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
