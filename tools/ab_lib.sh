#!/bin/bash
# Interleaved A/B of two kernel builds on the GPU box: the in-tree
# libmpgmres_hip.so ("new") against another build loaded through MPG_HIP_LIB
# ("old"), R rounds of tools/spmv_ab.py per case (in-cycle SpMV events) and
# then tools/ab_bench.sh on the bench line.
# usage: tools/ab_lib.sh OLD_LIB OUT_PREFIX R case [case ...]
set -u
old=$1; out=$2; R=$3; shift 3
cases=()
for c in "$@"; do cases+=(--case "$c"); done
mkdir -p gpurun_out
for ((r = 0; r < R; ++r)); do
  timeout -k 10 200 python -u tools/spmv_ab.py "${cases[@]}" --var MPG_AB=new --reps 3 >> "${out}_spmv.jsonl" || exit 3
  MPG_HIP_LIB=$old timeout -k 10 200 python -u tools/spmv_ab.py "${cases[@]}" --var MPG_AB=old --reps 3 >> "${out}_spmv.jsonl" || exit 3
done
tools/ab_bench.sh 5 "new||--steps 20" "old|MPG_HIP_LIB=$old|--steps 20" > "${out}_bench.txt"
python - "${out}_spmv.jsonl" <<'PY'
import json, statistics, sys
from collections import defaultdict
v = defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    v[(d["case"], d["variant"]["MPG_AB"])] += d["us"]
for k in sorted(v):
    print(k[0], k[1], "median us", statistics.median(v[k]))
PY
tail -2 "${out}_bench.txt"
