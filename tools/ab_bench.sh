#!/bin/bash
# Interleaved A/B runs of bench.py on the GPU box: every variant R times, in
# rotation, so drift hits all variants alike; prints it/s per run and the
# median per variant.
# usage: tools/ab_bench.sh ROUNDS "name|ENV=.. ENV2=..|bench args" ...
# (MPG_HIP_LIB=path/to/libmpgmres_hip.so in ENV loads another kernel build)
set -u
mkdir -p gpurun_out
R=$1; shift
declare -A vals
for ((r = 0; r < R; ++r)); do
  for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
    out=$(env $envs timeout -k 10 120 python bench.py --no-cpu-baseline $args 2>/dev/null | tail -1)
    rc=$?
    v=$(echo "$out" | python -c "import json,sys;print(json.loads(sys.stdin.read())['value'])" 2>/dev/null)
    if [ -z "$v" ]; then echo "[$name] run $r failed (rc=$rc)"; exit 3; fi
    echo "[$name] run $r: $v it/s"
    vals[$name]="${vals[$name]:-} $v"
  done
done
for spec in "$@"; do
  name="${spec%%|*}"
  echo "[$name] median $(python -c "import statistics,sys;print(statistics.median(map(float,sys.argv[1:])))" ${vals[$name]})  all:${vals[$name]}"
done
