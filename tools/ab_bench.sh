#!/bin/bash
# Interleaved A/B runs of bench.py on the GPU box: every variant R times, in
# rotation, so drift hits all variants alike; prints it/s per run and the
# median per variant.
# usage: tools/ab_bench.sh ROUNDS "name|ENV=.. ENV2=..|bench args" ...
# (MPG_HIP_LIB=path/to/libmpgmres_hip.so in ENV loads another kernel build)
# Each run keeps its own stderr (gpurun_out/ab_<name>_<r>.err) and the exit
# status of bench.py itself; a failed run stops the script with both named.
set -u
mkdir -p gpurun_out
R=$1; shift
declare -A vals
for ((r = 0; r < R; ++r)); do
  for spec in "$@"; do
    name="${spec%%|*}"; rest="${spec#*|}"; envs="${rest%%|*}"; args="${rest#*|}"
    err="gpurun_out/ab_${name}_${r}.err"
    out=$(env $envs timeout -k 10 120 python bench.py --no-cpu-baseline $args 2>"$err")
    rc=$?
    line=$(printf '%s\n' "$out" | grep '^{' | tail -1)
    v=$(printf '%s' "$line" | python -c "import json,sys;print(json.loads(sys.stdin.read())['value'])" 2>/dev/null)
    if [ $rc -ne 0 ] || [ -z "$v" ]; then
      echo "[$name] run $r failed: bench.py exit $rc (124/137: time limit), stderr in $err:"
      tail -5 "$err"
      exit 3
    fi
    echo "[$name] run $r: $v it/s"
    vals[$name]="${vals[$name]:-} $v"
  done
done
for spec in "$@"; do
  name="${spec%%|*}"
  echo "[$name] median $(python -c "import statistics,sys;print(statistics.median(map(float,sys.argv[1:])))" ${vals[$name]})  all:${vals[$name]}"
done
