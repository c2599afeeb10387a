#!/bin/bash
# Run GPU steps one after another on the gpurun box; stop at the first step
# that ends in anything other than pass (0) / test failures (1).
# usage: tools/gpu_steps.sh "name|timeout_s|command" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; to="${rest%%|*}"; cmd="${rest#*|}"
  start=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - start ))s"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$name] stopping the chain"; exit $rc; fi
done
