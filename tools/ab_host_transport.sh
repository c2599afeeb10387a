#!/bin/bash
# the ranks' CGS step all-reduces (k+1) x Gd partials per
# step when the update sums them itself (MPG_CGS_PARTIALS, default on) and
# k+1 sums otherwise. Interleaved A/B of the two on the shared-GPU N = 2
# rehearsal (two ranks on one GPU, collectives over gloo host memory).
#   tools/ab_host_transport.sh ROUNDS
set -u
R=${1:-3}
for ((r = 0; r < R; ++r)); do
  for v in 1 0; do
    out=$(MPG_CGS_PARTIALS=$v MPG_BENCH_SHARED_GPU=1 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + r * 2 + v)) bench.py --gpus 2 --steps 5 \
      --warmup 1 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0 2>/dev/null | grep '^{' | tail -1)
    [ -n "$out" ] || { echo "[partials=$v] run $r failed"; exit 3; }
    echo "[partials=$v] run $r: $(printf '%s' "$out" | python -c "import json,sys;print(json.loads(sys.stdin.read())['value'])") it/s"
  done
done
