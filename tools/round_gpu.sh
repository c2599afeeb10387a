#!/bin/bash
# The standard GPU battery of a round on the gpurun box: GPU tests, smoke,
# the bench line, its rocprofv3 kernel trace + stats, the two PMC passes
# (FETCH_SIZE and WRITE_SIZE apart, MI355X_MICROARCH.md §HBM) and the N = 2
# shared-GPU rehearsal. Every step has its own time limit (tools/gpu_steps.sh
# stops the chain at anything other than pass / test failures).
# usage: tools/round_gpu.sh TAG [steps...]   (default: all)
set -u
tag=${1:-r03}
shift || true
steps=${*:-"tests smoke bench prof pmc n2"}
cmds=()
for s in $steps; do
  case $s in
    tests) cmds+=("tests|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider") ;;
    smoke) cmds+=("smoke|240|python -u -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) cmds+=("bench|400|python -u bench.py > gpurun_out/${tag}_bench.json") ;;
    prof) cmds+=("prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 10 --no-cpu-baseline --hbm-rows 0") ;;
    pmc) cmds+=("pmcf|150|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hbm-rows 0")
         cmds+=("pmcw|150|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hbm-rows 0") ;;
    n2) cmds+=("n2|400|MPG_BENCH_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/${tag}_bench_n2.json") ;;
    configs) cmds+=("configs|600|python -u tools/bench_configs.py --out gpurun_out/${tag}_configs.jsonl") ;;
  esac
done
exec tools/gpu_steps.sh "${cmds[@]}"
