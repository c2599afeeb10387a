#!/bin/bash
# Round-4 performance battery on the gpurun box (one step per measurement,
# each under its own time limit; tools/gpu_steps.sh stops the chain at any
# failure other than pass / test failures).
#   tools/r04_perf.sh TAG [steps...]
# steps: probe bench b100 prof prof100 pmcf pmcw configs ab_pf ab_k0 c4pmc irr
set -u
tag=${1:-r04}
shift || true
steps=${*:-"probe bench b100 prof prof100 pmcf pmcw"}
cmds=()
for s in $steps; do
  case $s in
    probe) cmds+=("${tag}_probe|240|python3 tools/timing_probe.py > gpurun_out/${tag}_probe.json && python3 tools/timing_probe.py --rlen 100 > gpurun_out/${tag}_probe100.json") ;;
    bench) cmds+=("${tag}_bench|420|python -u bench.py > gpurun_out/${tag}_bench.json") ;;
    b100) cmds+=("${tag}_b100|240|python -u bench.py --rlen 100 --steps 5 --warmup 1 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0 > gpurun_out/${tag}_b100.json") ;;
    prof) cmds+=("${tag}_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 10 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0") ;;
    prof100) cmds+=("${tag}_prof100|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof100 -o bench -- python3 bench.py --rlen 100 --steps 5 --warmup 1 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0") ;;
    pmcf) cmds+=("${tag}_pmcf|150|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0") ;;
    pmcw) cmds+=("${tag}_pmcw|150|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o write -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0") ;;
    configs) cmds+=("${tag}_configs|900|python -u tools/bench_configs.py --cycles 6 --cpu-cycles 1 --out gpurun_out/${tag}_configs.jsonl") ;;
    ab_pf) cmds+=("${tag}_ab_pf|420|tools/ab_bench.sh 4 'pf0|MPG_CGS_PREFETCH=0|--hbm-rows 0 --surface-cycles 0' 'pf1|MPG_CGS_PREFETCH=1|--hbm-rows 0 --surface-cycles 0' > gpurun_out/${tag}_ab_pf.txt") ;;
    ab_k0) cmds+=("${tag}_ab_k0|600|tools/ab_bench.sh 3 'k0|MPG_FUSE_DOTS=0|--hbm-rows 0 --surface-cycles 0' 'k2|MPG_CGS_PARTIALS=1 MPG_FUSE_DOTS=1 MPG_FUSE_DOTS_K0=2|--hbm-rows 0 --surface-cycles 0' 'k4|MPG_CGS_PARTIALS=1 MPG_FUSE_DOTS=1 MPG_FUSE_DOTS_K0=4|--hbm-rows 0 --surface-cycles 0' 'k8|MPG_CGS_PARTIALS=1 MPG_FUSE_DOTS=1 MPG_FUSE_DOTS_K0=8|--hbm-rows 0 --surface-cycles 0' > gpurun_out/${tag}_ab_k0.txt") ;;
    c4pmc) for v in 0 1; do
             cmds+=("${tag}_c4f_share$v|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_c4_share${v}_fetch -o fetch -- python3 tools/spmv_ab.py --case c4 --var MPG_SELL_SHARE=$v --reps 1 --cycles 1")
             cmds+=("${tag}_c4h_share$v|200|timeout -s KILL 190 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${tag}_c4_share${v}_hit -o hit -- python3 tools/spmv_ab.py --case c4 --var MPG_SELL_SHARE=$v --reps 1 --cycles 1")
           done ;;
    irr) cmds+=("${tag}_irr|700|python -u tools/spmv_ab.py --case c4p --case fem27 --case fem27p --var spmv_format=auto --var spmv_format=csr --var spmv_format=sell,MPG_SELL_SIGMA=0 --reps 3 --cycles 1 > gpurun_out/${tag}_irr.jsonl") ;;
  esac
done
exec tools/gpu_steps.sh "${cmds[@]}"
