#!/bin/bash
# The GPU battery of a round on the gpurun box, one step per measurement, each
# under its own time limit (tools/gpu_steps.sh stops the chain at anything
# other than pass / test failures). Replaces the per-round r0x_*.sh scripts.
#   tools/battery.sh TAG step [step ...]
# steps:
#   suite    the whole GPU test suite            smoke    __graft_entry__.smoke()
#   bench    the default bench line               bench100 bench at GMRES(100)
#   prof     rocprofv3 kernel trace + stats of the bench command
#   pmcf / pmcw   FETCH_SIZE / WRITE_SIZE passes of the bench command (separate runs)
#   probe    tools/timing_probe.py                configs  tools/bench_configs.py
#   irr      irregular SpMV A/B (c4p, fem27, fem27p; auto / csr / sell)
#   irrpmc   FETCH_SIZE, WRITE_SIZE and TCC hit/miss passes of the irregular SpMVs
#   c4pmc    FETCH_SIZE and TCC hit/miss passes of C4's stepped SpMV
#   lappmc   FETCH_SIZE, WRITE_SIZE and TCC hit/miss passes of LAP-1M's SpMV
#   n2       bench --gpus 2 rehearsal with both ranks on GPU 0 (gloo host transport)
#   node     node-block SpMV A/B (tiles per workgroup, XCD order) on the 3-dof stand-ins
#   ranks    C4 / C5 rank blocks at P = 8 (tools/rank_blocks.py), and C4's under PMC
#   surfirr  the operator surface against the fused engine on fem27 and C4's stencil (node blocks)
set -u
tag=${1:?usage: tools/battery.sh TAG step...}
shift
nob="--no-cpu-baseline --hbm-rows 0 --surface-cycles 0"
cmds=()
for s in "$@"; do
  case $s in
    suite) cmds+=("${tag}_suite|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider") ;;
    smoke) cmds+=("${tag}_smoke|240|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'") ;;
    bench) cmds+=("${tag}_bench|420|python -u bench.py > gpurun_out/${tag}_bench.json") ;;
    bench100) cmds+=("${tag}_b100|240|python -u bench.py --rlen 100 --steps 5 --warmup 1 $nob > gpurun_out/${tag}_b100.json") ;;
    prof) cmds+=("${tag}_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 10 $nob > gpurun_out/${tag}_prof_bench.json") ;;
    pmcf) cmds+=("${tag}_pmcf|150|timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_pmc_fetch -o fetch -- python3 bench.py --steps 3 --warmup 1 $nob") ;;
    pmcw) cmds+=("${tag}_pmcw|150|timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_pmc_write -o write -- python3 bench.py --steps 3 --warmup 1 $nob") ;;
    probe) cmds+=("${tag}_probe|200|python3 tools/timing_probe.py --torch > gpurun_out/${tag}_probe.json") ;;
    configs) cmds+=("${tag}_configs|900|python -u tools/bench_configs.py --cycles 6 --cpu-cycles 1 --out gpurun_out/${tag}_configs.jsonl") ;;
    irr) cmds+=("${tag}_irr|700|python -u tools/spmv_ab.py --case c4p --case fem27 --case fem27p --var spmv_format=auto --var spmv_format=csr --var spmv_format=sell,MPG_SELL_SIGMA=0 --reps 3 --cycles 1 > gpurun_out/${tag}_irr.jsonl") ;;
    node) cmds+=("${tag}_node|600|python -u tools/spmv_ab.py --case fem27 --case fem27p --case c4p --case c4 --var spmv_format=node --var spmv_format=node,MPG_NODE_TPW=1 --var spmv_format=node,MPG_NODE_TPW=4 --var spmv_format=node,MPG_NODE_XCD=0 --var spmv_format=node,MPG_NODE_XCD=1 --reps 3 --cycles 1 > gpurun_out/${tag}_node.jsonl") ;;
    ranks) cmds+=("${tag}_ranks|300|python -u tools/rank_blocks.py --ranks 8 --config c4 c5 --which 0,big,last > gpurun_out/${tag}_ranks.jsonl")
           cmds+=("${tag}_rkf|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_rank_pmc/fetch -o fetch -- python3 tools/rank_blocks.py --ranks 8 --config c4 --which 0,big")
           cmds+=("${tag}_rkw|200|timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_rank_pmc/write -o write -- python3 tools/rank_blocks.py --ranks 8 --config c4 --which 0,big") ;;
    irrpmc) for c in c4p fem27 fem27p; do
              cmds+=("${tag}_${c}_f|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_irrpmc/${c}_fetch -o fetch -- python3 tools/spmv_ab.py --case $c --var spmv_format=auto --reps 1 --cycles 1")
              cmds+=("${tag}_${c}_w|200|timeout -s KILL 190 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${tag}_irrpmc/${c}_write -o write -- python3 tools/spmv_ab.py --case $c --var spmv_format=auto --reps 1 --cycles 1")
              cmds+=("${tag}_${c}_h|200|timeout -s KILL 190 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${tag}_irrpmc/${c}_hit -o hit -- python3 tools/spmv_ab.py --case $c --var spmv_format=auto --reps 1 --cycles 1")
            done ;;
    lappmc) for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:hit"; do
              cmds+=("${tag}_lap_${pass##*:}|200|timeout -s KILL 190 rocprofv3 --pmc ${pass%%:*} --output-format csv -d gpurun_out/${tag}_lappmc/${pass##*:} -o ${pass##*:} -- python3 tools/spmv_ab.py --case lap1m --var spmv_format=auto --reps 1 --cycles 1")
            done ;;
    c4pmc) cmds+=("${tag}_c4f|200|timeout -s KILL 190 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_c4pmc/fetch -o fetch -- python3 tools/spmv_ab.py --case c4 --var spmv_format=auto --reps 1 --cycles 1")
           cmds+=("${tag}_c4h|200|timeout -s KILL 190 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/${tag}_c4pmc/hit -o hit -- python3 tools/spmv_ab.py --case c4 --var spmv_format=auto --reps 1 --cycles 1") ;;
    surfirr) for sp in fem27:111 stencil27:111; do
               cmds+=("${tag}_surf_${sp%%:*}|400|python -u tools/surface_vs_fused.py cgs --spec=$sp --cycles=10")
             done ;;
    n2) cmds+=("${tag}_n2|400|MPG_BENCH_SHARED_GPU=1 python -u bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/${tag}_bench_n2.json") ;;
    *) echo "unknown step $s" >&2; exit 2 ;;
  esac
done
exec tools/gpu_steps.sh "${cmds[@]}"
