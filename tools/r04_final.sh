#!/bin/bash
# Round-4 closing battery on the gpurun box, one step per measurement, each
# under its own time limit (tools/gpu_steps.sh stops at anything other than
# pass / test failures): the GPU suite, smoke(), the bench line, the rocprofv3
# summary of the bench command, the timing probe, the BASELINE configs.
#   tools/r04_final.sh TAG
set -u
tag=${1:-r04z}
exec tools/gpu_steps.sh \
  "${tag}_suite|900|python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "${tag}_smoke|240|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "${tag}_bench|420|python -u bench.py > gpurun_out/${tag}_bench.json" \
  "${tag}_prof|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 10 --no-cpu-baseline --hbm-rows 0 --surface-cycles 0 > gpurun_out/${tag}_prof_bench.json" \
  "${tag}_probe|200|python3 tools/timing_probe.py --torch > gpurun_out/${tag}_probe.json" \
  "${tag}_configs|900|python -u tools/bench_configs.py --cycles 6 --cpu-cycles 1 --out gpurun_out/${tag}_configs.jsonl"
