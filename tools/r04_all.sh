#!/bin/bash
# Round-4 battery in one gpurun call: the new GPU tests, then the perf steps
# of tools/r04_perf.sh (each step has its own time limit).
set -u
tag=${1:-r04a}
tools/gpu_steps.sh "${tag}_tests|600|python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_m100_gpu.py tests/test_dist_gpu.py::test_fold_decision_is_collective tests/test_dist_gpu.py::test_rccl_single_rank_bits tests/test_dist_gpu.py::test_rccl_eager_matches_captured tests/test_dist_gpu.py::test_rccl_watchdog_names_rank_and_cycle tests/test_solve_gpu.py::test_long_restart_matches_oracle tests/test_solve_gpu.py::test_round4_kernel_variants_same_bits tests/test_solve_gpu.py::test_breakdown_report_and_stop tests/test_half_gpu.py::test_row_scaled_unscaling_on_every_sell_kernel tests/test_irregular_gpu.py" || exit $?
exec tools/r04_perf.sh "$tag" probe bench b100 prof prof100 pmcf pmcw
