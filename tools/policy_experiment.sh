#!/bin/bash
# Cache-policy study on the GPU box: the headline bench (and the C3/C5
# configs) with the default load policy, then rebuilt with non-temporal
# matrix streams (MPG_CSR_NT: CSR tiles incl. the fp64 residual; MPG_SELL_NT:
# the Arnoldi SELL slices). Each variant is a full rebuild of libmpgmres_hip.
# usage (on the box): bash tools/policy_experiment.sh
set -u
mkdir -p gpurun_out
bench() {  # name [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > gpurun_out/pol_$name.json 2> gpurun_out/pol_$name.err
  local rc=$?
  echo "[$name] rc=$rc $(python -c "import json;d=json.loads(open('gpurun_out/pol_$name.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'])" 2>/dev/null)"
  return $rc
}
run() {  # name flags
  local name=$1; shift
  make -C icl-mixed-precision-gmres_amd -j16 EXTRA_HIPFLAGS="$*" > gpurun_out/pol_build_$name.log 2>&1 || return 2
  bench $name MPG_NOP=0
}
touch icl-mixed-precision-gmres_amd/csrc/*.hip
run base "" || exit $?
bench base_cgspart MPG_CGS_PARTIALS=1 || exit $?
touch icl-mixed-precision-gmres_amd/csrc/*.hip
run csr_nt "-DMPG_CSR_NT=1" || exit $?
touch icl-mixed-precision-gmres_amd/csrc/*.hip
run sell_nt "-DMPG_SELL_NT=1" || exit $?
touch icl-mixed-precision-gmres_amd/csrc/*.hip
run both_nt "-DMPG_CSR_NT=1 -DMPG_SELL_NT=1" || exit $?
