#!/bin/bash
# Interleaved A/B of two kernel builds (libmpgmres_hip.so) on the in-cycle
# Arnoldi SpMV of tools/spmv_ab.py cases: every build R times, in rotation.
# usage: tools/lib_ab.sh R "name|path/to/libmpgmres_hip.so" ... -- CASE...
set -u
R=$1; shift
libs=()
while [ "$1" != "--" ]; do libs+=("$1"); shift; done
shift
cases=()
for c in "$@"; do cases+=(--case "$c"); done
for ((r = 0; r < R; ++r)); do
  for spec in "${libs[@]}"; do
    name="${spec%%|*}"; lib="${spec#*|}"
    MPG_HIP_LIB="$lib" timeout -k 10 300 python tools/spmv_ab.py "${cases[@]}" --var MPG_AB_BUILD="$name" --reps 3 --cycles 1 || exit $?
  done
done
