#!/bin/bash
# Interleaved A/B of another built tree (DIR with its own package, libraries
# and tools/spmv_ab.py) against this one on the in-cycle Arnoldi SpMV:
#   tools/tree_ab.sh R DIR CASE...
set -u
R=$1; other=$2; shift 2
cases=()
for c in "$@"; do cases+=(--case "$c"); done
for ((r = 0; r < R; ++r)); do
  (cd "$other" && timeout -k 10 300 python tools/spmv_ab.py "${cases[@]}" --var MPG_AB_TREE=other --reps 3 --cycles 1) || exit $?
  timeout -k 10 300 python tools/spmv_ab.py "${cases[@]}" --var MPG_AB_TREE=this --reps 3 --cycles 1 || exit $?
done
