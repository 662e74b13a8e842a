#!/bin/bash
# Exact refinement block size A/B (256 in-tree vs 64 = one wave, 128), pipelined rate, 3 rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in 1 2 3; do
  bash tools/gpu_libab.sh - build_var/rt64.so build_var/rt128.so || exit 1
done
