#!/bin/bash
# Extrema-scan occupancy / scale-group A/B (isolated extrema stage + pipelined rate), 2 rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in 1 2; do
  bash tools/gpu_libab.sh - build_var/xw5.so build_var/xw6.so build_var/xg3.so build_var/xg2.so || exit 1
done
