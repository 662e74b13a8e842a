#!/bin/bash
# One counter fill per detection (the block counts folded in): full GPU suite, then A/B vs the previous build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_r3w.log 2>&1 \
  || { tail -40 $O/pytest_gpu_r3w.log; exit 1; }
tail -1 $O/pytest_gpu_r3w.log
for rep in 1 2 3; do bash tools/gpu_libab.sh - build_var/prev.so || exit 1; done
