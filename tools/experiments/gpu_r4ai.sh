#!/bin/bash
# Octave 2's vertical pass with the next chunk prefetched (SIFT_VG2_PF=1; pf3: with a 3-block-per-CU bound):
# parity subset on pf3, then A/B against exp (no prefetch).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
SIFT_HIP_LIB=$R/build_var/pf3.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or large_radii or reference_itself" > $O/pytest_r4ai.log 2>&1 || { grep -E "passed|failed|assert" $O/pytest_r4ai.log | tail -10; exit 1; }
tail -n 1 $O/pytest_r4ai.log
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 "SIFT_HIP_LIB=$R/build_var/exp.so" "SIFT_HIP_LIB=$R/build_var/pf2.so" "SIFT_HIP_LIB=$R/build_var/pf3.so"
