#!/bin/bash
# k_gauss_rs (sliding register window, octaves >= 1): parity subset under the knob, then A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
SIFT_RS=1 SIFT_RS_R=24 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or unaligned or cfg5_radii or detect_matches_reference or range_detection" \
  > $O/pytest_r4t.log 2>&1 || { grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_r4t.log | tail -30; exit 1; }
tail -n 1 $O/pytest_r4t.log
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 SIFT_RS=0 "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0" SIFT_RS=1 "SIFT_RS=1 SIFT_RS_BLOCKS=512" "SIFT_RS=1 SIFT_RS_BLOCKS=1024" "SIFT_RS=1 SIFT_RS_R=24" "SIFT_RS=1 SIFT_HIP_LIB=$R/build_var/rs3.so" "SIFT_RS=1 SIFT_RS_BLOCKS=1024 SIFT_HIP_LIB=$R/build_var/rs3.so"
