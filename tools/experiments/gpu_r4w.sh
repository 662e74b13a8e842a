#!/bin/bash
# Split octaves: 16-row chunked k_gauss_vert + scale-parallel horizontal pass k_gauss_hsp. Parity subset on the
# product library, then A/B (ch8: the 8-row chunked split pass + tile kernel; exp SIFT_HSP=0: 16-row chunks + tile kernel).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or unaligned or cfg5_radii or detect_matches_reference or range_detection or saturated or reference_itself" \
  > $O/pytest_r4w.log 2>&1 || { grep -E "PASS|FAIL|Error|passed|failed|assert" $O/pytest_r4w.log | tail -30; exit 1; }
tail -n 1 $O/pytest_r4w.log
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 "SIFT_HSP=0 SIFT_HIP_LIB=$R/build_var/ch8.so" SIFT_HSP=0 SIFT_HSP=1 "SIFT_HSP=1 SIFT_HIP_LIB=$R/build_var/ch8.so" "SIFT_HSP=1 SIFT_VSPLIT_R=20"
