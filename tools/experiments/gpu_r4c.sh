#!/bin/bash
# k_gauss_wide: parity subset (planes bit-exact, radii, batches, bands, odd sizes), then A/B against k_gauss_dog.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or unaligned or cfg5_radii or detect_matches_reference or range_detection" \
  > $O/pytest_r4c.log 2>&1 || { grep -E "PASS|FAIL|Error" $O/pytest_r4c.log | tail -30; exit 1; }
grep -cE "PASSED" $O/pytest_r4c.log; tail -n 1 $O/pytest_r4c.log
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=60 timeout -k 10 600 bash tools/gpu_ab_oct.sh 2 SIFT_WIDE=0 SIFT_WIDE=1 "SIFT_WIDE=1 SIFT_WIDE_MINB=800" "SIFT_WIDE=1 SIFT_WIDE_R=32"
