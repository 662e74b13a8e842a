#!/bin/bash
# Octaves >= 1 beside octave 0 (SIFT_OCONC: octave-1 base from launch_seed0, side stream): parity under the knob, then A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
SIFT_OCONC=1 SIFT_RW=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or detect_matches_reference or cfg3_4k_o4_s5_matches_oracle" > $O/pytest_r4l.log 2>&1 || { grep -E "PASS|FAIL|Error" $O/pytest_r4l.log | tail -30; exit 1; }
grep -cE "PASSED" $O/pytest_r4l.log; tail -n 1 $O/pytest_r4l.log
STEPS=60 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 - SIFT_OCONC=1 "SIFT_OCONC=1 SIFT_RW=1 SIFT_RW_R=12" "SIFT_OCONC=1 SIFT_RW=1"
