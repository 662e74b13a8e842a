#!/bin/bash
# Round-3 first call: round artifacts on HEAD, then A/B of the LDS-resident
# small-octave kernel (experiments build, SIFT_GAUSS_LDS=1 vs 0).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
tools/gpu_round.sh r3a || exit 1
cd $R
echo "[$(date +%T)] parity with SIFT_GAUSS_LDS=1"
SIFT_HIP_LIB=$R/build_var/exp.so SIFT_GAUSS_LDS=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "planes_bit_exact or cfg3 or golden" > $O/pytest_lds.log 2>&1 || { echo "pytest lds failed"; tail -30 $O/pytest_lds.log; exit 1; }
tail -1 $O/pytest_lds.log
echo "[$(date +%T)] A/B SIFT_GAUSS_LDS"
SIFT_HIP_LIB=$R/build_var/exp.so tools/gpu_ab_oct.sh 2 "-" "SIFT_GAUSS_LDS=1" || exit 1
