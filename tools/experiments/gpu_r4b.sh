#!/bin/bash
# Diagnostics of the small octaves on the experiments build: plane stores off
# (SIFT_GAUSS_DBG=1), the LDS-resident base (SIFT_GAUSS_LDS=1), both.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=60 timeout -k 10 600 bash tools/gpu_ab_oct.sh 2 - SIFT_GAUSS_DBG=1 SIFT_GAUSS_LDS=1 "SIFT_GAUSS_LDS=1 SIFT_GAUSS_DBG=1" "SIFT_GAUSS_GROUPS=2,2,2" "SIFT_GAUSS_GROUPS=2,2,2 SIFT_GAUSS_DBG=1"
