#!/bin/bash
# k_gauss_pc with parts switched off (SIFT_GAUSS_DBG bits: 1 stores, 2 horizontal fmas, 4 vertical fmas, 8 window loads).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=30 timeout -k 10 600 bash tools/gpu_ab_oct.sh 1 "SIFT_RW=1 SIFT_RW_R=12" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=7" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=15" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=9" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=8"
