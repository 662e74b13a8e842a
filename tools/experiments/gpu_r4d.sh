#!/bin/bash
# L2 working set of the small octaves: blocks per CU capped (SIFT_GAUSS_BPC), k_gauss_dog and k_gauss_wide.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 1 SIFT_WIDE=0 "SIFT_WIDE=0 SIFT_GAUSS_BPC=3,3,3" "SIFT_WIDE=0 SIFT_GAUSS_BPC=2,2,2" "SIFT_WIDE=0 SIFT_GAUSS_BPC=1,1,1" SIFT_WIDE=1 "SIFT_WIDE=1 SIFT_GAUSS_BPC=2,2,2" "SIFT_WIDE=1 SIFT_GAUSS_BPC=1,1,1"
