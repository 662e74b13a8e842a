#!/bin/bash
# k_gauss_pc with the epilogue inside each radius variant; scale groups A/B for octave 2/3 through pc.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=40 timeout -k 10 600 bash tools/gpu_ab_oct.sh 2 SIFT_RW=0 "SIFT_RW=1 SIFT_RW_R=12" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=1" "SIFT_RW=1 SIFT_RW_R=24 SIFT_RW_MINB=2000"
