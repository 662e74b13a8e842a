#!/bin/bash
# k_gauss_rw<12> (octave 1): without plane stores, with a 4- / 2-wave register bound, and its stall counters.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=30 timeout -k 10 600 bash tools/gpu_ab_oct.sh 1 "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0" "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0 SIFT_GAUSS_DBG=1" "SIFT_RW=0 SIFT_GAUSS_DBG=1" "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0 SIFT_HIP_LIB=$R/build_var/rw4.so" "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0 SIFT_HIP_LIB=$R/build_var/rw2.so" || exit 1
timeout -k 10 600 bash tools/gpu_stall_pmc.sh rw12 "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0"
