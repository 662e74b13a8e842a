#!/bin/bash
# k_gauss_pc after the b128 read fix: strip read depth A/B and parts switched off.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for lib in exp exp_pf5; do
  echo "== $lib"
  SIFT_HIP_LIB=$R/build_var/$lib.so STEPS=30 timeout -k 10 600 bash tools/gpu_ab_oct.sh 1 SIFT_RW=0 "SIFT_RW=1 SIFT_RW_R=12" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=1" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=5" "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=3" || exit 1
done
