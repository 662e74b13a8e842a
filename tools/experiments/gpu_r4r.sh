#!/bin/bash
# Re-entry baseline: smoke, then the register-window small-octave kernels A/B (k_gauss_dog / k_gauss_pc / k_gauss_rw).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_r4r.log 2>&1 || { tail -20 $O/smoke_r4r.log; exit 1; }
tail -2 $O/smoke_r4r.log
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 SIFT_RW=0 "SIFT_RW=1 SIFT_RW_R=12" "SIFT_RW=1 SIFT_RW_R=12 SIFT_PC=0" "SIFT_RW=1 SIFT_RW_R=24 SIFT_RW_MINB=2000" "SIFT_RW=1 SIFT_RW_R=24 SIFT_PC=0"
