#!/bin/bash
# Stall / issue counters of the small-octave kernels: k_gauss_rw vs k_gauss_dog (experiments build).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
bash tools/gpu_stall_pmc.sh rw1 SIFT_RW=1 && bash tools/gpu_stall_pmc.sh rw0 SIFT_RW=0
