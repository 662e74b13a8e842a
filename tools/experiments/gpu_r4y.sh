#!/bin/bash
# Stall counters of the split-octave kernels (k_gauss_vert 16-row chunks, k_gauss_hsp).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
timeout -k 10 600 bash tools/gpu_stall_pmc.sh hsp SIFT_HSP=1
