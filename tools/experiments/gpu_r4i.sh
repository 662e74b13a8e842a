#!/bin/bash
# Stall counters of k_gauss_pc<12> (octave 1): full, and with every part switched off (SIFT_GAUSS_DBG=15).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
bash tools/gpu_stall_pmc.sh pc "SIFT_RW=1 SIFT_RW_R=12" && bash tools/gpu_stall_pmc.sh pc15 "SIFT_RW=1 SIFT_RW_R=12 SIFT_GAUSS_DBG=15"
