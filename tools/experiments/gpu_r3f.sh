#!/bin/bash
# Round 3, call f: word-pass A/B (bench image; saturated images through the
# stage probe in key mode), then the round artifacts (tools/gpu_round.sh r3f).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
echo "[$(date +%T)] stage probe, per-pixel keys (SIFT_XWORDS=0)"
SIFT_HIP_LIB=$R/build_var/exp4.so SIFT_XWORDS=0 timeout -k 10 150 python -u tools/stage_probe.py > $O/stage_probe_r3f_keys.txt 2>&1 || { echo "probe keys failed"; tail -20 $O/stage_probe_r3f_keys.txt; exit 1; }
grep -v amdgpu.ids $O/stage_probe_r3f_keys.txt
echo "[$(date +%T)] A/B word pass on the bench image"
SIFT_HIP_LIB=$R/build_var/exp4.so tools/gpu_ab_oct.sh 2 "-" "SIFT_XWORDS=0" || exit 1
echo "[$(date +%T)] round artifacts"
tools/gpu_round.sh r3f || exit 1
