#!/bin/bash
# Patch capture with per-unit slots (no atomics): parity + A/B against the scan without capture.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_r4p.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest_r4p.log | tail -30; exit 1; }
grep -c PASSED $O/pytest_r4p.log; tail -n 1 $O/pytest_r4p.log
STEPS=100 timeout -k 10 600 bash tools/gpu_ab_oct.sh 2 - "SIFT_HIP_LIB=$R/build_var/nopatch.so" "SIFT_HIP_LIB=$R/build_var/patch_w4.so"
timeout -k 10 120 ./tools/calib/d2h_probe 1024 > $O/d2h_probe_r4p.txt 2>&1 || { cat $O/d2h_probe_r4p.txt; exit 1; }
cat $O/d2h_probe_r4p.txt
