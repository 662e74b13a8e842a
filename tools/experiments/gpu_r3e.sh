#!/bin/bash
# Round 3, call e: full GPU suite (ambiguous-word exact pass, saturated images),
# stage probe (seed 1 saturated vs seed 42), A/B of the word pass on the bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r3e.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAIL|Error" $O/pytest_r3e.log | head -30; tail -5 $O/pytest_r3e.log; exit 1; }
tail -1 $O/pytest_r3e.log; grep -h "saturated\|dot lattice" $O/pytest_r3e.log | head
echo "[$(date +%T)] stage-API extrema probe"
timeout -k 10 200 python tools/stage_probe.py > $O/stage_probe_r3e.txt 2>&1 || { echo "probe failed"; tail -20 $O/stage_probe_r3e.txt; exit 1; }
grep -v amdgpu.ids $O/stage_probe_r3e.txt
SIFT_HIP_LIB=$R/build_var/exp4.so SIFT_XWORDS=0 timeout -k 10 200 python tools/stage_probe.py > $O/stage_probe_r3e_keys.txt 2>&1 || { echo "probe keys failed"; tail -20 $O/stage_probe_r3e_keys.txt; exit 1; }
grep -v amdgpu.ids $O/stage_probe_r3e_keys.txt
echo "[$(date +%T)] A/B word pass on the bench image"
SIFT_HIP_LIB=$R/build_var/exp4.so tools/gpu_ab_oct.sh 2 "-" "SIFT_XWORDS=0" || exit 1
echo "[$(date +%T)] done"
