#!/bin/bash
# Round 3, call g: hybrid word/pixel exact pass: parity subset, A/B vs per-pixel keys, probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
echo "[$(date +%T)] pytest subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "saturated or cfg3 or lattice or golden or batch or planes or reference_itself or 1080" > $O/pytest_r3g.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAIL|Error" $O/pytest_r3g.log | head -30; tail -5 $O/pytest_r3g.log; exit 1; }
tail -1 $O/pytest_r3g.log
echo "[$(date +%T)] stage probe (words)"
timeout -k 10 150 python -u tools/stage_probe.py > $O/stage_probe_r3g.txt 2>&1 || { echo "probe failed"; tail -20 $O/stage_probe_r3g.txt; exit 1; }
grep -v amdgpu.ids $O/stage_probe_r3g.txt
echo "[$(date +%T)] A/B word pass on the bench image"
SIFT_HIP_LIB=$R/build_var/exp5.so tools/gpu_ab_oct.sh 3 "-" "SIFT_XWORDS=0" || exit 1
echo "[$(date +%T)] done"
