#!/bin/bash
# Round 3, call h: JS + batch + ABI tests (host batch entry point, detectBatch).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
echo "[$(date +%T)] pytest subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "js or batch or abi" > $O/pytest_r3h.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAIL|Error" $O/pytest_r3h.log | head -30; tail -5 $O/pytest_r3h.log; exit 1; }
tail -1 $O/pytest_r3h.log
