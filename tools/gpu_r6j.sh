#!/bin/bash
# r6j: GPU suite + smoke on the shipping build.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6j_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/r6j_pytest_gpu.log; exit 1; }
tail -3 $O/r6j_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/r6j_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/r6j_smoke.log; exit 1; }
cat $O/r6j_smoke.log
