#!/bin/bash
# Refinement band order (SIFT_BAND_ORDER): GPU suite, kernel-trace and
# FETCH_SIZE of k_refine_fast per setting, pipelined bench A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_border.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_border.log; exit 1; }
tail -2 $O/pytest_border.log
fi
for X in 0 1; do
  cd /tmp
  SIFT_BAND_ORDER=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bo$X -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_bo$X.err || { echo "trace failed"; tail -5 $O/prof_bo$X.err; exit 1; }
  grep -E "k_refine_fast|k_band" $O/prof_bo$X/run_kernel_stats.csv | cut -d, -f1-4 | sed "s/^/BO=$X /"
  SIFT_BAND_ORDER=$X timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bo$X -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sustain-s 0 > /dev/null 2> $O/pmc_bo$X.err || { echo "pmc failed"; tail -5 $O/pmc_bo$X.err; exit 1; }
done
cd $R
bash tools/gpu_envab_oct.sh 2 SIFT_BAND_ORDER=0 SIFT_BAND_ORDER=1
