#!/bin/bash
# Round 3, call h: JS + batch + ABI tests (host batch entry point, detectBatch).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
echo "[$(date +%T)] pytest subset"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "js or batch or abi" > $O/pytest_r3h.log 2>&1 || { echo "pytest failed"; grep -E "^E |FAIL|Error" $O/pytest_r3h.log | head -30; tail -5 $O/pytest_r3h.log; exit 1; }
tail -1 $O/pytest_r3h.log
fi
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
  SIFT_HIP_LIB=$R/build_var/exp5.so SIFT_XWORDS=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xw$m -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_xw$m.err || { echo "trace $m failed"; tail -5 $O/prof_xw$m.err; exit 1; }
  echo "SIFT_XWORDS=$m"; python3 $R/tools/kstats.py $O/prof_xw$m/run_kernel_stats.csv | grep -E "extrema|exact|emit"
done
