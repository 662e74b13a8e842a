#!/bin/bash
# Quick GPU check: selected tests (-k expression), one bench line, one
# pipelined kernel trace.  usage: tools/gpu_quick.sh <tag> "<pytest -k expr>"
TAG=$1; K=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd $R || exit 1
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/t_$TAG.log 2>&1 || { echo tests failed; tail -30 $O/t_$TAG.log; exit 1; }
  tail -2 $O/t_$TAG.log
fi
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b_$TAG.json 2> $O/b_$TAG.err || { echo bench failed; tail -5 $O/b_$TAG.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > /dev/null 2> $O/prof_$TAG.err || { echo trace failed; exit 1; }
echo done
