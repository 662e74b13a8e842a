#!/bin/bash
# bench.py under each --overlap mode (and octave0 with 3 in flight)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for m in none octave0 gaussian refinement full octave0:3; do
  mode=${m%%:*}; n=2; [ "$m" != "$mode" ] && n=${m##*:}
  timeout -k 10 200 python $R/bench.py --steps 40 --warmup 5 --no-cpu-baseline --overlap $mode --inflight $n > $O/mode_${mode}_$n.json 2> $O/mode_${mode}_$n.err || { echo "mode $m failed"; tail -5 $O/mode_${mode}_$n.err; exit 1; }
  echo "mode $m ok"
done
