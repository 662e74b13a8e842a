#!/bin/bash
# Pipelining sweep on the current build: --overlap mode x detections in flight.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
for m in octave0:3 octave0:2 octave0:4 refinement:3 full:3 phased:3 gaussian:3 octave0:3; do
  mode=${m%%:*}; n=${m##*:}
  timeout -k 10 200 python $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --overlap $mode --inflight $n > $O/sw.json 2> $O/sw.err || { echo "mode $m failed"; tail -5 $O/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sw.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'])"
done
