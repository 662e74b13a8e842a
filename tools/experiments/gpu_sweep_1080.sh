#!/bin/bash
# 1080p pipelining: detections in flight x overlap mode (BASELINE cfg 2 / cfg 4).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
for m in octave0:3 octave0:4 octave0:6 full:4 full:6 octave0:8; do
  mode=${m%%:*}; n=${m##*:}
  timeout -k 10 200 python $R/bench.py --width 1920 --height 1080 --steps 200 --warmup 10 --no-cpu-baseline --overlap $mode --inflight $n > $O/sw.json 2> $O/sw.err || { echo "mode $m failed"; tail -5 $O/sw.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sw.json').read().strip().splitlines()[-1]); print('$m', d['value'], d['ms_per_step'])"
done
