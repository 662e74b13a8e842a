#!/bin/bash
# bench.py throughput vs detections in flight (octave0 ordering and full overlap)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
for m in octave0:3 octave0:4 octave0:5 full:3 full:4; do
  mode=${m%%:*}; n=${m##*:}
  timeout -k 10 200 python $R/bench.py --steps 60 --warmup 6 --no-cpu-baseline --overlap $mode --inflight $n > $O/infl_${mode}_$n.json 2> $O/infl_${mode}_$n.err || { echo "mode $m failed"; tail -5 $O/infl_${mode}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/infl_${mode}_$n.json')); print('$m', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
