#!/bin/bash
# Pipelined bench: detections in flight per GPU (3 = default vs 2, 4), 2 rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in 1 2; do
  for n in 3 4 2; do
    timeout -k 10 150 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --inflight $n > $O/inf.json 2> $O/inf.err || { tail -3 $O/inf.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/inf.json').read().strip().splitlines()[-1]);print('inflight $n', d['value'], d['ms_per_step'], d['sustained']['value'])"
  done
done
