#!/bin/bash
# Pipelined bench: detections in flight per GPU (2 / 3 / 4 / 5) on the final round-4 build, alternated, 3 reps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in 1 2 3 4; do
  for n in 2 3 5; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sustain-s 0 --inflight $n > $O/inf_$n.json 2> $O/inf_$n.err || { echo "inflight $n failed"; tail -3 $O/inf_$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/inf_$n.json').read().strip().splitlines()[-1]); print('inflight $n', d['value'], d['ms_per_step'])"
  done
done
