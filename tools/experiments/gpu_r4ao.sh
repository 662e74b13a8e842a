#!/bin/bash
# Pipelined bench: overlap point x detections in flight (2 / 3) on the final round-4 build, alternated, 3 reps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in 1 2 3; do
  for ov in octave0 gaussian full; do
    for n in 2 3; do
      timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sustain-s 0 --inflight $n --overlap $ov > $O/ov.json 2> $O/ov.err || { echo "$ov $n failed"; tail -3 $O/ov.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ov.json').read().strip().splitlines()[-1]); print('overlap $ov inflight $n', d['value'], d['ms_per_step'])"
    done
  done
done
