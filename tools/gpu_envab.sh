#!/bin/bash
# Pipelined bench per environment setting, alternated and repeated.
# usage: tools/gpu_envab.sh <reps> "<VAR=val ...>"...   ("-" = no extra env)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
reps=$1; shift
for r in $(seq $reps); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python $R/bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/envab_$i.json 2> $O/envab_$i.err || { echo "setting '$e' failed"; tail -5 $O/envab_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/envab_$i.json')); print('[$e]', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
  done
done
