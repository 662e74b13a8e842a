#!/bin/bash
# r6p: hardware queues / contexts in flight for the default 4K bench (env only), alternated, 2 reps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
for rep in 1 2; do
  i=0
  for e in "-" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=8 --inflight 4" "- --inflight 4" "GPU_MAX_HW_QUEUES=8 --inflight 5"; do
    i=$((i+1)); envp=${e%% --*}; args=""; [[ "$e" == *"--"* ]] && args="--${e#*--}"; [ "$envp" = "-" ] && envp=""
    env $envp timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sustain-s 3 $args > $O/r6p_$i.json 2> $O/r6p_$i.err || { echo "bench '$e' failed"; tail -5 $O/r6p_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r6p_$i.json')); print('[$e]', d['value'], d['ms_per_step'], d['sustained']['value'], d['config']['inflight_per_gpu'], d['verified'])"
  done
done
