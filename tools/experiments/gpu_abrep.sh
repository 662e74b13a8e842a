#!/bin/bash
# Pipelined bench value per library variant, alternated and repeated (noise check).
# usage: tools/gpu_abrep.sh <reps> <variant>...   (<name>_prio: SIFT_OCT0_PRIO=1)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
reps=$1; shift
for r in $(seq $reps); do
  for v in "$@"; do
    P=0; case $v in *_prio) P=1;; esac
    SIFT_OCT0_PRIO=$P SIFT_HIP_LIB=$R/build_var/$v.so timeout -k 10 200 python $R/bench.py --steps 200 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > $O/abr_$v.json 2> $O/abr_$v.err || { echo "variant $v bench failed"; tail -5 $O/abr_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/abr_$v.json')); print('$v', d['value'], d['ms_per_step'], d['stages_ms'])"
  done
done
