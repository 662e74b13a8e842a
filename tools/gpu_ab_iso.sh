#!/bin/bash
# A/B of library builds (build_ab/<name>.so), alternated, <reps> reps: throughput, isolated pass and per-octave times.
# usage: tools/gpu_ab_iso.sh <tag> <reps> <name>...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
tag=$1; reps=$2; shift 2
for rep in $(seq $reps); do
  for v in "$@"; do
    SIFT_HIP_LIB=$R/build_ab/$v.so timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/${tag}_$v.json 2> $O/${tag}_$v.err || { echo "bench $v failed"; tail -5 $O/${tag}_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${tag}_$v.json')); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'pass', r['launch_ms'], r['frac'], [o['iso_ms'] for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'], 'ref', r['refine_stage']['iso_ms'], d['verified'])"
  done
done
