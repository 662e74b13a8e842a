#!/bin/bash
# Isolated per-octave Gaussian times and pipelined throughput per library
# build (SIFT_HIP_LIB); "-" = the in-tree library.  Variants alternate over
# REPS rounds (default 2) so box drift hits every variant alike.
# usage: [REPS=n] [STEPS=n] tools/gpu_libab.sh lib1.so[:VAR=v,VAR2=w] lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for rep in $(seq 1 ${REPS:-2}); do
for l in "$@"; do
  lib=${l%%:*}; ev=""; [ "$lib" != "$l" ] && ev=$(echo "${l#*:}" | tr ',' ' ')
  if [ "$lib" = "-" ]; then e="$ev"; else e="SIFT_HIP_LIB=$R/$lib $ev"; fi
  env $e timeout -k 10 150 python bench.py --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --sustain-s 0 ${BENCH_ARGS} > $O/lab.json 2>$O/lab.err || { echo "$l failed"; tail -3 $O/lab.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/lab.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$l', d['value'], d['ms_per_step'], 'pass iso', r['launch_ms'], [o['iso_ms'] for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'], 'ref', r['refine_stage']['iso_ms'], 'ok', d['verified'])"
done
done
