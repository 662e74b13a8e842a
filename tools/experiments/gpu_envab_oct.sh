#!/bin/bash
# Pipelined bench + isolated pass per environment setting, alternated and
# repeated, with the per-octave isolated launch times.  Optional first step:
# GPU parity tests selected by PYTEST_K (run under every setting's env? no:
# under the last setting given in PYTEST_ENV).
# usage: tools/gpu_envab_oct.sh <reps> "<VAR=val ...>"...   ("-" = no extra env)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R || exit 1
if [ -n "${PYTEST_K:-}" ]; then
  env ${PYTEST_ENV:-} timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" > $O/pytest_envab.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_envab.log; exit 1; }
  tail -2 $O/pytest_envab.log
fi
reps=$1; shift
for r in $(seq $reps); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/envab_$i.json 2> $O/envab_$i.err || { echo "setting '$e' failed"; tail -5 $O/envab_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/envab_$i.json')); r=d['roofline']; print('[$e]', d['value'], d['ms_per_step'], 'pass', r['launch_ms'], r['frac'], [o['iso_ms'] for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'])"
  done
done
