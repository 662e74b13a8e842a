#!/bin/bash
# GPU parity tests selected by PYTEST_K (optional), then the bench's
# isolated per-octave pass times and pipelined rate per environment setting,
# alternated and repeated.  usage: PYTEST_K=... tools/gpu_ab_oct.sh <reps> "<VAR=val ...>"...  ("-" = no extra env)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -k "$PYTEST_K" > $O/pytest_ab.log 2>&1 || { echo "pytest failed"; grep -E "PASS|FAIL|Error|error" $O/pytest_ab.log | tail -30; exit 1; }
  grep -cE "PASSED" $O/pytest_ab.log; tail -1 $O/pytest_ab.log
fi
reps=$1; shift
for r in $(seq $reps); do
  i=0
  for e in "$@"; do
    i=$((i+1)); [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline --sustain-s 0 ${BENCH_ARGS:-} > $O/ab_$i.json 2> $O/ab_$i.err || { echo "setting '$e' failed"; tail -5 $O/ab_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_$i.json')); r=d['roofline']; print('[$e]', d['value'], d['ms_per_step'], 'pass', r['launch_ms'], round(r['frac'],3), [round(o['iso_ms'],4) for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'], 'r', r.get('refine_stage',{}).get('iso_ms'), 'kp', d['keypoints'])"
  done
done
