#!/bin/bash
# Banded Gaussian pass (SIFT_OBANDS): GPU parity suite with bands, then the
# pipelined bench and the isolated pass per band count.
# usage: tools/gpu_bands_ab.sh "<band counts>" [pytest args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R || exit 1
NB=${1:-"1 2 4 8"}
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
  SIFT_OBANDS=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${2:-} > $O/pytest_bands.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_bands.log; exit 1; }
  tail -2 $O/pytest_bands.log
fi
for r in 1 2; do
  for b in $NB; do
    SIFT_OBANDS=$b timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/bands_$b.json 2> $O/bands_$b.err || { echo "bench bands=$b failed"; tail -5 $O/bands_$b.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bands_$b.json')); r=d['roofline']; print('bands=$b', d['value'], d['ms_per_step'], 'pass iso', r['launch_ms'], 'frac', r['frac'], 'per-oct', [o['iso_ms'] for o in r['per_octave']], 'pipelined pass', r['pipelined']['ms'])"
  done
done
