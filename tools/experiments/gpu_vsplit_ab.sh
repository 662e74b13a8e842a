#!/bin/bash
# Split vertical pass A/B: isolated per-octave Gaussian times at 4K O4 and 8K
# O6 with SIFT_VSPLIT_R = 0 (off), 40 (default), 20; then the 8-shard model.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd $R || exit 1
for geo in "3840 2160 4" "7680 4320 6"; do
  set -- $geo
  for v in 0 40 20; do
    SIFT_VSPLIT_R=$v timeout -k 10 150 python bench.py --width $1 --height $2 --octaves $3 --steps 20 --warmup 3 --no-cpu-baseline > $O/vs.json 2>$O/vs.err || { echo "bench $geo $v failed"; tail -3 $O/vs.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('$O/vs.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$1x$2 vsplit_r=$v', d['value'], d['ms_per_step'], 'pass iso', r['launch_ms'], r['frac'], [(o['octave'], o['iso_ms']) for o in r['per_octave']])"
  done
done
timeout -k 10 200 python tools/shard_time_device.py 8 5 > $O/shard8_vs.json 2> $O/shard8_vs.err || { echo shard failed; tail -3 $O/shard8_vs.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/shard8_vs.json'));print('shard8', d['critical_path_ms'], d['whole_ms'], d['identical'], d['per_rank_ms'], d['tail_octave_ms'], d['merge_ms'])"
