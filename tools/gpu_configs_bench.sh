#!/bin/bash
# Bench lines for every BASELINE configuration that fits one GPU (cfg 1 is CPU
# plumbing): cfg 2 (1080p O4 S5), cfg 3 (4K O4 S5, the metric's), cfg 4 (1080p x 8
# per GPU), cfg 5 (8K O6 S5 whole image, and as --shard-image at N=1).
# 8 hardware queues: the small and batched configurations then run 4 contexts (bench.py, r5w_schedule_ab.txt).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export GPU_MAX_HW_QUEUES=8  # the box exports 4
run() {  # name, args
  local n=$1; shift
  timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 "$@" > $O/cfg_$n.json 2> $O/cfg_$n.err || { echo "$n failed"; tail -3 $O/cfg_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/cfg_$n.json').read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print('$n', d['value'], d['unit'], d['ms_per_step'], 'pass frac', r.get('frac'))"
}
run cfg2_1080p --width 1920 --height 1080
run cfg3_4k
run cfg4_1080p_x8 --width 1920 --height 1080 --batch 8
run cfg5_8k_whole --width 7680 --height 4320 --octaves 6
timeout -k 10 200 python bench.py --shard-image --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 > $O/cfg_cfg5_shard.json 2> $O/cfg_cfg5_shard.err || { echo shard failed; exit 1; }
python3 -c "import json; d=json.loads(open('$O/cfg_cfg5_shard.json').read().strip().splitlines()[-1]); print('cfg5_shard_image_n1', d['value'], d['unit'], d['ms_per_step'])"
