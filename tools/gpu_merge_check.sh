#!/bin/bash
# Shard / merge / collective tests, then the 8-shard critical-path model.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "shard or merge or dist or cfg5_8k_o6_s5_whole" > $O/t_merge.log 2>&1 || { echo tests failed; tail -30 $O/t_merge.log; exit 1; }
tail -1 $O/t_merge.log
timeout -k 10 200 python tools/shard_time_device.py 8 5 > $O/shard8_m.json 2> $O/shard8_m.err || { echo shard failed; tail -5 $O/shard8_m.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/shard8_m.json'));print(d['critical_path_ms'], d['merge_ms'], d['per_rank_ms'], d['identical'])"
