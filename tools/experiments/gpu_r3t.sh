#!/bin/bash
# Seed-only kernels with 8 outputs per thread: range / shard tests, cfg 5 model.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "range or shard or dist or gather or next_seed or whole_vs" > $O/pytest_r3t.log 2>&1 \
  || { tail -40 $O/pytest_r3t.log; exit 1; }
tail -1 $O/pytest_r3t.log
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r3t.json 2> $O/shard8_r3t.err || { tail -5 $O/shard8_r3t.err; exit 1; }
grep "^{" $O/shard8_r3t.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['critical_path_ms'], d['tail_octave_ms'], d['shard_ms'], d['merge_ms'], d['whole_ms'], d['speedup_vs_whole'], d['identical'])"
