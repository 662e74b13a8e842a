#!/bin/bash
# Seed-only tail octaves and padded-list merges: range / shard / dist tests,
# then the cfg 5 critical-path model and its kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -m gpu -x -v \
  --timeout 300 --timeout-method thread -k "range or shard or dist or gather or next_seed or whole_vs" > $O/pytest_r3m.log 2>&1 \
  || { tail -40 $O/pytest_r3m.log; exit 1; }
tail -3 $O/pytest_r3m.log
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r3m.json 2> $O/shard8_r3m.err || { tail -5 $O/shard8_r3m.err; exit 1; }
grep "^{" $O/shard8_r3m.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_shard_r3m -o run -- python $R/tools/shard_time_device.py 8 2 300 > /dev/null 2> $O/prof_shard_r3m.err || { tail -5 $O/prof_shard_r3m.err; exit 1; }
echo traced
