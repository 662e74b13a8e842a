#!/bin/bash
# cfg 5 critical-path model (band keypoint gather beside the tails), then a
# kernel trace of the same run for the tail pieces' gaps.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r3l.json 2> $O/shard8_r3l.err || { tail -5 $O/shard8_r3l.err; exit 1; }
grep "^{" $O/shard8_r3l.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_shard_r3l -o run -- python $R/tools/shard_time_device.py 8 2 300 > /dev/null 2> $O/prof_shard_r3l.err || { tail -5 $O/prof_shard_r3l.err; exit 1; }
echo traced
