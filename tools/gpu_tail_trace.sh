#!/bin/bash
# cfg 5 critical-path model on the current build, then a kernel trace of the
# same run (tail pieces' kernels and gaps: tools/experiments/tail_gaps.py, run here on the CPU).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r5ai.json 2> $O/shard8_r5ai.err || { tail -5 $O/shard8_r5ai.err; exit 1; }
grep "^{" $O/shard8_r5ai.json | cut -c1-300
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/prof_shard_r5ai -o run -- python $R/tools/shard_time_device.py 8 2 300 > /dev/null 2> $O/prof_shard_r5ai.err || { tail -5 $O/prof_shard_r5ai.err; exit 1; }
echo traced
