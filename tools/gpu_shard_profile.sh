#!/bin/bash
# cfg 5 artifacts: per-rank critical path of the 8K row-band shards (2/4/8),
# one GPU running the shards in turn, and the bench's --shard-image line at N=1.
# usage: tools/gpu_shard_profile.sh <tag>
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
for n in 8 4 2; do
  timeout -k 10 200 python tools/shard_time_device.py $n 5 > $O/shard${n}_$TAG.json 2> $O/shard${n}_$TAG.err || { echo "shard $n failed"; tail -5 $O/shard${n}_$TAG.err; exit 1; }
done
timeout -k 10 200 python bench.py --shard-image --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_shard_$TAG.json 2> $O/bench_shard_$TAG.err || { echo "shard bench failed"; tail -5 $O/bench_shard_$TAG.err; exit 1; }
echo shard done
