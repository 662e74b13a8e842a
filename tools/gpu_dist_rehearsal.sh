#!/bin/bash
# The bench's collective paths on a one-GPU box: torchrun, world size 1,
# nccl (SIFT_BENCH_DIST=1), default mode and --shard-image, plus the RCCL tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > $O/t_dist.log 2>&1 || { echo "dist tests failed"; tail -20 $O/t_dist.log; exit 1; }
tail -1 $O/t_dist.log
SIFT_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_dist1.json 2> $O/bench_dist1.err || { echo "dist bench failed"; tail -20 $O/bench_dist1.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_dist1.json').read().strip().splitlines()[-1]); print('dist world1', d['value'], d['ms_per_step'], d['config']['parallelism'], 'sustained', d.get('sustained'))"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nodist.json 2> $O/bench_nodist.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench_nodist.json').read().strip().splitlines()[-1]); print('no dist', d['value'], d['ms_per_step'])"
SIFT_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 1 --shard-image --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_dist1_shard.json 2> $O/bench_dist1_shard.err || { echo "dist shard bench failed"; tail -20 $O/bench_dist1_shard.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_dist1_shard.json').read().strip().splitlines()[-1]); print('dist world1 shard', d['value'], d['ms_per_step'], d.get('parts_ms_per_step'))"
