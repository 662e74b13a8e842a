#!/bin/bash
# Full GPU suite, smoke, bench, cfg 5 model (exact refinement on 256-thread
# blocks, seed-only tail octaves, padded-list merges).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_r3n.log 2>&1 \
  || { tail -40 $O/pytest_gpu_r3n.log; exit 1; }
tail -2 $O/pytest_gpu_r3n.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 300 python bench.py > $O/bench_r3n.json 2> $O/bench_r3n.err || { tail -5 $O/bench_r3n.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r3n.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['verified'])"
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r3n.json 2> $O/shard8_r3n.err || { tail -5 $O/shard8_r3n.err; exit 1; }
grep "^{" $O/shard8_r3n.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r3n_iso -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_r3n_iso.err || { tail -5 $O/prof_r3n_iso.err; exit 1; }
echo traced
