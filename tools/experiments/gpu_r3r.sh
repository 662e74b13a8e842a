#!/bin/bash
# Exact refinement: one wave per patch for whole images, 256 threads for tail pieces.
# Full GPU suite, pipelined A/B against the one-wave build, cfg 5 model.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu_r3r.log 2>&1 \
  || { tail -40 $O/pytest_gpu_r3r.log; exit 1; }
tail -1 $O/pytest_gpu_r3r.log
for rep in 1 2; do bash tools/gpu_libab.sh - build_var/rt64.so || exit 1; done
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r3r.json 2> $O/shard8_r3r.err || { tail -5 $O/shard8_r3r.err; exit 1; }
grep "^{" $O/shard8_r3r.json
