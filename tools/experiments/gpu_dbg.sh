#!/bin/bash
# Kernel traces of the bench under SIFT_GAUSS_DBG probe settings:
# tools/gpu_dbg.sh <setting>...   (bit 1 no stores, 2 no vertical, 4 no horizontal pass)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  SIFT_GAUSS_DBG=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/dbg_$v -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/dbg_$v.json 2> $O/dbg_$v.err || { echo "setting $v failed"; tail -5 $O/dbg_$v.err; exit 1; }
  echo "setting $v ok"
done
