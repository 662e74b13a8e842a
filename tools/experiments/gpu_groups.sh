#!/bin/bash
# Kernel trace of the isolated bench per SIFT_GAUSS_GROUPS setting.
# usage: tools/gpu_groups.sh <groups>...   ("def" = built-in choice; "1,4,4" = octaves 1..3)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for g in "$@"; do
  t=grp_${g//,/_}
  if [ "$g" = def ]; then unset SIFT_GAUSS_GROUPS; else export SIFT_GAUSS_GROUPS=$g; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$t -o run -- python $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --overlap none --inflight 2 > $O/$t.json 2> $O/$t.err || { echo "groups $g failed"; tail -5 $O/$t.err; exit 1; }
done
unset SIFT_GAUSS_GROUPS
python3 $R/tools/gauss_oct.py $(for g in "$@"; do echo $O/grp_${g//,/_}/run_kernel_trace.csv; done)
