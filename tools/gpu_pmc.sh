#!/bin/bash
# On the GPU box: PMC counter passes over a short bench run (one pass per group).
# usage: tools/gpu_pmc.sh <tag> "<counters pass 1>" "<counters pass 2>" ... [-- extra bench args]
TAG=$1; shift
PASSES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do PASSES+=("$1"); shift; done
[ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for C in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$i -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $O/pmc_${TAG}_$i.err || { echo "pass $i failed"; tail -5 $O/pmc_${TAG}_$i.err; exit 1; }
  echo "pass $i ok: $C"
done
