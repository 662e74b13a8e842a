#!/bin/bash
# On the GPU box: bench line + rocprofv3 kernel-trace stats + PMC passes.
# usage: tools/gpu_bench_profile.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-run}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
echo "[$(date +%T)] bench" 
timeout -k 10 400 python bench.py --steps 20 --warmup 3 "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail -20 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
echo "[$(date +%T)] kernel trace"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/bench_prof_$TAG.json 2> $O/prof_$TAG.err || { echo prof failed; tail -20 $O/prof_$TAG.err; exit 1; }
echo "[$(date +%T)] pmc FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmcf_$TAG -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $O/pmcf_$TAG.err || { echo pmc fetch failed; tail -20 $O/pmcf_$TAG.err; exit 1; }
echo "[$(date +%T)] pmc WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmcw_$TAG -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $O/pmcw_$TAG.err || { echo pmc write failed; tail -20 $O/pmcw_$TAG.err; exit 1; }
echo "[$(date +%T)] done"
find $O -name "*stats*.csv" | head
