#!/bin/bash
# On the GPU box: parity tests, bench line, kernel-trace profile.
# usage: tools/gpu_check.sh <tag> [pytest -k expr]
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
timeout -k 10 400 python -m pytest tests -m gpu -q "${K[@]}" > $O/pytest_gpu_$TAG.log 2>&1
echo "pytest rc=$?"; tail -8 $O/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail -5 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2> $O/prof_$TAG.err
echo "prof rc=$?"
