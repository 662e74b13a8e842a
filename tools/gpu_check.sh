#!/bin/bash
# On the GPU box: parity tests, smoke, bench line, kernel-trace profile.
# usage: tools/gpu_check.sh <tag> [pytest -k expr]
# Every GPU step has its own time limit; the first failure ends the script.
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
K=()
if [ -n "$2" ]; then K=(-k "$2"); fi
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${K[@]}" > $O/pytest_gpu_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
echo "[$(date +%T)] smoke"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -20 $O/smoke_$TAG.log; exit 1; }
cat $O/smoke_$TAG.log
echo "[$(date +%T)] bench"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail -5 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
echo "[$(date +%T)] rocprofv3 kernel trace"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_prof_$TAG.json 2> $O/prof_$TAG.err
rc=$?
echo "prof rc=$rc"
cat $O/bench_prof_$TAG.json
exit $rc
