#!/bin/bash
# Round artifacts on the GPU box: parity tests, smoke, bench line (with the
# CPU baseline), rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes.
# usage: tools/gpu_round.sh <tag>
TAG=${1:-round}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
if [ "${SKIP_PYTEST:-0}" != 1 ]; then  # SKIP_PYTEST=1: the tests ran in a call of their own
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu_$TAG.log; exit 1; }
tail -3 $O/pytest_gpu_$TAG.log
fi
echo "[$(date +%T)] smoke"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo smoke failed; tail -20 $O/smoke_$TAG.log; exit 1; }
cat $O/smoke_$TAG.log
echo "[$(date +%T)] bench"
timeout -k 10 300 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo bench failed; tail -5 $O/bench_$TAG.err; exit 1; }
cat $O/bench_$TAG.json
cd /tmp
echo "[$(date +%T)] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 > $O/bench_prof_$TAG.json 2> $O/prof_$TAG.err || { echo "trace failed"; tail -5 $O/prof_$TAG.err; exit 1; }
echo "[$(date +%T)] kernel trace, --overlap none (isolated kernels)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_iso -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > $O/bench_prof_${TAG}_iso.json 2> $O/prof_${TAG}_iso.err || { echo "trace failed"; tail -5 $O/prof_${TAG}_iso.err; exit 1; }
i=0
for C in FETCH_SIZE WRITE_SIZE "TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1)); N=(FETCH_SIZE WRITE_SIZE TA); N=${N[$((i-1))]}
  echo "[$(date +%T)] pmc $C"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$N -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sustain-s 0 > /dev/null 2> $O/pmc_${TAG}_$N.err || { echo "pmc $C failed"; tail -5 $O/pmc_${TAG}_$N.err; exit 1; }
done
echo "[$(date +%T)] pmc SQ instruction counts (optional)"
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_${TAG}_SQ -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sustain-s 0 > /dev/null 2> $O/pmc_${TAG}_SQ.err || { echo "pmc SQ failed (optional)"; tail -3 $O/pmc_${TAG}_SQ.err; }
echo "[$(date +%T)] done"
