#!/bin/bash
# Extrema scan XCD banding A/B (isolated kernels + pipelined bench) and the
# Infinity-Cache residency probe.  usage: tools/gpu_xcd_mall.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R || exit 1
timeout -k 10 200 python tools/mall_probe.py > $O/mall_probe.txt 2>&1 || { echo "mall probe failed"; tail -20 $O/mall_probe.txt; exit 1; }
cat $O/mall_probe.txt
for X in 0 1; do
  cd /tmp
  SIFT_XXCD=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_xxcd$X -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap none --inflight 2 > $O/bench_xxcd${X}_iso.json 2> $O/prof_xxcd$X.err || { echo "trace failed"; tail -5 $O/prof_xxcd$X.err; exit 1; }
  grep -E "k_extrema|k_refine_fast" $O/prof_xxcd$X/run_kernel_stats.csv | cut -d, -f1-4
  SIFT_XXCD=$X timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_xxcd$X -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/pmc_xxcd$X.err || { echo "pmc failed"; tail -5 $O/pmc_xxcd$X.err; exit 1; }
done
cd $R
bash tools/gpu_envab.sh 2 SIFT_XXCD=0 SIFT_XXCD=1
