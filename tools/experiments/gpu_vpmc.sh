#!/bin/bash
# Memory-path counters of the Gaussian kernels under SIFT_GAUSS_DBG settings:
# tools/gpu_vpmc.sh <setting>...
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
C="TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for v in "$@"; do
  SIFT_GAUSS_DBG=$v timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/vpmc_$v -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/vpmc_$v.err || { echo "setting $v failed"; tail -5 $O/vpmc_$v.err; exit 1; }
  echo "setting $v ok"
done
