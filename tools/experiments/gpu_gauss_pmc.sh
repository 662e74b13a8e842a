#!/bin/bash
# Counter passes over the Gaussian kernels (short bench run each).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=$1; shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" "SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_WR SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$i -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > /dev/null 2> $O/pmc_${TAG}_$i.err || { echo "pass $i failed"; tail -5 $O/pmc_${TAG}_$i.err; exit 1; }
  echo "pass $i ok"
done
