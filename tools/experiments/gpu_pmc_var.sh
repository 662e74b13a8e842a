#!/bin/bash
# Counter passes for one library variant: tools/gpu_pmc_var.sh <variant> <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
V=$1; TAG=$2
mkdir -p $O
export TMPDIR=/tmp SIFT_HIP_LIB=$R/build_var/$V.so
cd /tmp
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${TAG}_$i -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2> $O/pmc_${TAG}_$i.err || { echo "pass $i failed"; tail -5 $O/pmc_${TAG}_$i.err; exit 1; }
  echo "pass $i ok"
done
