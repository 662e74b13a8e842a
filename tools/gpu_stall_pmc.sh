#!/bin/bash
# Stall / issue / memory-path counters of every kernel of the bench's
# detections, one rocprofv3 --pmc pass per counter group (hardware limits:
# 8 SQ, 2 TA, 4 TCP, 4 TCC per pass), for one setting:
#   tools/gpu_stall_pmc.sh <tag> "<VAR=val ...>"   ("-" = no extra env)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
TAG=$1; E=$2; [ "$E" = "-" ] && E=""
cd /tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  env $E timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/stall_${TAG}_$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0 > /dev/null 2> $O/stall_${TAG}_$i.err || { echo "pass $i failed"; tail -5 $O/stall_${TAG}_$i.err; exit 1; }
done
echo "$TAG ok"
