#!/bin/bash
# r6a: stall breakdown of the pass kernels (isolated detections, one rocprofv3
# --pmc pass per counter group) + a default bench line on the same box.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 300 python bench.py > $O/r6a_bench.json 2> $O/r6a_bench.err || { echo bench failed; tail -5 $O/r6a_bench.err; exit 1; }
cat $O/r6a_bench.json
cd /tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
         "SQ_INSTS_BRANCH SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_IFETCH SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/stall_r6a_$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 1 > /dev/null 2> $O/stall_r6a_$i.err || { echo "pass $i failed"; tail -5 $O/stall_r6a_$i.err; [ $i -lt 5 ] && exit 1; }
  echo "pass $i ok"
done
echo done
