#!/bin/bash
# r6c: scale groups / tile counts of the pipelined streamed kernels (experiments build), then stall counters of
# k_gauss_rwp<24> and k_gauss_rwp<48,l64> (one rocprofv3 --pmc pass per counter group).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
LIB=$R/build_ab/${VAR:-exp2}.so
for rep in 1 2; do
  i=0
  for e in "SIFT_RWP=0" "SIFT_RWP=1 SIFT_RWP_BIG=1" "SIFT_RWP=1 SIFT_RWP_BIG=1 SIFT_RW_MINB=1400" "SIFT_RWP=1 SIFT_RWP_BIG=1 SIFT_RW_MINB=1" "SIFT_RWP=1 SIFT_RWP_BIG=0 SIFT_RWS=3"; do
    i=$((i+1))
    env SIFT_HIP_LIB=$LIB $e timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/r6c_$i.json 2> $O/r6c_$i.err || { echo "bench '$e' failed"; tail -5 $O/r6c_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r6c_$i.json')); r=d['roofline']; print('[$e]', d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], [o['iso_ms'] for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'], 'ref', r['refine_stage']['iso_ms'], d['verified'])"
  done
done
cd /tmp
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU GRBM_GUI_ACTIVE" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  SIFT_HIP_LIB=$LIB SIFT_RWP=1 SIFT_RWP_BIG=1 timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/stall_r6c_$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 1 > /dev/null 2> $O/stall_r6c_$i.err || { echo "pass $i failed"; tail -5 $O/stall_r6c_$i.err; exit 1; }
  echo "pass $i ok"
done
