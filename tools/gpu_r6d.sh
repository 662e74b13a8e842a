#!/bin/bash
# r6d: which TCC (L2) request counters gfx950 exposes, then the refinement's L2->memory read requests by size
# (FETCH_SIZE's 2x correction was calibrated on wide streaming reads; k_refine_fast gathers 12-byte segments).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/r6d_counters.txt 2>&1 || true
grep -o 'TCC_EA0_RD[A-Z0-9_]*\|TCC_EA0_WR[A-Z0-9_]*\|TCC_REQ\b\|TCC_READ\b\|TCC_BUBBLE\b\|TCC_EA0_RDREQ_DRAM[A-Z0-9_]*' $O/r6d_counters.txt | sort -u > $O/r6d_tcc.txt || true
cat $O/r6d_tcc.txt
i=0
for C in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum GRBM_GUI_ACTIVE" "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/stall_r6d_$i -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 1 > /dev/null 2> $O/stall_r6d_$i.err && echo "pass $i ok" || { echo "pass $i failed"; tail -3 $O/stall_r6d_$i.err; }
done
