#!/bin/bash
# r6e: refinement gather order / in-flight window: band rows (build constant) and blocks per CU (SIFT_REFINE_LDS),
# bench + one PMC pass each (L2->fabric read requests, the DRAM share, L2 hits) for k_refine_fast.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
run() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env SIFT_HIP_LIB=$R/build_ab/$lib.so "$@" timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/r6e_$tag.json 2> $O/r6e_$tag.err || { echo "bench $tag failed"; tail -5 $O/r6e_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/r6e_$tag.json')); r=d['roofline']; print('$tag', d['value'], d['ms_per_step'], 'pass', r['launch_ms'], 'x', r['extrema_stage']['iso_ms'], 'ref', r['refine_stage']['iso_ms'], d['verified'])"
  (cd /tmp && env SIFT_HIP_LIB=$R/build_ab/$lib.so "$@" timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/stall_r6e_$tag -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 1 > /dev/null 2> $O/stall_r6e_$tag.err) || { echo "pmc $tag failed"; tail -3 $O/stall_r6e_$tag.err; return 1; }
}
for rep in 1 2; do
  run b16 exp3 || exit 1
  run b4 br4 || exit 1
  run b64 br64 || exit 1
  run b16lds exp3 SIFT_REFINE_LDS=60000 || exit 1
  run nob exp3 SIFT_BAND_ORDER=0 || exit 1
done
