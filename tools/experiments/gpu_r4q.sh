#!/bin/bash
# Exact patches from the split pass's vertical sums (SIFT_VSUM_EXACT), capture compiled out,
# pooled host buffers in the addon: full GPU suite, JS bench, A/B of the exact refinement.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_r4q.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest_r4q.log | tail -30; exit 1; }
grep -c PASSED $O/pytest_r4q.log; tail -n 1 $O/pytest_r4q.log
timeout -k 10 600 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_r4q.json > $O/js_bench_r4q.log 2>&1 || { tail -20 $O/js_bench_r4q.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/js_bench_r4q.json'))
for k in ['detect','detect_typed','detectAsync','detectAsync_typed_queued','detectAsync_objects_queued','detectAsync_typed_queued_inflight1']:
    v=d.get(k,{}); print(k, {x: (round(v[x],2) if isinstance(v.get(x),float) else v.get(x)) for x in ['wall_ms','ms_per_image','mpix_per_s','queued_mpix_per_s','keypoints','d2h_ms','h2d_ms']})
print('stages', round(d['stages']['total_ms'],1), 'ms', 'dog read GB/s', round(d['stages'].get('dog_stage_read_gb_per_s',0),2), {k: round(v,2) for k,v in d['stages'].items() if k.endswith('_ms')})"
STEPS=100 timeout -k 10 600 bash tools/gpu_ab_oct.sh 2 - "SIFT_HIP_LIB=$R/build_var/exp.so SIFT_VSUM_EXACT=0"
