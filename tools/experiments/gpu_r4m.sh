#!/bin/bash
# NaN-propagating scan (no -fno-honor-nans): non-finite foreign DoG + JS tests, JS bench, bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_js.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_r4m.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest_r4m.log | tail -30; exit 1; }
grep -c PASSED $O/pytest_r4m.log; tail -n 1 $O/pytest_r4m.log
timeout -k 10 600 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_r4m.json > $O/js_bench_r4m.log 2>&1 || { tail -20 $O/js_bench_r4m.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/js_bench_r4m.json'))
for k in ['detect','detect_typed','detectAsync','detectAsync_typed_queued','detectAsync_objects_queued','detectAsync_typed_queued_inflight1']:
    v=d.get(k,{}); print(k, {x: (round(v[x],2) if isinstance(v.get(x),float) else v.get(x)) for x in ['wall_ms','ms_per_image','mpix_per_s','queued_mpix_per_s','keypoints']})
print('stages', round(d['stages']['total_ms'],1), 'ms')"
STEPS=100 timeout -k 10 300 bash tools/gpu_ab_oct.sh 2 -
