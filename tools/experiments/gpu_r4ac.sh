#!/bin/bash
# JS front door with huge-page pool buffers: JS parity tests, then the JS bench at 4K.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_js.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_js_r4ac.log 2>&1 || { tail -30 $O/pytest_js_r4ac.log; exit 1; }
tail -n 1 $O/pytest_js_r4ac.log
cat /sys/kernel/mm/transparent_hugepage/enabled 2>/dev/null
timeout -k 10 600 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_r4ac.json > $O/js_bench_r4ac.log 2>&1 || { tail -20 $O/js_bench_r4ac.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/js_bench_r4ac.json'))
for k in ['detect','detect_typed','detectAsync','detectAsync_typed_queued','detectAsync_objects_queued']:
    v=d.get(k,{}); print(k, {x: (round(v[x],2) if isinstance(v.get(x),float) else v.get(x)) for x in ['wall_ms','ms_per_image','mpix_per_s','queued_mpix_per_s','keypoints'] if x in v})
s=d['stages']; print('stages', {k:(round(v,2) if isinstance(v,float) else v) for k,v in s.items() if k!='what'})"
