#!/bin/bash
# Registered result buffers (ABI 8): ABI + JS tests, plane readback probe, JS bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_js.py tests/test_abi.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "js or abi or plane or stage or golden" > $O/pytest_r4ak.log 2>&1 || { tail -30 $O/pytest_r4ak.log; exit 1; }
tail -n 1 $O/pytest_r4ak.log
timeout -k 10 200 python tools/plane_d2h_probe.py > $O/plane_probe_r4ak.json 2>&1 || { tail -5 $O/plane_probe_r4ak.json; exit 1; }
cat $O/plane_probe_r4ak.json
timeout -k 10 600 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_r4ak.json > $O/js_bench_r4ak.log 2>&1 || { tail -20 $O/js_bench_r4ak.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/js_bench_r4ak.json'))
for k in ['detect','detect_typed','detectAsync_typed_queued']:
    v=d.get(k,{}); print(k, {x: (round(v[x],2) if isinstance(v.get(x),float) else v.get(x)) for x in ['wall_ms','ms_per_image','mpix_per_s','keypoints'] if x in v})
s=d['stages']; print('stages', {k:(round(v,2) if isinstance(v,float) else v) for k,v in s.items() if k!='what'})"
