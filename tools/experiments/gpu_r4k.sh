#!/bin/bash
# JS front door: JS parity tests (pool, typed format), the JS bench at 4K; then the k_gauss_pc A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests/test_js.py tests/test_gpu_parity.py::test_foreign_dog_with_nonfinite_values tests/test_gpu_parity.py::test_foreign_dog_is_exact -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_js_r4k.log 2>&1 || { tail -30 $O/pytest_js_r4k.log; exit 1; }
tail -n 1 $O/pytest_js_r4k.log
timeout -k 10 600 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_r4k.json > $O/js_bench_r4k.log 2>&1 || { tail -20 $O/js_bench_r4k.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/js_bench_r4k.json'))
for k in ['detect','detect_typed','detectAsync','detectAsync_typed_queued','detectAsync_objects_queued','detectAsync_typed_queued_inflight1']:
    v=d.get(k,{}); print(k, {x: round(v[x],2) if isinstance(v.get(x),float) else v.get(x) for x in ['wall_ms','ms_per_image','mpix_per_s','queued_mpix_per_s','keypoints']})
print('stages', round(d['stages']['total_ms'],1), 'ms')"
bash tools/gpu_r4j.sh
