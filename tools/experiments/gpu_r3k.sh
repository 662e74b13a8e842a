#!/bin/bash
# 8K O6 S5 against the oracle in all three summation orders (the reference's
# 2D order included), the 4K configuration tests, the saturated-image test,
# then the bench.  A heartbeat line every 30 s while the oracle runs.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
( s=0; while sleep 30; do s=$((s+30)); echo "[heartbeat] ${s}s"; done ) & HB=$!
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dist.py -m gpu -x -v -s --timeout 900 --timeout-method thread \
  -k "cfg5_8k or cfg3_4k or saturated or dist or shard or gather" > $O/pytest_r3k.log 2>&1; rc=$?
kill $HB
grep -E "PASS|FAIL|Error|low-contrast:|oracle \(|passed|failed" $O/pytest_r3k.log
[ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py > $O/bench_r3k.json 2> $O/bench_r3k.err || { tail -5 $O/bench_r3k.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r3k.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['roofline']['extrema_stage'])"
