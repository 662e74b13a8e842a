#!/bin/bash
# r6o: the JS drop-in bench on the round-6 build (4K and 1080p, one run each), plus the JS suite.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 400 python tools/js_bench/bench_js.py --out $O/r6o_js_bench_4k.json > $O/r6o_js_4k.log 2>&1 || { echo "js 4k failed"; tail -20 $O/r6o_js_4k.log; exit 1; }
timeout -k 10 300 python tools/js_bench/bench_js.py --width 1920 --height 1080 --out $O/r6o_js_bench_1080p.json > $O/r6o_js_1080p.log 2>&1 || { echo "js 1080p failed"; tail -20 $O/r6o_js_1080p.log; exit 1; }
tail -2 $O/r6o_js_4k.log $O/r6o_js_1080p.log
