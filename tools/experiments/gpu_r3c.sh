#!/bin/bash
# Full GPU suite on the default build, then A/B: previous build (exp.so) vs
# the new one (exp2.so: generic vertical interior path, 16-row split pass),
# and the split pass from radius 20 (octave 2) on the new one.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r3c.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_r3c.log; exit 1; }
tail -1 $O/pytest_r3c.log
tools/gpu_ab_oct.sh 2 "SIFT_HIP_LIB=$R/build_var/exp.so" "SIFT_HIP_LIB=$R/build_var/exp2.so" "SIFT_HIP_LIB=$R/build_var/exp2.so SIFT_VSPLIT_R=20" || exit 1
echo "[$(date +%T)] JS drop-in bench (4K)"
timeout -k 10 300 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_4k.json > $O/js_bench_4k.log 2>&1 || { echo "js bench failed"; tail -20 $O/js_bench_4k.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/js_bench_4k.json')); print({k: d[k] for k in ('detect','detectAsync','stages')})"
echo "[$(date +%T)] stage-API extrema probe"
timeout -k 10 200 python tools/stage_probe.py > $O/stage_probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/stage_probe.txt; exit 1; }
cat $O/stage_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof_stage -o run -- python3 $R/tools/stage_probe.py > $O/stage_probe_prof.txt 2>&1 || { echo "probe trace failed"; tail -5 $O/stage_probe_prof.txt; exit 1; }
echo done
cd $R
echo "[$(date +%T)] cfg5 shard model (8 shards) + trace"
timeout -k 10 300 python tools/shard_time_device.py 8 5 > $O/shard8.json 2> $O/shard8.err || { echo "shard timer failed"; tail -20 $O/shard8.err; exit 1; }
cat $O/shard8.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof_shard8 -o run -- python3 $R/tools/shard_time_device.py 8 2 > /dev/null 2> $O/prof_shard8.err || { echo "shard trace failed"; tail -5 $O/prof_shard8.err; exit 1; }
echo done2
cd $R
echo "[$(date +%T)] cfg4 shape: 1080p x 8 per GPU, in-flight depth / overlap"
for a in "--inflight 3" "--inflight 4" "--inflight 6" "--inflight 4 --overlap none" "--inflight 8 --overlap none"; do
  timeout -k 10 200 python bench.py --width 1920 --height 1080 --batch 8 --steps 30 --warmup 5 --no-cpu-baseline --sustain-s 0 $a > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 $a failed"; tail -5 $O/cfg4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg4.json')); print('[$a]', d['value'], d['ms_per_step'], round(d['roofline']['frac'],3))"
done
