#!/bin/bash
# Round 3, call d: full GPU suite (incl. batch tests), cfg4 batched vs per-image,
# JS drop-in bench, stage-API extrema probe, cfg5 shard model + trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
if [ "${SKIP_PYTEST:-0}" != 1 ]; then
echo "[$(date +%T)] pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_r3d.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_r3d.log | head -30; tail -30 $O/pytest_r3d.log; exit 1; }
tail -1 $O/pytest_r3d.log
fi
if [ "${SKIP_CFG4:-0}" != 1 ]; then
echo "[$(date +%T)] cfg4: 1080p x 8 per GPU"
for a in "--batch-mode launch" "--batch-mode launch --inflight 2" "--batch-mode launch --inflight 4" "--batch-mode images" "--batch-mode images --inflight 4"; do
  timeout -k 10 200 python bench.py --width 1920 --height 1080 --batch 8 --steps 30 --warmup 5 --no-cpu-baseline --sustain-s 0 $a > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 $a failed"; tail -5 $O/cfg4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cfg4.json')); r=d['roofline']; print('[$a]', d['value'], d['ms_per_step'], 'pass', r['launch_ms'], round(r['frac'],3), [round(o['iso_ms'],4) for o in r['per_octave']], 'verified', d['verified'])"
  cp $O/cfg4.json "$O/cfg4_$(echo $a | tr ' -' '__').json"
done
fi
echo "[$(date +%T)] strip-ordered refinement: parity subset, then A/B"
SIFT_HIP_LIB=$R/build_var/exp3.so SIFT_REFINE_STRIP=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cfg3 or golden or reference_itself or batch" > $O/pytest_strip.log 2>&1 || { echo "pytest strip failed"; tail -30 $O/pytest_strip.log; exit 1; }
tail -1 $O/pytest_strip.log
for e in "-" "SIFT_REFINE_STRIP=4" "SIFT_REFINE_STRIP=2" "SIFT_REFINE_STRIP=1" "-" "SIFT_REFINE_STRIP=4"; do
  ee=$e; [ "$e" = "-" ] && ee=""
  env SIFT_HIP_LIB=$R/build_var/exp3.so $ee timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/strip.json 2> $O/strip.err || { echo "strip $e failed"; tail -5 $O/strip.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/strip.json')); print('[$e]', d['value'], d['ms_per_step'], d['stages_ms'], d['verified'])"
done
cd /tmp && export TMPDIR=/tmp
for e in "SIFT_REFINE_STRIP=0" "SIFT_REFINE_STRIP=4"; do
  env SIFT_HIP_LIB=$R/build_var/exp3.so $e timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_strip_$e -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sustain-s 0 > /dev/null 2> $O/pmc_strip.err || { echo "pmc strip failed"; tail -5 $O/pmc_strip.err; exit 1; }
  env SIFT_HIP_LIB=$R/build_var/exp3.so $e timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_strip_$e -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_strip.err || { echo "trace strip failed"; tail -5 $O/prof_strip.err; exit 1; }
done
cd $R
echo "[$(date +%T)] JS drop-in bench (4K)"
timeout -k 10 300 python tools/js_bench/bench_js.py --reps 10 --out $O/js_bench_4k.json > $O/js_bench_4k.log 2>&1 || { echo "js bench failed"; tail -20 $O/js_bench_4k.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/js_bench_4k.json')); print({k: d[k] for k in ('detect','detectAsync','stages')})"
echo "[$(date +%T)] stage-API extrema probe"
timeout -k 10 200 python tools/stage_probe.py > $O/stage_probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/stage_probe.txt; exit 1; }
cat $O/stage_probe.txt
echo "[$(date +%T)] cfg5 shard model (8 shards)"
timeout -k 10 300 python tools/shard_time_device.py 8 5 > $O/shard8.json 2> $O/shard8.err || { echo "shard timer failed"; tail -20 $O/shard8.err; exit 1; }
cat $O/shard8.json
cd /tmp && export TMPDIR=/tmp
echo "[$(date +%T)] traces"
timeout -k 10 200 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $O/prof_stage -o run -- python3 $R/tools/stage_probe.py > $O/stage_probe_prof.txt 2>&1 || { echo "probe trace failed"; tail -5 $O/stage_probe_prof.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_shard8 -o run -- python3 $R/tools/shard_time_device.py 8 2 > /dev/null 2> $O/prof_shard8.err || { echo "shard trace failed"; tail -5 $O/prof_shard8.err; exit 1; }
echo "[$(date +%T)] done"
