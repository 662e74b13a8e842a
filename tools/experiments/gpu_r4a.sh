#!/bin/bash
# Round-4 baseline on a fresh box: bench line with per-octave isolated pass times, isolated kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --sustain-s 0 > $O/r4a_bench.json 2> $O/r4a_bench.err || { tail -5 $O/r4a_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/r4a_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], 'pass', r['launch_ms'], round(r['frac'],3), [round(o['iso_ms'],4) for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'])"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4a_iso -o run -- python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > $O/bench_prof_r4a_iso.json 2> $O/prof_r4a_iso.err || { echo "trace failed"; tail -5 $O/prof_r4a_iso.err; exit 1; }
echo done
