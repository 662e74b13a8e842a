#!/bin/bash
# phased vs octave0 schedules (bench.py --overlap), a few in-flight depths
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "phased or async" > $O/pt_phased.log 2>&1 || { echo "tests failed"; tail -20 $O/pt_phased.log; exit 1; }
tail -1 $O/pt_phased.log
for m in octave0:3 phased:3 phased:4 octave0:3 phased:3; do
  mode=${m%%:*}; n=${m##*:}
  timeout -k 10 200 python $R/bench.py --steps 60 --warmup 6 --no-cpu-baseline --overlap $mode --inflight $n > $O/ph_${mode}_$n.json 2> $O/ph_${mode}_$n.err || { echo "mode $m failed"; tail -5 $O/ph_${mode}_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/ph_${mode}_$n.json')); print('$m', d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"
done
