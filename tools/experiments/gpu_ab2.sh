#!/bin/bash
# A/B of library variants: isolated kernel trace + pipelined bench value per variant.
# usage: tools/gpu_ab2.sh <variant>...   (build_var/<variant>.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  SIFT_HIP_LIB=$R/build_var/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/ab2_$v -o run -- python $R/bench.py --steps 8 --warmup 2 --no-cpu-baseline --overlap none --inflight 2 > $O/ab2_$v.iso.json 2> $O/ab2_$v.err || { echo "variant $v trace failed"; tail -5 $O/ab2_$v.err; exit 1; }
  SIFT_HIP_LIB=$R/build_var/$v.so timeout -k 10 200 python $R/bench.py --steps 60 --warmup 6 --no-cpu-baseline > $O/ab2_$v.json 2>> $O/ab2_$v.err || { echo "variant $v bench failed"; tail -5 $O/ab2_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/ab2_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
python3 $R/tools/gauss_oct.py $(for v in "$@"; do echo $O/ab2_$v/run_kernel_trace.csv; done)
