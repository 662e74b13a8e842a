#!/bin/bash
# A/B timing of library variants: kernel trace per variant (bench, 5 steps).
# usage: tools/gpu_ab.sh <variant>...   (build_var/<variant>.so)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  SIFT_HIP_LIB=$R/build_var/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/ab_$v -o run -- python $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $O/ab_$v.json 2> $O/ab_$v.err || { echo "variant $v failed"; tail -5 $O/ab_$v.err; exit 1; }
  echo "variant $v ok"
done
