#!/bin/bash
# Isolated kernel traces of extrema-scan timing probes (build_var/<v>.so); the
# probes change results, so only the trace matters (bench output ignored).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "$@"; do
  SIFT_HIP_LIB=$R/build_var/$v.so timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/xp_$v -o run -- python $R/bench.py --steps 6 --warmup 2 --no-cpu-baseline --overlap none --inflight 2 > /dev/null 2> $O/xp_$v.err || { echo "variant $v failed"; tail -5 $O/xp_$v.err; exit 1; }
done
python3 $R/tools/gauss_oct.py $(for v in "$@"; do echo $O/xp_$v/run_kernel_trace.csv; done)
