#!/bin/bash
# Kernel traces (isolated detections) of the split-octave variants: ch8 + tile kernel, CH16 + tile kernel, CH16 + k_gauss_hsp.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp || exit 1
i=0
for E in "SIFT_HSP=0 SIFT_HIP_LIB=$R/build_var/ch8.so" "SIFT_HSP=0 SIFT_HIP_LIB=$R/build_var/exp.so" "SIFT_HSP=1 SIFT_HIP_LIB=$R/build_var/exp.so"; do
  i=$((i+1))
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4x_$i -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > $O/bench_r4x_$i.json 2> $O/prof_r4x_$i.err || { echo "trace $i failed"; tail -5 $O/prof_r4x_$i.err; exit 1; }
done
echo done
