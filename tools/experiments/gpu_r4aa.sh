#!/bin/bash
# k_gauss_vert (4K octave 3) timed per scale: SIFT_VERT_ONLY=s runs only scale s's blocks (timing only).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp; cd /tmp || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so SIFT_HSP=0
for V in -1 7 6 4 1; do
  SIFT_VERT_ONLY=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4aa_$V -o run -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_r4aa_$V.err || { echo "trace $V failed"; tail -5 $O/prof_r4aa_$V.err; exit 1; }
done
echo done
