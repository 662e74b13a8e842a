#!/bin/bash
# Split pass on the matrix cores (k_gauss_vert_mfma): parity subset on the product library (planes bit-exact in GPU
# order incl. radii up to 188, 8K, the 4K reference itself), then A/B with the VALU split pass and kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or cfg5 or range_detection or saturated or reference_itself or exact" \
  > $O/pytest_r4af.log 2>&1 || { grep -E "PASS|FAIL|Error|passed|failed|assert" $O/pytest_r4af.log | tail -30; exit 1; }
tail -n 1 $O/pytest_r4af.log
export SIFT_HIP_LIB=$R/build_var/exp.so
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 SIFT_VERT_MFMA=0 SIFT_VERT_MFMA=1 || exit 1
export TMPDIR=/tmp; cd /tmp || exit 1
for V in 0 1; do
  SIFT_VERT_MFMA=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4af_$V -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_r4af_$V.err || { echo "trace $V failed"; tail -5 $O/prof_r4af_$V.err; exit 1; }
  SIFT_VERT_MFMA=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4af8k_$V -o run -- python $R/bench.py --width 7680 --height 4320 --octaves 6 --steps 5 --warmup 2 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > $O/bench_r4af8k_$V.json 2> $O/prof_r4af8k_$V.err || { echo "trace8k $V failed"; tail -5 $O/prof_r4af8k_$V.err; exit 1; }
done
echo done
