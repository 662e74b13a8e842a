#!/bin/bash
# Scan loop without back-edge load drains (x_settle) + k_gauss_vert prefetch through the loop-top copy:
# parity subset on the product library, then A/B against xs0 (neither) and kernel traces of both.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or unaligned or cfg5_radii or detect_matches_reference or range_detection or saturated or reference_itself or nonfinite or exact" \
  > $O/pytest_r4z.log 2>&1 || { grep -E "PASS|FAIL|Error|passed|failed|assert" $O/pytest_r4z.log | tail -30; exit 1; }
tail -n 1 $O/pytest_r4z.log
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 "SIFT_HSP=0 SIFT_HIP_LIB=$R/build_var/xs0.so" "SIFT_HSP=0 SIFT_HIP_LIB=$R/build_var/exp.so" "SIFT_HSP=1 SIFT_HIP_LIB=$R/build_var/exp.so" || exit 1
export TMPDIR=/tmp; cd /tmp || exit 1
i=0
for L in xs0 exp; do export SIFT_HSP=$([ $L = exp ] && echo 1 || echo 0)
  i=$((i+1))
  SIFT_HIP_LIB=$R/build_var/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4z_$L -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > $O/bench_r4z_$L.json 2> $O/prof_r4z_$L.err || { echo "trace $L failed"; tail -5 $O/prof_r4z_$L.err; exit 1; }
done
echo done
