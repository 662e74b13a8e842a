#!/bin/bash
# Register-window octave 1 with the vertical pass on the matrix cores (k_gauss_mx, SIFT_MX=1, experiments build):
# parity subset under the knob, then A/B with k_gauss_rw and kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
export SIFT_HIP_LIB=$R/build_var/exp.so
SIFT_MX=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread \
  -k "planes_bit_exact or large_radii or batch or row_band or degenerate or unaligned or range_detection or saturated or reference_itself or detect_matches_reference" \
  > $O/pytest_r4ag.log 2>&1 || { grep -E "PASS|FAIL|Error|passed|failed|assert" $O/pytest_r4ag.log | tail -30; exit 1; }
tail -n 1 $O/pytest_r4ag.log
STEPS=40 timeout -k 10 900 bash tools/gpu_ab_oct.sh 2 SIFT_MX=0 SIFT_MX=1 "SIFT_MX=1 SIFT_GAUSS_DBG=1" || exit 1
export TMPDIR=/tmp; cd /tmp || exit 1
for V in 0 1; do
  SIFT_MX=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_r4ag_$V -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --sustain-s 0 --overlap none --inflight 2 > /dev/null 2> $O/prof_r4ag_$V.err || { echo "trace $V failed"; tail -5 $O/prof_r4ag_$V.err; exit 1; }
done
echo done
