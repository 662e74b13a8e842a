#!/bin/bash
# r6b: GPU suite on the shipping build, then an A/B of the pipelined streamed
# kernels on the experiments build (alternated, 2 reps):
#   "SIFT_RWP=0"                 round-5 kernels (octave 2 k_gauss_rw<24,true>, octave 3 split pass + tile kernel)
#   "SIFT_RWP=1 SIFT_RWP_BIG=0"  octave 2 on k_gauss_rwp<24>
#   "SIFT_RWP=1 SIFT_RWP_BIG=1"  ... and octave 3 on k_gauss_rwp<48, l64>
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r6b_pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/r6b_pytest_gpu.log; exit 1; }
tail -3 $O/r6b_pytest_gpu.log
for rep in 1 2; do
  i=0
  for e in "SIFT_RWP=0" "SIFT_RWP=1 SIFT_RWP_BIG=0" "SIFT_RWP=1 SIFT_RWP_BIG=1"; do
    i=$((i+1))
    env SIFT_HIP_LIB=$R/build_ab/${VAR:-exp2}.so $e timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu-baseline > $O/r6b_$i.json 2> $O/r6b_$i.err || { echo "bench '$e' failed"; tail -5 $O/r6b_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/r6b_$i.json')); r=d['roofline']; print('[$e]', d['value'], d['ms_per_step'], r['launch_ms'], r['frac'], [o['iso_ms'] for o in r['per_octave']], 'x', r['extrema_stage']['iso_ms'], 'ref', r['refine_stage']['iso_ms'], d['verified'])"
  done
done
