#!/bin/bash
# Where the fused octave-0 extrema cost goes: isolated octave-0 and extrema
# stage times with the decisions / stores switched off (SIFT_GAUSS_DBG bits).
for v in "SIFT_FUSE=0" "SIFT_FUSE=1" "SIFT_FUSE=1 SIFT_GAUSS_DBG=2" "SIFT_FUSE=1 SIFT_GAUSS_DBG=1" "SIFT_FUSE=0 SIFT_GAUSS_DBG=1"; do
  env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap none --inflight 2 > gpurun_out/ab.json 2>/dev/null || { echo "$v failed"; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$v', d['value'], 'oct0 iso', r['octave0']['iso_ms'], 'extrema iso', r['extrema_stage']['iso_ms'])"
done
