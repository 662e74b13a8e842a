set -e
for v in "SIFT_FUSE=0" "SIFT_FUSE=1" "SIFT_FUSE=1 SIFT_GAUSS_DBG=2" "SIFT_FUSE=0 SIFT_GAUSS_DBG=1" "SIFT_FUSE=1 SIFT_GAUSS_DBG=3"; do
  env $v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap none --inflight 2 > gpurun_out/ab.json 2>/dev/null
  python3 -c "
import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);r=d['roofline']
print('$v', d['value'], 'oct0 iso', r['octave0']['iso_ms'], 'extrema iso', r['extrema_stage']['iso_ms'])"
done
