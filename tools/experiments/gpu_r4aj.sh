#!/bin/bash
# cfg 5 on the round-4 build: merge / shard parity tests, then the 8-shard device model (tools/shard_time_device.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "merge or shard or row_band or cfg5 or dist" \
  > $O/pytest_r4aj.log 2>&1 || { grep -E "passed|failed|assert|Error" $O/pytest_r4aj.log | tail -10; exit 1; }
tail -n 1 $O/pytest_r4aj.log
timeout -k 10 400 python tools/shard_time_device.py 8 5 300 > $O/shard8_r4aj.json 2> $O/shard8_r4aj.err || { tail -5 $O/shard8_r4aj.err; exit 1; }
grep "^{" $O/shard8_r4aj.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ['whole_ms','shard_ms','tail_octave_ms','merge_ms','critical_path_ms','critical_path_serial_gathers_ms','speedup_vs_whole','identical']})"
