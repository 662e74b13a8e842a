#!/usr/bin/env python3
"""cfg 5 (8K, O=6, S=5) on one GPU, device-resident: whole-image detection
(input in HBM, keypoints left in HBM) vs the same image as n row-band shards
run in turn through sift_amd.shard.detect_sharded_device_local, with per-part
times -- the critical path n devices would see is the slowest rank (its band
+ the tail octave it detects) + the merge (plus two all-gathers, not timed
here).
usage: tools/shard_time_device.py [n_shards] [reps]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd import shard  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W, H, O, S = 7680, 4320, 6, 5
img = blob_image(W, H, seed=42)
d_img = torch.from_numpy(img).to("cuda:0")
p = sift_amd.make_params(O, S)
ctx = sift_amd.Context(0)
n_whole = ctx.detect_device(d_img.data_ptr(), W, H, p)
whole = ctx.keypoints().tobytes()
t_whole = []
for _ in range(reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.detect_device(d_img.data_ptr(), W, H, p)
    t_whole.append(time.perf_counter() - t0)
merged, plan = shard.detect_sharded_device_local(ctx, d_img, p, n)  # warm-up
same = merged.cpu().numpy().tobytes() == whole
timers = []
for _ in range(reps):
    tm = {}
    shard.detect_sharded_device_local(ctx, d_img, p, n, timer=tm)
    timers.append(tm)
keys = timers[0].keys()
med = {k: float(np.median([t[k] for t in timers])) * 1e3 for k in keys}
shards = [med["shard%d" % r] for r in range(len(plan.bands))]
tails = {t: med["tail%d" % t] for t in shard.tail_octaves(plan, len(plan.bands))}
owner = shard.tail_octaves(plan, len(plan.bands))
per_rank = [shards[r] + sum(v for t, v in tails.items() if owner[t] == r) for r in range(len(plan.bands))]
crit = max(per_rank) + med["merge"]
print(json.dumps({"config": "8K 7680x4320 O6 S5, device-resident (image in HBM, keypoints in HBM)",
                  "n_shards": n, "K": plan.K, "bands": plan.bands, "crops": plan.crops,
                  "whole_ms": round(1e3 * float(np.median(t_whole)), 3),
                  "shard_ms": [round(x, 3) for x in shards],
                  "tail_octave_ms": {str(t): round(v, 3) for t, v in tails.items()},
                  "tail_owner": {str(t): r for t, r in owner.items()},
                  "per_rank_ms": [round(x, 3) for x in per_rank],
                  "merge_ms": round(med["merge"], 3),
                  "critical_path_ms": round(crit, 3),
                  "critical_path_note": "slowest rank (its band + the tail octave it detects) + the block merge; "
                                        "the two all-gathers (octave-(K+1) base rows, keypoints) are not in it",
                  "speedup_vs_whole": round(1e3 * float(np.median(t_whole)) / crit, 2),
                  "keypoints": n_whole, "identical": bool(same)}))
