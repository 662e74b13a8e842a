#!/usr/bin/env python3
"""Host-time probe of one cfg 5 tail piece (8K O6 S5, 8 bands, deepest tail
octave): wall time of each Python / library step of run_tail_octave_device,
and the library's own GPU stage times (HIP events), median of `reps`.
usage: tools/tail_host_probe.py [reps]"""
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

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
W, H, O, S = 7680, 4320, 6, 5
d_img = torch.from_numpy(blob_image(W, H, seed=42)).to("cuda:0")
p = sift_amd.make_params(O, S)
ctx = sift_amd.Context(0)
plan = shard.plan_bands(W, H, p, 8)
parts = [shard.run_shard_device(ctx, d_img, p, plan, r)[2] for r in range(len(plan.bands))]
base = torch.cat(parts).contiguous()
t = O - 1
rec = {k: [] for k in ("params", "ready", "call", "kp_copy", "counts", "total")}
gpu = []
for i in range(reps + 2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pp = sift_amd.make_params(t + 1, S, p.min_blur, p.assumed_blur, p.min_interpixel_distance, p.flags)
    h, w = shard.octave_dims(W, H, O)[plan.K + 1]
    t1 = time.perf_counter()
    shard.torch_ready(base)
    t2 = time.perf_counter()
    n = ctx.detect_from_seed_range_device(base.data_ptr(), plan.K + 1, t, W, H, pp)
    t3 = time.perf_counter()
    kp = shard._device_keypoints(ctx, n, torch, base.device)
    t4 = time.perf_counter()
    c = ctx.block_counts()
    t5 = time.perf_counter()
    if i >= 2:
        for k, v in zip(rec, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0)):
            rec[k].append(v * 1e3)
        gpu.append(ctx.timings())
med = {k: round(float(np.median(v)), 4) for k, v in rec.items()}
gs = {k: round(float(np.median([g[k] for g in gpu])), 4) for k in gpu[0]}
print({"piece": "tail octave %d from the octave-%d base (%dx%d)" % (t, plan.K + 1, w, h), "wall_ms": med,
       "library_stage_ms": gs, "keypoints": int(n)})
