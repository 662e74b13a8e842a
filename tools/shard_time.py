#!/usr/bin/env python3
"""cfg 5 (8K, O=6, S=5) on one GPU: whole-image detection vs the same image
as n row-band shards run in turn (sift_amd.shard.detect_sharded_local), with
per-part times -- the redundant halo work a row-band split costs, and the
critical path n devices would see (slowest shard + gathers + tail).
usage: tools/shard_time.py [n_shards] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd import shard  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
W, H, O, S = 7680, 4320, 6, 5
img = blob_image(W, H, seed=42)
p = sift_amd.make_params(O, S)
ctx = sift_amd.Context(0)
whole = ctx.detect(img, p).copy()  # warm-up + reference
t_whole = []
for _ in range(reps):
    t0 = time.perf_counter()
    ctx.detect(img, p)
    t_whole.append(time.perf_counter() - t0)
plan = shard.plan_bands(W, H, p, n)
t_parts, seeds, parts = [], [], []
steps = {}
for rep in range(reps + 1):
    tp, seeds, parts = [], [], []
    for r in range(len(plan.bands)):
        t0 = time.perf_counter()
        kp, org, seed = shard.run_shard(ctx, img, p, plan, r, timer=steps if rep else None)
        tp.append(time.perf_counter() - t0)
        parts.append((kp, org))
        seeds.append(seed)
    t0 = time.perf_counter()
    if plan.has_tail:
        parts.append(shard.run_tail(ctx, np.concatenate(seeds), p, plan))
    tp.append(time.perf_counter() - t0)
    if rep:
        t_parts.append(tp)
merged = shard.merge(parts)
same = merged.tobytes() == whole.tobytes()
tp = np.median(np.array(t_parts), axis=0)
print(json.dumps({"config": "8K 7680x4320 O6 S5, host image in/keypoints out (includes H2D/D2H)",
                  "n_shards": n, "K": plan.K, "bands": plan.bands, "crops": plan.crops,
                  "whole_ms": round(1e3 * float(np.median(t_whole)), 3),
                  "shard_ms": [round(1e3 * float(x), 3) for x in tp[:-1]],
                  "tail_ms": round(1e3 * float(tp[-1]), 3),
                  "sum_ms": round(1e3 * float(tp.sum()), 3),
                  "critical_path_ms": round(1e3 * float(tp[:-1].max() + tp[-1]), 3),
                  "shard_steps_ms_per_rep": {k: round(1e3 * v / reps, 3) for k, v in steps.items()},
                  "keypoints": int(whole.shape[0]), "identical": bool(same)}))
