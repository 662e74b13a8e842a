#!/usr/bin/env python3
"""cfg 5 (8K, O=6, S=5) on one GPU, device-resident: whole-image detection
(input in HBM, keypoints left in HBM) vs the same image as n row-band shards
run in turn through sift_amd.shard.detect_sharded_device_local, with per-part
times.  The phases of n devices are sequential: every tail octave starts from
the gathered octave-(K+1) base, which needs every band, so the critical path
is the slowest band + the base all-gather + the slowest tail octave + the
keypoint all-gather + the merge.  The two all-gathers are timed here at their
real sizes under nccl (RCCL) at world size 1 -- a device-local copy, the
lower bound of the xGMI transfer -- and modelled at `--xgmi-gbs` (the bytes
one rank receives over its xGMI links).
usage: tools/shard_time_device.py [n_shards] [reps] [xgmi_GBps]"""
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
xgmi = float(sys.argv[3]) if len(sys.argv) > 3 else 300.0  # GB/s into one rank (7 links x ~50 GB/s used)
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

# The two all-gathers at their real sizes (padded to the largest part, as
# shard.gather_rows sends them), timed under nccl at world size 1.
import torch.distributed as dist  # noqa: E402
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dist.init_process_group("nccl", rank=0, world_size=1)
seed_rows = [(lambda a: a[1] - a[0])(shard._seed_rows(plan, r)) for r in range(len(plan.bands))]
cols = sift_amd.octave_dims(W, H, O)[plan.K + 1][1]


def t_gather(nbytes_per_rank, world):
    send = torch.zeros(nbytes_per_rank, dtype=torch.uint8, device="cuda:0")
    recv = torch.empty(nbytes_per_rank * 1, dtype=torch.uint8, device="cuda:0")
    ts = []
    for i in range(reps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dist.all_gather_into_tensor(recv, send)
        torch.cuda.synchronize()
        if i >= 2:
            ts.append(time.perf_counter() - t0)
    local = float(np.median(ts)) * 1e3
    # the world-1 call's own time (launch + copy: the latency floor) + the
    # bytes received from the other ranks at the modelled xGMI rate
    model = local + nbytes_per_rank * (world - 1) / (xgmi * 1e9) * 1e3
    return local, model


# Keypoints per rank: a band's (octaves 0..K, its own rows; abs_y decides the
# band here, a model) and a tail owner's (its octaves > K).
kpa = np.frombuffer(whole, dtype=sift_amd.KEYPOINT_DTYPE)
band_n = [int(((kpa["octave"] <= plan.K) & (kpa["abs_y"] >= lo) & (kpa["abs_y"] < hi)).sum())
          for lo, hi in plan.bands]
tail_n = [0] * len(plan.bands)
for t, r in owner.items():
    tail_n[r] += int((kpa["octave"] == t).sum())
base_pad = max(seed_rows) * cols * 8
kp_pad = max(band_n) * 48   # parts are padded to the largest
tkp_pad = max(max(tail_n), 1) * 48
base_local, base_model = t_gather(base_pad, n)
kp_local, kp_model = t_gather(kp_pad, n)
tkp_local, tkp_model = t_gather(tkp_pad, n)
dist.destroy_process_group()
# The band keypoints' all-gather runs during the tail octaves (shard.detect_sharded_device);
# after the tail only the tail keypoints are gathered.
tail_max = max(tails.values() or [0.0])
crit = max(shards) + base_model + max(tail_max + tkp_model, kp_model) + med["merge"]
crit_serial = max(shards) + base_model + tail_max + kp_model + tkp_model + med["merge"]
print(json.dumps({"config": "8K 7680x4320 O6 S5, device-resident (image in HBM, keypoints in HBM)",
                  "n_shards": n, "K": plan.K, "bands": plan.bands, "crops": plan.crops,
                  "whole_ms": round(1e3 * float(np.median(t_whole)), 3),
                  "shard_ms": [round(x, 3) for x in shards],
                  "tail_octave_ms": {str(t): round(v, 3) for t, v in tails.items()},
                  "tail_owner": {str(t): r for t, r in owner.items()},
                  "per_rank_ms": [round(x, 3) for x in per_rank],
                  "merge_ms": round(med["merge"], 3),
                  "base_gather": {"bytes_per_rank": base_pad, "nccl_world1_ms": round(base_local, 3),
                                  "model_ms": round(base_model, 3)},
                  "band_keypoints_per_rank": band_n, "tail_keypoints_per_rank": tail_n,
                  "kp_gather": {"bytes_per_rank": kp_pad, "nccl_world1_ms": round(kp_local, 3),
                                "model_ms": round(kp_model, 3)},
                  "tail_kp_gather": {"bytes_per_rank": tkp_pad, "nccl_world1_ms": round(tkp_local, 3),
                                     "model_ms": round(tkp_model, 3)},
                  "xgmi_GBps_model": xgmi,
                  "critical_path_ms": round(crit, 3),
                  "critical_path_serial_gathers_ms": round(crit_serial, 3),
                  "critical_path_note": "every tail octave starts from the gathered base: slowest band + base "
                                        "all-gather (model) + max(slowest tail octave + tail-keypoint all-gather, "
                                        "band-keypoint all-gather running beside the tail) (models: world-1 call time + bytes "
                                        "from the other ranks at xgmi_GBps_model) + the two block merges of the padded "
                                        "gathered lists",
                  "speedup_vs_whole": round(1e3 * float(np.median(t_whole)) / crit, 2),
                  "keypoints": n_whole, "identical": bool(same)}))
