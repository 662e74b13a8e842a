#!/usr/bin/env python3
"""Throughput of the MI355X SIFT scale-space extrema path.

One step = one pass of the hot path over one synthetic image per GPU:
Gaussian scale space + DoG (k_gauss_dog), 26-neighbour extrema scan with
ordering and exact tie resolution, quadratic refinement -- all through the
C ABI (sift_detect_device, input already resident in HBM).  With N > 1 GPUs
(one process per GPU, torchrun), every rank processes its own image and the
keypoint lists are all-gathered over RCCL (xGMI) each step: weak scaling.

Prints ONE JSON line (rank 0).  Workload defaults to BASELINE.json's metric
configuration: 3840x2160 (4K), 4 octaves x 5 scales.

`roofline` is SURVEY.md §8d's north-star quantity, the whole Gaussian+DoG
pass (one k_gauss_dog launch per octave): B_alg = 4WH + sum_o 4 P_o (S+3) +
sum_o 4 P_o (S+2) (the input read, every Gaussian and DoG plane written in
fp32) divided by the pass's HIP-event time on the context's stream, one image
at a time; `per_octave`, `pipelined`, `octave0` and `extrema_stage` break it
down.  `traffic` is the pass's HBM bytes (every pass launch of one image)
from the rocprofv3 PMC summary of the latest round (profiles/*pmc*.json,
tools/pmc_launches.py, or --pmc) when it matches the config, split per
octave in `per_octave[o].traffic`.  `sustained` re-runs the pipelined loop for --sustain-s seconds after
the timed region (a steady-state rate over thousands of images, beside the
K-step `value`).
"""
import argparse
import glob
import json
import math
import os
import re
import sys
import time


ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def metric_name(W, H, O, S, batch=1):
    """BASELINE.json's metric string, with this run's image size and pyramid
    (3840x2160 is the baseline's "4K")."""
    size = "4K" if (W, H) == (3840, 2160) else "%dx%d" % (W, H)
    return "Mpix/s through Gaussian+DoG+extrema, %s img%s, %d oct × %d scales; %% HBM roofline" % (
        size, " x %d per GPU" % batch if batch > 1 else "", O, S)


def octave_dims(W, H, O):
    h, w, out = 2 * H, 2 * W, []
    for o in range(O):
        if o:
            h, w = (h + 1) // 2, (w + 1) // 2
        out.append((h, w))
    return out


def alg_bytes(W, H, O, S, skip_gauss):
    P = [h * w for h, w in octave_dims(W, H, O)]
    b = 4 * W * H + sum(4 * p * (S + 2) for p in P)
    if skip_gauss:
        b += sum(8 * p for p in P[1:])  # fp64 seeds written instead of the Gaussian planes
    else:
        b += sum(4 * p * (S + 3) for p in P)
    return b


def octave_bytes(W, H, O, S, skip_gauss):
    """Algorithmic bytes of each octave's Gaussian+DoG launch (they sum to
    alg_bytes): its planes written in fp32, plus the input read for octave 0
    (skip_gauss: the fp64 seed of octave o >= 1 is written instead of its
    Gaussian planes)."""
    out = []
    for o, (h, w) in enumerate(octave_dims(W, H, O)):
        b = 4 * h * w * (S + 2) + (4 * W * H if o == 0 else 0)
        b += (8 * h * w if o > 0 else 0) if skip_gauss else 4 * h * w * (S + 3)
        out.append(b)
    return out


def oct0_bytes(W, H, S, skip_gauss):
    """Algorithmic bytes of octave 0's Gaussian+DoG launch."""
    return octave_bytes(W, H, 1, S, skip_gauss)[0]


def extrema_bytes(W, H, O, S):
    """Algorithmic bytes of the extrema scan: every DoG plane read once."""
    return sum(4 * h * w * (S + 2) for h, w in octave_dims(W, H, O))


def _round_key(path):
    """Sort key of a profile's round tag: r4v < r4al < r5a (round, then the
    letter suffix in a..z, aa..az order)."""
    m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
    if not m:
        return (-1, 0, "")
    return (int(m.group(1)), len(m.group(2)), m.group(2))


def load_pmc(cfg_key, path=None):
    """The PMC summary of this configuration (tools/pmc_launches.py): the one
    named by --pmc, else the committed profiles/*pmc*.json of the latest
    round tag whose config_key matches."""
    paths = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")),
                                       key=_round_key, reverse=True)
    for p in paths:
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("config_key") == cfg_key and d.get("pass_hbm_bytes"):
            return d, os.path.relpath(p, ROOT)
    return None, None


def cpu_baseline(img_full, O, S, sample_w, sample_h, threads=1):
    """The oracle's reference-faithful 2D-kernel port on a crop, with `threads`
    threads in its blur loops (1 = the scalar port)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    crop = img_full[:sample_h, :sample_w].copy()
    p = orc.make_params(O, S)
    orc.set_threads(threads)
    try:
        t0 = time.perf_counter()
        nk, nc = orc.detect_count(crop, p, orc.CONV_2D)
        dt = time.perf_counter() - t0
    finally:
        orc.set_threads(1)
    return {"value": round(sample_w * sample_h / dt / 1e6, 6), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": "%dx%d crop of the same synthetic image, %d oct x %d scales, G+DoG+extrema+refine, "
                      "reference 2D-kernel algorithm restated in C (oracle/sift_oracle.c CONV_2D%s), "
                      "%.1f s, %d keypoints" % (sample_w, sample_h, O, S,
                                                ", blur loops over %d OpenMP threads" % threads if threads > 1
                                                else "", dt, nk)}


def cpu_baseline_js(img_full, O, S, sample_w, sample_h):
    """a clean-room single-threaded JavaScript
    restatement of the reference's 2D-kernel algorithm (tools/js_restatement/
    sift_restated.mjs, pinned to the reference's golden lists by
    tests/test_js_restatement.py), timed under the host's Node on a crop."""
    import shutil
    import subprocess
    import tempfile
    import numpy as np
    node = shutil.which("node")
    if node is None:
        return None
    crop = np.ascontiguousarray(img_full[:sample_h, :sample_w], dtype="<f4")
    with tempfile.TemporaryDirectory() as td:
        crop.tofile(os.path.join(td, "img.f32"))
        r = subprocess.run([node, os.path.join(ROOT, "tools", "js_restatement", "sift_restated.mjs"),
                            os.path.join(td, "img.f32"), str(sample_w), str(sample_h), str(O), str(S)],
                           capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        return {"value": None, "error": r.stderr[-300:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    return {"value": round(sample_w * sample_h / d["seconds"] / 1e6, 6), "unit": "Mpix/s", "cores": 1,
            "kind": "restatement",
            "sample": "%dx%d crop of the same synthetic image, %d oct x %d scales, G+DoG+extrema+refine, "
                      "reference 2D-kernel algorithm restated in JavaScript (tools/js_restatement/sift_restated.mjs, "
                      "flat Float64Array planes), Node %s, one thread, %.1f s, %d keypoints"
                      % (sample_w, sample_h, O, S, d["node"], d["seconds"], d["keypoints"])}


def host_cores():
    """CPU threads this process may use (the GPU box's share is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:  # OpenMP allows a list ("8,2"): the first level is what one process gets
        cap = int(os.environ.get("OMP_NUM_THREADS", "16").split(",")[0])
    except ValueError:
        cap = 16
    return max(1, min(n, cap))


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=None, help="default 3840 (7680 with --shard-image)")
    ap.add_argument("--height", type=int, default=None, help="default 2160 (4320 with --shard-image)")
    ap.add_argument("--octaves", type=int, default=None, help="default 4 (6 with --shard-image)")
    ap.add_argument("--scales", type=int, default=5)
    ap.add_argument("--skip-gauss-planes", action="store_true",
                    help="keypoints-only mode: do not materialise the Gaussian planes")
    ap.add_argument("--batch", type=int, default=1,
                    help="independent images per GPU per step (BASELINE cfg 4: --width 1920 --height 1080 "
                         "--batch 8 on 8 GPUs = 64 images per step)")
    ap.add_argument("--batch-mode", default="launch", choices=["launch", "images"],
                    help="with --batch B > 1: launch = the B images as ONE batched detection per step "
                         "(sift_detect_batch_device: one launch per stage over the batch), images = B separate "
                         "detections per step")
    ap.add_argument("--inflight", type=int, default=None,
                    help="detections in flight per GPU (one context each; the host settles image k while "
                         "image k+1 runs).  Default under --overlap full (the default schedule): 3 for single "
                         "images of >= 4 Mpix (4K: 3 > 4 by 1-2 %%, profiles/r5w_schedule_ab.txt), 4 for smaller "
                         "images and batched launches when GPU_MAX_HW_QUEUES >= 8, else 3; under an ordered "
                         "--overlap: 2 for single images of >= 4 Mpix (profiles/r4am_inflight_ab.txt), 3 otherwise")
    ap.add_argument("--overlap", default=None,
                    choices=["none", "octave0", "gaussian", "refinement", "full", "phased"],
                    help="how consecutive images overlap on the GPU: none = contexts share one stream; "
                         "octave0 / gaussian / refinement = own streams, image k+1 starts once image k has "
                         "passed that point (sift_order_after: software pipelining); full = own streams, "
                         "no ordering.  Default: full (profiles/r5w_schedule_ab.txt).  Per-kernel durations "
                         "(roofline.achieved) include any overlap")
    ap.add_argument("--shard-image", action="store_true",
                    help="BASELINE cfg 5: ONE image per step split over all ranks in row bands (sift_amd.shard."
                         "detect_sharded_device: band octaves, all-gathered next-octave base, tail octaves one per "
                         "rank, block-major merge); strong scaling.  Defaults to 7680x4320, 6 octaves x 5 scales "
                         "unless --width/--height/--octaves are given")
    ap.add_argument("--sustain-s", type=float, default=5.0,
                    help="seconds of the same pipelined loop after the timed region, reported as `sustained` "
                         "(0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=None,
                    help="PMC summary (tools/pmc_launches.py) for roofline.traffic; default: the committed "
                         "profiles/*pmc*.json of the latest round tag for this configuration")
    ap.add_argument("--cpu-sample", default="1920x1080", help="crop WxH timed on the CPU oracle")
    ap.add_argument("--cpu-sample-js", default="1920x1080",
                    help="crop WxH timed on the single-threaded JS restatement (the C port's crop; about 15 s on the GPU box)")
    args = ap.parse_args()
    big = args.shard_image
    args.width = args.width or (7680 if big else 3840)
    args.height = args.height or (4320 if big else 2160)
    args.octaves = args.octaves or (6 if big else 4)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        # the driver launches N ranks for --gpus N; any other pairing would report a wrong n_gpus
        print("bench.py: --gpus %d but WORLD_SIZE=%d: launch %d processes (torchrun --nproc-per-node %d)"
              % (args.gpus, world, args.gpus, args.gpus), file=sys.stderr)
        return 2

    import numpy as np
    import torch
    import sift_amd
    from sift_amd.synth import blob_image

    dist = None
    # SIFT_BENCH_DIST=1: the collective path at world size 1 too (rehearsal of
    # the N > 1 code on a one-GPU box under torchrun)
    if world > 1 or os.environ.get("SIFT_BENCH_DIST") == "1":
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")  # RCCL over xGMI
    dev = local_rank
    W, H, O, S = args.width, args.height, args.octaves, args.scales
    if args.shard_image:
        return bench_shard_image(args, dist, world, rank, dev)
    flags = sift_amd.F_SKIP_GAUSS_PLANES if args.skip_gauss_planes else 0
    params = sift_amd.make_params(O, S, flags=flags)

    img = blob_image(W, H, seed=42 + rank)
    d_img = torch.from_numpy(img).to("cuda:%d" % dev)
    Bt = max(1, args.batch)
    batched = Bt > 1 and args.batch_mode == "launch"
    if args.overlap is None:
        # contexts with no ordering between them (4K single images: 7.18 against 7.00 Gpix/s for
        # octave0 with two, and steadier; 1080p singles and batches of 8 with four contexts: +7 / +3 %
        # over octave0 with three; profiles/r5w_schedule_ab.txt)
        args.overlap = "full"
    if batched and args.overlap == "phased":
        print("bench.py: --overlap phased does not apply to batched launches", file=sys.stderr)
        return 2
    d_imgs = None
    if batched:  # B distinct images back to back in HBM (image 0 is the rank's usual image)
        d_imgs = torch.from_numpy(np.stack([img] + [blob_image(W, H, seed=1000 + 64 * rank + i)
                                                   for i in range(1, Bt)])).to("cuda:%d" % dev)
    torch.cuda.synchronize(dev)
    # in flight (overlap full; profiles/r5w_schedule_ab.txt): 3 for single images of 4 Mpix and more
    # (4K: 3 > 4 by 1-2 %; 8K: equal); for smaller single images and batched launches 4 when the process
    # runs with GPU_MAX_HW_QUEUES >= 8 (1080p: 6.31-6.46 against 6.10 Gpix/s with 3; 1080p x 8: 7.35-7.45
    # against 7.14-7.18) -- with the runtime's default 4 queues a fourth context shares a queue with
    # another and they run in turn (1080p: 5.26-5.30), so 3 there.  The variable is read when the HIP
    # runtime loads, before this script runs: it has to come from the caller's environment.  Under an
    # ordered schedule 2 for large single images (octave0: 2 > 3 by 1.5-2 %, r4am_inflight_ab.txt).
    hwq = int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    if args.inflight is not None:
        nin = max(1, args.inflight)
    elif args.overlap == "full":
        nin = 3 if (args.batch == 1 and W * H >= 4000000) or hwq < 8 else 4
    else:
        nin = 3 if args.batch > 1 or W * H < 4000000 else 2
    ctxs = [sift_amd.Context(dev)]
    own = args.overlap != "none"
    after = {"octave0": sift_amd.AFTER_OCTAVE0, "gaussian": sift_amd.AFTER_GAUSSIAN,
             "refinement": sift_amd.AFTER_REFINEMENT}.get(args.overlap)
    ctxs += [sift_amd.Context(dev, share=None if own else ctxs[0]) for _ in range(nin - 1)]
    ctx = ctxs[0]

    gather = None
    if dist is not None:
        # every image's keypoint list reaches every rank (RCCL all-gather over
        # xGMI); the records gather is left in flight under the next images'
        # detections (the counts gather is the step's only synchronisation)
        from sift_amd.dist import PipelinedKeypointGather
        gather = PipelinedKeypointGather("cuda:%d" % dev, depth=nin)

    stage = {"gauss_dog_ms": 0.0, "extrema_ms": 0.0, "refine_ms": 0.0, "gauss_oct0_ms": 0.0}
    oct_ms = [0.0] * O

    phased = args.overlap == "phased"
    pend = [None]  # phased: the image whose extrema + refinement are not enqueued yet

    def launch(i):
        c = ctxs[i % nin]
        if phased:
            # HBM-bound phases of consecutive images alternate: octave 0 of
            # image i runs after image i-2's refinement and before image
            # i-1's extrema scan; the small octaves (fp64 / TA bound) of one
            # image overlap the extrema + refinement of the previous one.
            if i >= 2:
                c.order_after(ctxs[(i - 2) % nin], sift_amd.AFTER_REFINEMENT)
            c.detect_begin_async(d_img.data_ptr(), W, H, params)
            if pend[0] is not None:
                p = ctxs[pend[0] % nin]
                p.order_after(c, sift_amd.AFTER_OCTAVE0)
                p.detect_end_async()
            pend[0] = i
            return
        if after is not None and i > 0 and nin > 1:
            c.order_after(ctxs[(i - 1) % nin], after)
        if batched:
            c.detect_batch_device_async(d_imgs.data_ptr(), Bt, W, H, params)
        else:
            c.detect_device_async(d_img.data_ptr(), W, H, params)

    def flush():
        if pend[0] is not None:
            ctxs[pend[0] % nin].detect_end_async()
            pend[0] = None

    def finish(i, acc):
        c = ctxs[i % nin]
        n = c.detect_wait()
        if dist is not None:
            n = sum(gather(n, lambda buf, cap: c.copy_keypoints_device(buf.data_ptr(), cap)))
        if acc:
            t = c.timings()
            for k in stage:
                stage[k] += t[k]
            for o, v in enumerate(c.octave_timings()):
                oct_ms[o] += v
        return n

    # Warm-up: every context settles its capacities synchronously first.
    for i in range(max(args.warmup, nin)):
        launch(i)
        flush()
        finish(i, False)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    for c in ctxs:
        c.synchronize()
    t0 = time.perf_counter()
    n_total = 0
    NI = args.steps * (1 if batched else Bt)  # detections (images, or batches) in the timed region
    for i in range(NI):  # image i is enqueued before image i-(nin-1) is settled
        launch(i)
        if i >= nin - 1:
            n_total = finish(i - (nin - 1), True)
    flush()
    for i in range(max(0, NI - (nin - 1)), NI):
        n_total = finish(i, True)
    if gather is not None:
        gather.drain()  # the last records gathers complete inside the timed region
    for c in ctxs:
        c.synchronize()
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # What the timed region computed: the keypoint records of its last image
    # (the pipelined own-stream schedule), checked after the measurements
    # against a synchronous detection of the same input on a fresh context.
    kp_timed = ctxs[(NI - 1) % nin].keypoints().tobytes()
    # Steady state: the same pipelined loop for a few seconds (thousands of
    # images; no per-image host work beyond the settle), its own clock.
    # The image count comes from the timed region's max-over-ranks time, so
    # every rank runs the same number of per-image collectives.
    sustained = None
    if args.sustain_s > 0:
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(dev)
        n_sus = max(nin, int(math.ceil(args.sustain_s / max(elapsed / NI, 1e-6))))
        t1 = time.perf_counter()
        for ns in range(n_sus):
            launch(NI + ns)
            if ns >= nin - 1:
                finish(NI + ns - (nin - 1), False)
        ns = n_sus
        flush()
        for i in range(max(0, ns - (nin - 1)), ns):
            finish(NI + i, False)
        for c in ctxs:
            c.synchronize()
        torch.cuda.synchronize(dev)
        ts = time.perf_counter() - t1
        if dist is not None:
            e = torch.tensor([ts], dtype=torch.float64, device="cuda:%d" % dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            ts = float(e.item())
        ipd = Bt if batched else 1  # images per detection
        sustained = {"images_per_gpu": ns * ipd, "seconds": round(ts, 3),
                     "value": round(world * ns * ipd * W * H / ts / 1e6, 3), "unit": "Mpix/s",
                     "ms_per_image": round(ts / (ns * ipd) * 1e3, 4)}
    # After the timed region: the same detection alone (one image in flight,
    # nothing overlapping), so the kernel's isolated duration is on record
    # beside its pipelined one.
    iso = {"gauss_dog_ms": 0.0, "gauss_oct0_ms": 0.0, "extrema_ms": 0.0, "refine_ms": 0.0}
    iso_oct = [0.0] * O
    n_iso = 10
    for _ in range(n_iso):
        if batched:
            ctx.detect_batch_device_async(d_imgs.data_ptr(), Bt, W, H, params)
        else:
            ctx.detect_device_async(d_img.data_ptr(), W, H, params)
        ctx.detect_wait()
        t = ctx.timings()
        for k in iso:
            iso[k] += t[k] / n_iso
        for o, v in enumerate(ctx.octave_timings()):
            iso_oct[o] += v / n_iso
    pass_kernels = ctx.pass_kernels()  # the library's own record of the launches (sift_last_pass_kernels)
    with sift_amd.Context(dev) as vctx:
        if batched:  # the batch against the same images detected one by one
            ref = []
            for b in range(Bt):
                vctx.detect_device(d_imgs[b].data_ptr(), W, H, params)
                ref.append(vctx.keypoints().tobytes())
            verified = b"".join(ref) == kp_timed
        else:
            vctx.detect_device(d_img.data_ptr(), W, H, params)
            verified = vctx.keypoints().tobytes() == kp_timed
    if not verified:
        print("bench.py: rank %d: the timed region's last keypoint list differs from a synchronous detection"
              % rank, file=sys.stderr)
    K = args.steps
    ms_per_step = elapsed / K * 1e3
    value = world * Bt * W * H / (elapsed / K) / 1e6
    counts = ctxs[(NI - 1) % nin].counts()

    if rank == 0:
        gauss_ms = stage["gauss_dog_ms"] / NI
        oct0_ms = stage["gauss_oct0_ms"] / NI
        ipd = Bt if batched else 1  # the pass of one detection covers ipd images
        B = ipd * alg_bytes(W, H, O, S, args.skip_gauss_planes)
        Bo = [ipd * b for b in octave_bytes(W, H, O, S, args.skip_gauss_planes)]
        B0 = Bo[0]
        gbs = lambda b, ms: b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        cfg_key = "%dx%d_o%d_s%d%s" % (W, H, O, S, "_nogauss" if args.skip_gauss_planes else "")
        pmc, pmc_src = load_pmc(cfg_key, args.pmc)
        pass_traffic = pmc["pass_hbm_bytes"] if pmc else None
        oct0_traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        oct_traffic = {}
        for r in (pmc or {}).get("per_octave", []):
            oct_traffic[tuple(r["octaves"])] = r["hbm_bytes"]
        pipelined_note = ("pipelined: %d images in flight on %d streams, each launch's window includes "
                          "waiting for CUs held by the other images' kernels" % (nin, nin)
                          if own and nin > 1 else "one image at a time")
        B_x = ipd * extrema_bytes(W, H, O, S)
        iso_pass = iso["gauss_dog_ms"]
        out = {
            "metric": metric_name(W, H, O, S, Bt),
            "value": round(value, 3),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": "%s%dx%d gray f32 image%s per GPU per step, %d octaves x %d scales, "
                            "Gaussian+DoG+extrema+refine (keypoints out)%s" %
                            ("%d x " % Bt if Bt > 1 else "", W, H, "s" if Bt > 1 else "", O, S,
                             ", Gaussian planes not materialised" if args.skip_gauss_planes else ""),
                "width": W, "height": H, "octaves": O, "scales_per_octave": S,
                "images_per_gpu": Bt, "global_batch": world * Bt, "inflight_per_gpu": nin,
                "batch_launch": batched,
                "streams_per_gpu": nin if own else 1,
                "overlap": args.overlap,
                "parallelism": ("dp%d (%d image%s per GPU, RCCL keypoint all-gather)" % (world, Bt, "s" if Bt > 1 else "")
                                if world > 1 else "single GPU"),
                "planes": "fp32 out, fp64 accumulation/seeds",
            },
            "sustained": sustained,
            "stages_ms": {k: round(v / NI, 4) for k, v in stage.items()},
            "keypoints": counts["keypoints"],
            "candidates": counts["candidates"],
            "keypoints_all_ranks": n_total,
            "verified": verified,
            "verified_what": (("rank 0: the last timed batch's keypoint records (one batched detection of %d "
                               "distinct images, pipelined schedule, %d contexts) byte-identical to the %d images "
                               "detected one by one (sift_detect_device) on a fresh context" % (Bt, nin, Bt))
                              if batched else
                              ("rank 0: the last timed image's keypoint records (pipelined schedule, %d contexts) "
                               "byte-identical to a synchronous sift_detect_device of the same input on a fresh "
                               "context" % nin)),
            "roofline": {
                "bound": "hbm",
                "kernel": "Gaussian+DoG pass: every launch of one image's %d octaves%s (%s)" %
                          (O, ", each over the batch of %d images" % Bt if batched else "", pass_kernels),
                "achieved": round(gbs(B, iso_pass), 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(gbs(B, iso_pass) / HBM_PEAK_GBS, 4),
                "traffic": pass_traffic,
                "traffic_source": pmc_src,
                "alg_bytes_per_launch": B,
                "alg_bytes_formula": ("4WH + sum_o 4P_o(S+2) + sum_{o>=1} 8P_o" if args.skip_gauss_planes
                                      else "4WH + sum_o 4P_o(S+3) + sum_o 4P_o(S+2)"),
                "launch_ms": round(iso_pass, 5),
                "measured": ("HIP events on the context stream around the pass (first octave launch to the end "
                             "of the last), one image at a time, averaged over %d images run right after the "
                             "timed region (SURVEY.md §8d's north-star quantity; the pipelined window of the "
                             "timed region is `pipelined`)" % n_iso),
                "per_octave": [
                    {"octave": o, "plane": list(octave_dims(W, H, O)[o]), "alg_bytes": Bo[o],
                     "iso_ms": round(iso_oct[o], 5), "iso_frac": round(gbs(Bo[o], iso_oct[o]) / HBM_PEAK_GBS, 4),
                     "pipelined_ms": round(oct_ms[o] / NI, 5),
                     "traffic": next((v for k, v in oct_traffic.items() if o in k), None),
                     "traffic_octaves": next((list(k) for k in oct_traffic if o in k), None)}
                    for o in range(O)],
                "pipelined": {
                    "what": "the same pass inside the timed region (%s), HIP events, averaged over %d images" %
                            (pipelined_note, NI),
                    "ms": round(gauss_ms, 5),
                    "achieved": round(gbs(B, gauss_ms), 1),
                    "frac": round(gbs(B, gauss_ms) / HBM_PEAK_GBS, 4),
                },
                "octave0": {
                    "what": "octave 0's k_gauss_dog launch alone (HBM-store bound)",
                    "alg_bytes": B0,
                    "iso_ms": round(iso["gauss_oct0_ms"], 5),
                    "iso_frac": round(gbs(B0, iso["gauss_oct0_ms"]) / HBM_PEAK_GBS, 4),
                    "pipelined_ms": round(oct0_ms, 5),
                    "pipelined_frac": round(gbs(B0, oct0_ms) / HBM_PEAK_GBS, 4),
                    "traffic": oct0_traffic,
                    "traffic_source": pmc_src,
                },
                "extrema_stage": {
                    "what": "extrema stage (scan of every DoG plane + ordered emission + exact re-decisions), "
                            "one image at a time",
                    "alg_bytes": B_x,
                    "alg_bytes_formula": "sum_o 4P_o(S+2)",
                    "iso_ms": round(iso["extrema_ms"], 5),
                    "iso_frac": round(gbs(B_x, iso["extrema_ms"]) / HBM_PEAK_GBS, 4),
                },
                "refine_stage": {
                    "what": "refinement stage (fast pass from the scan's captured patches / DoG gathers, exact "
                            "re-decisions, compaction), one image at a time",
                    "iso_ms": round(iso["refine_ms"], 5),
                },
            },
            "cpu_baseline": None,
            "cpu_baseline_all_cores": None,
            "cpu_baseline_js": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            sw, sh = (int(v) for v in args.cpu_sample.split("x"))
            out["cpu_baseline"] = cpu_baseline(img, O, S, min(sw, W), min(sh, H))
            nt = host_cores()
            if nt > 1:  # the port on 1 core and on all the cores this process may use
                out["cpu_baseline_all_cores"] = cpu_baseline(img, O, S, min(sw, W), min(sh, H), threads=nt)
            jw, jh = (int(v) for v in args.cpu_sample_js.split("x"))
            out["cpu_baseline_js"] = cpu_baseline_js(img, O, S, min(jw, W), min(jh, H))
        print(json.dumps(out), flush=True)
    for c in reversed(ctxs):
        c.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


def bench_shard_image(args, dist, world, rank, dev):
    """BASELINE cfg 5: one image per step, row bands over the ranks (strong
    scaling): value = input pixels of one image / time per image."""
    import torch
    import sift_amd
    from sift_amd import shard
    from sift_amd.synth import blob_image
    W, H, O, S = args.width, args.height, args.octaves, args.scales
    params = sift_amd.make_params(O, S)
    img = blob_image(W, H, seed=42)
    d_img = torch.from_numpy(img).to("cuda:%d" % dev)
    ctx = sift_amd.Context(dev)
    run = (lambda tm=None: shard.detect_sharded_device(ctx, d_img, params, timer=tm)) if dist is not None else \
        (lambda tm=None: shard.detect_sharded_device_local(ctx, d_img, params, 1, timer=tm))
    for _ in range(max(1, args.warmup)):
        out, plan = run()
    n_kp = int(out.shape[0])
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    parts = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out, plan = run(parts)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cuda:%d" % dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    K = args.steps
    if rank == 0:
        out = {
            "metric": metric_name(W, H, O, S) + " (one image split over the GPUs)",
            "value": round(W * H / (elapsed / K) / 1e6, 3),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": "one %dx%d gray f32 image per step split over %d GPU%s in row bands (BASELINE cfg 5), "
                            "%d octaves x %d scales, Gaussian+DoG+extrema+refine, whole-image keypoints on every "
                            "rank" % (W, H, world, "s" if world > 1 else "", O, S),
                "width": W, "height": H, "octaves": O, "scales_per_octave": S,
                "parallelism": "row bands: octaves 0..%d on overlapping crops, octave-%d base all-gathered, tail "
                               "octaves one per rank, counts + keypoints all-gathered, block-major merge"
                               % (plan.K, plan.K + 1) if world > 1 else "single GPU (one band)",
                "bands": plan.bands, "K": plan.K,
            },
            "parts_ms_per_step": {k: round(v / K * 1e3, 4) for k, v in parts.items()},
            "keypoints": n_kp,
            "roofline": None,
            "cpu_baseline": None,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
