"""Row-band sharding of ONE image over several devices (cfg 5).

The reference runs one image in one Web Worker; there is nothing to mirror
here beyond its results, which a sharded run reproduces bit for bit.

Octaves depend on each other only through the fp64 base of the next octave
(background.js:114-118), and every pixel's Gaussian is the same fma chain on
its clamped neighbourhood (translation invariant in y).  So:

* shard r owns the input rows [lo_r, hi_r) (boundaries at multiples of
  2^(O-1), whole rows in every octave) and runs the leading octaves 0..K on a
  crop [c0_r, c1_r) that extends its band by a margin M_K input rows
  (sift_set_row_origin + sift_detect, num_octaves = K + 1).  Rows at least
  M_K from an interior crop edge are exactly the whole-image rows: the margin
  is the sum of the octaves' vertical radii in input rows (a row of octave o
  reads base rows +-r_o, the base of octave o+1 is octave o's scale S at even
  rows) plus 8 octave-K rows for the extremum test (+-1) and up to five
  refinement moves with their 3x3x3 patches;
* the shard keeps the keypoints whose candidate row it owns and its owned
  rows of the octave-(K+1) base (SIFT_F_EXPORT_NEXT_SEED);
* the owned base rows of all shards, in band order, are the whole base of
  octave K+1; the trailing octaves K+1..O-1 (a few % of the work at 8K: radii
  double per octave, so a band cannot carry their margins) run from it on one
  device (sift_detect_from_seed);
* the keypoints of all shards and the tail, ordered by their candidate
  (octave, scale, y, x) -- the reference's candidate order -- are the
  whole-image keypoints.

K is the deepest octave whose margin fits the thinnest band (scaled by
`max_overhead`), so the redundant halo work stays bounded.

Exchange: the base rows and the keypoint lists are gathered once each
(all_gather over RCCL/xGMI with torch.distributed, or in-process for a single
device driving several shards).  No other data crosses devices.

Two drivers: detect_sharded / detect_sharded_local work on host arrays
(all_gather_object); detect_sharded_device / detect_sharded_device_local keep
the image, keypoints, origins and base rows in HBM (crops are pointer
offsets, all_gather_into_tensor, merge by argsort on the device).  K is
chosen by a cost model of the critical path (octave_cost).
"""
import math
import os
import time

import numpy as np

from . import (F_EXPORT_NEXT_SEED, F_KEYPOINT_ORIGINS, KEYPOINT_DTYPE, make_params, octave_dims, schedule)


def _js_round(v):
    f = math.floor(v)
    return f + 1 if v - f >= 0.5 else f


def octave_radii(params):
    """Blur radius of every (octave, scale) (sift.js:38-44; the octave seed is a copy)."""
    _, sig = schedule(params)
    O, NS = sig.shape
    return [[0 if (o > 0 and s == 0) else int(_js_round(3.0 * sig[o][s])) for s in range(NS)] for o in range(O)]


def margin_rows(radii, K):
    """Input rows a crop needs beyond a band for exact octaves 0..K (see module doc)."""
    d = 0.0
    for o in range(K + 1):
        d += max(radii[o]) * 2.0 ** (o - 1)
    return int(math.ceil(d + 8 * 2.0 ** (K - 1)))


class BandPlan:
    def __init__(self, width, height, num_octaves, K, bands, crops):
        self.width, self.height, self.num_octaves = width, height, num_octaves
        self.K = K                # octaves 0..K on crops; K+1..O-1 from the gathered base
        self.bands = bands        # owned input rows [lo, hi) per shard
        self.crops = crops        # crop input rows [c0, c1) per shard

    @property
    def has_tail(self):
        return self.K + 1 < self.num_octaves

    def __repr__(self):
        return "BandPlan(K=%d, bands=%s, crops=%s)" % (self.K, self.bands, self.crops)


def plan_bands(width, height, params, n_shards, max_overhead=0.5):
    """Owned bands, crops and the split octave K for n_shards shards."""
    O = params.num_octaves
    align = 2 ** (O - 1)
    units = -(-height // align)
    n = max(1, min(int(n_shards), units))
    cuts = [min(height, (units * r // n) * align) for r in range(n + 1)]
    cuts[-1] = height
    bands = [(cuts[r], cuts[r + 1]) for r in range(n)]
    if n == 1:
        return BandPlan(width, height, O, O - 1, bands, [(0, height)])
    band_min = min(hi - lo for lo, hi in bands)
    radii = octave_radii(params)
    k_max = 0
    for k in range(O - 1, -1, -1):
        if margin_rows(radii, k) <= max_overhead * band_min:
            k_max = k
            break

    def crops_for(K):
        M = margin_rows(radii, K)
        step = 2 ** K
        return [(max(0, lo - M) // step * step, min(height, hi + M)) for lo, hi in bands]

    # Among the splits the margin allows, the one with the shortest critical
    # path: the largest crop's octaves 0..K, then the tail K+1..O-1 on one
    # device (shard_cost).  Deeper splits shorten the tail but grow the crops.
    cost = [octave_cost(width, height, radii, o) for o in range(O)]
    best = None
    for K in range(k_max, -1, -1):
        crops = crops_for(K)
        frac = max(c1 - c0 for c0, c1 in crops) / float(height)
        t = frac * sum(cost[:K + 1]) + sum(cost[K + 1:])
        if best is None or t < best[0]:
            best = (t, K, crops)
    forced = os.environ.get("SIFT_SHARD_K")  # experiments: force the split octave (clamped to the margin's bound)
    if forced is not None:
        K = max(0, min(k_max, int(forced)))
        return BandPlan(width, height, O, K, bands, crops_for(K))
    return BandPlan(width, height, O, best[1], bands, best[2])


# Cost model of one octave of a whole W x H input, in seconds on one MI355X:
# per octave pixel, both separable passes of every scale (2r+1 fp64 taps
# each) plus the stores, the extrema scan and the refinement (~90 tap
# equivalents), at ~1.06e-13 s per tap-pixel, plus ~30 us of launch and tail
# latency per octave (fitted to the 4K per-octave kernel times of DESIGN.md
# section 6).
def octave_cost(width, height, radii, o):
    h, w = octave_dims(width, height, o + 1)[o]
    taps = sum(2 * (2 * r + 1) for r in radii[o]) + 90
    return h * w * taps * 1.06e-13 + 30e-6


def _owned(org, lo, hi, last):
    """Keypoints whose candidate row (octave rows, column 2 of org) lies in input rows [lo, hi)."""
    o = org[:, 0]
    y = org[:, 2]
    lo_o = np.where(o == 0, 2 * lo, lo >> np.maximum(o - 1, 0))
    hi_o = np.where(o == 0, 2 * hi, hi >> np.maximum(o - 1, 0))
    keep = y >= lo_o
    if not last:
        keep &= y < hi_o
    return keep


def _tick(timer, key, t0):
    if timer is not None:
        t = time.perf_counter()
        timer[key] = timer.get(key, 0.0) + t - t0
        return t
    return t0


def run_shard(ctx, img, params, plan, r, timer=None):
    """Shard r on ctx: (keypoints, origins, owned rows of the octave-(K+1) base or None).
    timer: optional dict accumulating wall seconds per step."""
    lo, hi = plan.bands[r]
    c0, c1 = plan.crops[r]
    K = plan.K
    last = r == len(plan.bands) - 1
    flags = params.flags | F_KEYPOINT_ORIGINS | (F_EXPORT_NEXT_SEED if plan.has_tail else 0)
    p = make_params(K + 1, params.scales_per_octave, params.min_blur, params.assumed_blur,
                    params.min_interpixel_distance, flags)
    ctx.set_row_origin(c0)
    t0 = time.perf_counter()
    try:
        kp = ctx.detect(img[c0:c1], p)
        t0 = _tick(timer, "detect", t0)
        org = ctx.keypoint_origins()
        t0 = _tick(timer, "origins", t0)
        seed = ctx.next_seed() if plan.has_tail else None
        t0 = _tick(timer, "seed", t0)
    finally:
        ctx.set_row_origin(0)
    keep = _owned(org, lo, hi, last)
    part = None
    if seed is not None:
        s0 = (lo >> K) - (c0 >> K)
        s1 = seed.shape[0] if last else (hi >> K) - (c0 >> K)
        part = np.ascontiguousarray(seed[s0:s1])
    out = kp[keep], org[keep], part
    _tick(timer, "filter", t0)
    return out


def run_tail(ctx, base, params, plan):
    """Octaves K+1..O-1 of the whole image from the gathered octave-(K+1) base."""
    p = make_params(params.num_octaves, params.scales_per_octave, params.min_blur, params.assumed_blur,
                    params.min_interpixel_distance, params.flags | F_KEYPOINT_ORIGINS)
    h, w = octave_dims(plan.width, plan.height, plan.num_octaves)[plan.K + 1]
    if base.shape != (h, w):
        raise ValueError("gathered base %s != octave %d dims %s" % (base.shape, plan.K + 1, (h, w)))
    kp = ctx.detect_from_seed(base, plan.K + 1, plan.width, plan.height, p)
    return kp, ctx.keypoint_origins()


def merge(parts):
    """Keypoints of all shards (+ tail) in the reference's candidate order."""
    kps = [k for k, _ in parts if len(k)]
    if not kps:
        return np.zeros(0, dtype=KEYPOINT_DTYPE)
    kp = np.concatenate(kps)
    org = np.concatenate([o for k, o in parts if len(k)])
    order = np.lexsort((org[:, 3], org[:, 2], org[:, 1], org[:, 0]))
    return kp[order]


def detect_sharded_local(ctx, img, params, n_shards, max_overhead=0.5):
    """All shards on one context in turn (one device): the sharded algorithm
    without the collectives -- a parity harness and a single-device fallback."""
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape
    plan = plan_bands(W, H, params, n_shards, max_overhead)
    parts, seeds = [], []
    for r in range(len(plan.bands)):
        kp, org, seed = run_shard(ctx, img, params, plan, r)
        parts.append((kp, org))
        seeds.append(seed)
    if plan.has_tail:
        parts.append(run_tail(ctx, np.concatenate(seeds), params, plan))
    return merge(parts), plan


def detect_sharded(ctx, img, params, group=None, max_overhead=0.5):
    """One shard per rank of torch.distributed (RCCL on ROCm): every rank
    passes the same image; all ranks return the whole image's keypoints.
    Two gathers: the owned base rows (then the tail runs on rank 0) and the
    keypoint lists."""
    import torch.distributed as dist
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    plan = plan_bands(W, H, params, world, max_overhead)
    mine = []
    seed = None
    if rank < len(plan.bands):
        kp, org, seed = run_shard(ctx, img, params, plan, rank)
        mine.append((kp, org))
    if plan.has_tail:
        seeds = [None] * world
        dist.all_gather_object(seeds, seed, group=group)
        if rank == 0:
            base = np.concatenate([s for s in seeds if s is not None])
            mine.append(run_tail(ctx, base, params, plan))
    gathered = [None] * world
    dist.all_gather_object(gathered, mine, group=group)
    return merge([p for g in gathered for p in g]), plan


# ---------------------------------------------------------------------------
# Device-resident driver: the image, the crops (pointer offsets into the
# whole image), the keypoints, their origins and the base rows stay in HBM;
# owned-row filtering and the ordered merge are torch ops on the device, the
# gathers are all_gather_into_tensor over RCCL.  Records are 48-byte
# sift_keypoint rows of a uint8 tensor.
# ---------------------------------------------------------------------------
REC = KEYPOINT_DTYPE.itemsize


def _seed_rows(plan, r):
    """Rows [s0, s1) of shard r's octave-(K+1) base that it owns, in its crop's rows."""
    lo, hi = plan.bands[r]
    c0, c1 = plan.crops[r]
    K = plan.K
    h_crop = octave_dims(plan.width, c1 - c0, K + 2)[K + 1][0]
    s0 = (lo >> K) - (c0 >> K)
    s1 = h_crop if r == len(plan.bands) - 1 else (hi >> K) - (c0 >> K)
    return s0, s1


def _device_lists(ctx, n, torch, dev):
    kp = torch.empty((max(n, 1), REC), dtype=torch.uint8, device=dev)
    org = torch.empty((max(n, 1), 4), dtype=torch.int32, device=dev)
    if n:
        ctx.copy_keypoints_device(kp.data_ptr(), n)
        ctx.copy_keypoint_origins_device(org.data_ptr(), 4 * n)
    return kp[:n], org[:n]


def torch_ready(t):
    """Wait until torch's work producing `t` is done.  The C ABI runs on its
    own HIP stream (another runtime instance than torch's), which nothing
    orders after torch's stream: every sift_* call that reads a buffer torch
    wrote (the image, a gathered base) must come after this."""
    if t.is_cuda:
        import torch
        torch.cuda.current_stream(t.device).synchronize()


def _device_keypoints(ctx, n, torch, dev):
    kp = torch.empty((max(n, 1), REC), dtype=torch.uint8, device=dev)
    if n:
        ctx.copy_keypoints_device(kp.data_ptr(), n)
    return kp[:n]


def run_shard_device(ctx, d_img, params, plan, r):
    """Shard r from the whole image `d_img` (H x W fp32 torch tensor on ctx's
    device): (keypoints uint8 [n, 48] on the device -- only those whose
    candidate row the shard owns, filtered in the library's compaction
    (sift_set_owned_rows) --, their counts per (octave, scale) block (int64
    numpy [K+1 octaves * S]), owned rows of the octave-(K+1) base fp64
    [rows, cols] on the device or None).  The sift_* copies into the returned
    tensors complete before they return, so torch may read them at once."""
    import torch
    dev = d_img.device
    torch_ready(d_img)
    lo, hi = plan.bands[r]
    c0, c1 = plan.crops[r]
    K = plan.K
    last = r == len(plan.bands) - 1
    W = plan.width
    flags = params.flags | (F_EXPORT_NEXT_SEED if plan.has_tail else 0)
    p = make_params(K + 1, params.scales_per_octave, params.min_blur, params.assumed_blur,
                    params.min_interpixel_distance, flags)
    ctx.set_row_origin(c0)
    ctx.set_owned_rows(lo, -1 if last else hi)
    try:
        n = ctx.detect_device(d_img.data_ptr() + c0 * W * 4, W, c1 - c0, p)
        kp = _device_keypoints(ctx, n, torch, dev)
        counts = ctx.block_counts()
        part = None
        if plan.has_tail:
            s0, s1 = _seed_rows(plan, r)
            rows, cols = ctx.next_seed_dims()
            part = torch.empty((s1 - s0, cols), dtype=torch.float64, device=dev)
            ctx.copy_next_seed_device(part.data_ptr(), part.numel(), s0, s1)
    finally:
        ctx.set_row_origin(0)
        ctx.set_owned_rows(-1)
    return kp, counts, part


def run_tail_device(ctx, d_base, params, plan):
    """Octaves K+1..O-1 from the gathered base (fp64 torch tensor on the device)."""
    import torch
    p = make_params(params.num_octaves, params.scales_per_octave, params.min_blur, params.assumed_blur,
                    params.min_interpixel_distance, params.flags | F_KEYPOINT_ORIGINS)
    h, w = octave_dims(plan.width, plan.height, plan.num_octaves)[plan.K + 1]
    if tuple(d_base.shape) != (h, w):
        raise ValueError("gathered base %s != octave %d dims %s" % (tuple(d_base.shape), plan.K + 1, (h, w)))
    d_base = d_base.contiguous()
    torch_ready(d_base)  # the all-gather / concatenation that made it is only enqueued on torch's stream
    n = ctx.detect_from_seed_device(d_base.data_ptr(), plan.K + 1, plan.width, plan.height, p)
    return _device_lists(ctx, n, torch, d_base.device)


def tail_octaves(plan, world):
    """Tail octave -> rank: the trailing octaves K+1..O-1 are detected one per
    rank; each rank builds the tail's Gaussian chain only as far as its octave
    (sift_detect_from_seed_range_device), so the deepest octave is the
    longest piece.  The deepest go to the ranks with the smallest crops (the
    first and last bands carry a margin on one side only)."""
    if not plan.has_tail:
        return {}
    n = len(plan.crops)
    ranks = sorted(range(min(world, n)), key=lambda r: (plan.crops[r][1] - plan.crops[r][0], r))
    tail = list(range(plan.num_octaves - 1, plan.K, -1))
    return {t: ranks[i % len(ranks)] for i, t in enumerate(tail)}


def run_tail_octave_device(ctx, d_base, params, plan, t):
    """Keypoints of tail octave t alone (uint8 [n, 48] on the device) and
    their block counts, from the gathered octave-(K+1) base: octaves K+1..t
    are built, only t is scanned (sift_detect_from_seed_range_device)."""
    import torch
    p = make_params(t + 1, params.scales_per_octave, params.min_blur, params.assumed_blur,
                    params.min_interpixel_distance, params.flags)
    h, w = octave_dims(plan.width, plan.height, plan.num_octaves)[plan.K + 1]
    if tuple(d_base.shape) != (h, w):
        raise ValueError("gathered base %s != octave %d dims %s" % (tuple(d_base.shape), plan.K + 1, (h, w)))
    d_base = d_base.contiguous()
    torch_ready(d_base)  # the all-gather / concatenation that made it is only enqueued on torch's stream
    n = ctx.detect_from_seed_range_device(d_base.data_ptr(), plan.K + 1, t, plan.width, plan.height, p)
    return _device_keypoints(ctx, n, torch, d_base.device), ctx.block_counts()


def _blocks(counts, O, S):
    """Block counts of a part padded to all O * S blocks (a band or tail part
    covers only its leading octaves)."""
    out = np.zeros(O * S, dtype=np.int64)
    out[:len(counts)] = counts
    return out


def merge_device(ctx, kps, counts, O, S):
    """Ordered merge without a sort: parts are row bands in row order (plus
    tail octaves), each sorted by candidate (octave, scale, y, x), so the
    reference's order is block-major over (octave, scale), then part order
    (sift_merge_keypoint_blocks_device).  counts: per part, its keypoints per
    block (host)."""
    import torch
    kp = torch.cat(kps).contiguous() if len(kps) > 1 else kps[0].contiguous()
    out = torch.empty_like(kp)
    if kp.shape[0]:
        torch_ready(kp)
        ctx.merge_keypoint_blocks_device(kp.data_ptr(), np.stack([_blocks(c, O, S) for c in counts]),
                                         out.data_ptr())
    return out


def _sync(t):
    if t.is_cuda:
        import torch
        torch.cuda.synchronize(t.device)


def detect_sharded_device_local(ctx, d_img, params, n_shards, max_overhead=0.5, timer=None):
    """All shards on one device in turn (device-resident): the sharded
    algorithm without the collectives -- one rank's band after another, then
    every tail octave as its own piece, then the block merge.  Returns (uint8
    [n, 48] keypoints on the device, plan).  timer: optional dict of per-part
    seconds (each part synchronised, so the parts can be summed into a
    modelled critical path)."""
    import torch
    H, W = d_img.shape
    O, S = params.num_octaves, params.scales_per_octave
    plan = plan_bands(W, H, params, n_shards, max_overhead)
    kps, counts, seeds = [], [], []
    for r in range(len(plan.bands)):
        t0 = time.perf_counter()
        kp, cnt, seed = run_shard_device(ctx, d_img, params, plan, r)
        _sync(d_img)
        _tick(timer, "shard%d" % r, t0)
        kps.append(kp)
        counts.append(cnt)
        seeds.append(seed)
    tkps, tcounts = [], []
    if plan.has_tail:
        base = torch.cat(seeds)
        for t in sorted(tail_octaves(plan, len(plan.bands))):
            t0 = time.perf_counter()
            kp, cnt = run_tail_octave_device(ctx, base, params, plan, t)
            _sync(d_img)
            _tick(timer, "tail%d" % t, t0)
            tkps.append(kp)
            tcounts.append(cnt)
    # The parts laid out as the all-gathers leave them (padded to the largest
    # part), then the distributed driver's merge: bands, then tail octaves.
    band = _pad_parts(kps, d_img.device)
    tail = _pad_parts(tkps, d_img.device) if tkps else None
    nb = int(sum(int(np.sum(c)) for c in counts))
    nt = int(sum(int(np.sum(c)) for c in tcounts))
    out = torch.empty((nb + nt, REC), dtype=torch.uint8, device=d_img.device)
    _sync(d_img)
    t0 = time.perf_counter()
    _merge_padded(ctx, band[0], band[1], np.stack([_blocks(c, O, S) for c in counts]), out[:nb])
    if tail is not None:
        _merge_padded(ctx, tail[0], tail[1], np.stack([_blocks(c, O, S) for c in tcounts]), out[nb:])
    _sync(d_img)
    _tick(timer, "merge", t0)
    return out, plan


def _pad_parts(parts, dev):
    """Parts laid out back to back at the stride of the largest (the layout
    gather_rows_start's all-gather leaves), as (buffer, stride)."""
    import torch
    m = max(max(p.shape[0] for p in parts), 1)
    buf = torch.zeros((len(parts) * m, REC), dtype=torch.uint8, device=dev)
    for i, p in enumerate(parts):
        buf[i * m:i * m + p.shape[0]] = p
    return buf, m


def _merge_padded(ctx, buf, m, blocks, out):
    """Block-major merge of parts stored at stride m in buf (blocks: int64
    [parts, O*S] per-part block counts) into out: each part's padding is a
    trailing negative count, skipped by the merge (no strip copy)."""
    blocks = np.asarray(blocks, dtype=np.int64)
    n = blocks.sum(axis=1)
    if int(n.sum()) == 0:
        return
    ext = np.zeros((blocks.shape[0], blocks.shape[1] + 1), dtype=np.int64)
    ext[:, :-1] = blocks
    ext[:, -1] = -(m - n)
    torch_ready(buf)
    ctx.merge_keypoint_blocks_device(buf.data_ptr(), ext, out.data_ptr())


def gather_rows_start(t, counts, group=None):
    """Start an all_gather of a ragged first dimension (every rank knows all
    counts): pad to the largest, all_gather_into_tensor with async_op (under
    nccl it runs on RCCL's own stream, beside later work on the library's
    stream).  gather_rows_finish waits and strips."""
    import torch
    import torch.distributed as dist
    world = len(counts)
    m = max(max(counts), 1)
    send = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    send[:t.shape[0]] = t
    recv = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    work = dist.all_gather_into_tensor(recv, send, group=group, async_op=True)
    return work, recv, m, list(counts), send


def gather_rows_finish(pending):
    """The rank-order concatenation of a gather_rows_start."""
    import torch
    work, recv, m, counts, _send = pending
    work.wait()
    return torch.cat([recv[i * m:i * m + counts[i]] for i in range(len(counts))])


def gather_rows(t, counts, group=None):
    """all_gather of a ragged first dimension: the rank-order concatenation."""
    return gather_rows_finish(gather_rows_start(t, counts, group))


_SIDE_GROUPS = {}


def side_group(group=None):
    """A second communicator over the ranks of `group` (created collectively
    on first use; every rank calls detect_sharded_device).  RCCL runs the
    collectives of one communicator in issue order on one stream, so the band
    keypoints' all-gather (10.9 MB per rank at 8K) issued on the main group
    would hold back the base all-gather every tail octave waits for; on its
    own communicator it runs beside the base gather and the tail octaves."""
    import torch.distributed as dist
    # The cache holds the group object it was made for (so its id cannot be
    # reused while cached) and, for the default world, the world group of the
    # time: a destroy_process_group / init_process_group cycle makes a new
    # world, and the stale side communicator is dropped, not reused.
    owner = group if group is not None else dist.distributed_c10d._get_default_group()
    key = id(group) if group is not None else None
    ent = _SIDE_GROUPS.get(key)
    if ent is not None and ent[0] is owner:
        return ent[1]
    if group is None:
        g = dist.new_group()
    else:  # only the group's ranks call this
        g = dist.new_group(ranks=dist.get_process_group_ranks(group), use_local_synchronization=True)
    _SIDE_GROUPS[key] = (owner, g)
    return g


def _gather_counts(cnt, world, group, dev):
    """Every rank's per-(octave, scale) block counts (int64 [world, O*S] host)."""
    import torch
    import torch.distributed as dist
    mine = torch.from_numpy(np.asarray(cnt, dtype=np.int64)).to(dev)
    out = torch.zeros(world * mine.numel(), dtype=torch.int64, device=mine.device)
    dist.all_gather_into_tensor(out, mine, group=group)
    return out.view(world, -1).cpu().numpy()


def detect_sharded_device(ctx, d_img, params, group=None, max_overhead=0.5, timer=None):
    """One shard per rank, device-resident (RCCL with the nccl backend).
    Rank r runs its row band (octaves 0..K, keypoints of its own rows), the
    owned rows of the octave-(K+1) base are all-gathered, every tail octave is
    detected by one rank (tail_octaves: the deepest on the smallest crops), then the per-(octave, scale) counts and
    the keypoints are all-gathered and merged block-major (no sort).  Every
    rank returns the whole image's keypoints (uint8 [n, 48] on its device) in
    the reference's order."""
    import torch
    import torch.distributed as dist
    H, W = d_img.shape
    O, S = params.num_octaves, params.scales_per_octave
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = d_img.device
    plan = plan_bands(W, H, params, world, max_overhead)
    nb = len(plan.bands)
    t0 = time.perf_counter()
    if rank < nb:
        kp, cnt, seed = run_shard_device(ctx, d_img, params, plan, rank)
    else:
        kp, cnt, seed = torch.zeros((0, REC), dtype=torch.uint8, device=dev), np.zeros(0, np.int64), None
    t0 = _tick(timer, "band", t0)
    # The band keypoints' all-gather starts as soon as the bands are done and
    # runs on its own communicator (side_group: its own RCCL stream) while the
    # base all-gather and the tail octaves run; only the (few) tail keypoints
    # are gathered after the tail.  The merge takes the band parts, then the
    # tail parts: no block holds both (the tail octaves are K+1..O-1), so
    # block-major-then-part order is unchanged.
    band_counts = _gather_counts(_blocks(cnt, O, S), world, group, dev)
    band = gather_rows_start(kp, [int(c) for c in band_counts.sum(axis=1)],
                             side_group(group) if plan.has_tail else group)
    nb_kp = int(band_counts.sum())
    if not plan.has_tail:
        band[0].wait()
        t0 = _tick(timer, "kp_gather", t0)
        out = torch.empty((nb_kp, REC), dtype=torch.uint8, device=dev)
        _merge_padded(ctx, band[1], band[2], band_counts, out)
        _tick(timer, "merge", t0)
        return out, plan
    cols = octave_dims(W, H, plan.num_octaves)[plan.K + 1][1]
    rows = [(lambda a: a[1] - a[0])(_seed_rows(plan, r)) if r < nb else 0 for r in range(world)]
    mine = seed if seed is not None else torch.zeros((0, cols), dtype=torch.float64, device=dev)
    base = gather_rows(mine, rows, group)
    t0 = _tick(timer, "base_gather", t0)
    tkps, tcnts = [torch.zeros((0, REC), dtype=torch.uint8, device=dev)], [np.zeros(O * S, np.int64)]
    for t, owner in sorted(tail_octaves(plan, world).items()):  # a rank's list stays in block order
        if owner == rank:
            tk, tc = run_tail_octave_device(ctx, base, params, plan, t)
            tkps.append(tk)
            tcnts.append(_blocks(tc, O, S))
    t0 = _tick(timer, "tail", t0)
    tail_counts = _gather_counts(np.sum(tcnts, axis=0), world, group, dev)
    tail = gather_rows_start(torch.cat(tkps), [int(c) for c in tail_counts.sum(axis=1)], group)
    tail[0].wait()
    band[0].wait()
    t0 = _tick(timer, "kp_gather", t0)
    # The gathered lists stay padded (a trailing negative count per rank skips
    # the padding); the band blocks (octaves 0..K) precede the tail blocks
    # (octaves K+1..O-1) in block order, so the two merges fill out in turn.
    out = torch.empty((nb_kp + int(tail_counts.sum()), REC), dtype=torch.uint8, device=dev)
    _merge_padded(ctx, band[1], band[2], band_counts, out[:nb_kp])
    _merge_padded(ctx, tail[1], tail[2], tail_counts, out[nb_kp:])
    _tick(timer, "merge", t0)
    return out, plan
