"""Row-band sharding of one image (sift_amd/shard.py, SURVEY.md §8e cfg 5):
the band plan, candidate ownership, the ordered merge, and the two gathers
of detect_sharded over torch.distributed (gloo, world size 2) with a stand-in
context.  The GPU parity of the whole scheme (merged shards == whole image,
bit for bit) is tests/test_gpu_parity.py::test_row_band_shards_match_whole_image."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import sift_amd
from sift_amd import KEYPOINT_DTYPE, octave_dims
from sift_amd.shard import _owned, margin_rows, merge, octave_radii, plan_bands


@pytest.mark.parametrize("W,H,O,S,n,ov", [
    (480, 360, 4, 3, 2, 0.5), (640, 600, 5, 3, 4, 4.0), (7680, 4320, 6, 5, 8, 0.5),
    (7680, 4320, 6, 5, 2, 0.5), (512, 520, 4, 5, 5, 0.05), (100, 37, 3, 3, 9, 0.5), (64, 64, 2, 3, 1, 0.5),
])
def test_plan_invariants(W, H, O, S, n, ov):
    p = sift_amd.make_params(O, S)
    plan = plan_bands(W, H, p, n, ov)
    align = 2 ** (O - 1)
    assert plan.bands[0][0] == 0 and plan.bands[-1][1] == H
    for (lo, hi), (lo2, _) in zip(plan.bands, plan.bands[1:]):
        assert hi == lo2 and lo % align == 0 and hi % align == 0 and hi > lo
    M = margin_rows(octave_radii(p), plan.K) if len(plan.bands) > 1 else 0
    for (lo, hi), (c0, c1) in zip(plan.bands, plan.crops):
        assert c0 % (2 ** plan.K) == 0 and 0 <= c0 <= lo and hi <= c1 <= H
        assert c0 == 0 or lo - c0 >= M
        assert c1 == H or c1 - hi >= M
    assert 0 <= plan.K <= O - 1


def test_ownership_partitions_candidates():
    p = sift_amd.make_params(5, 3)
    H = 600
    plan = plan_bands(640, H, p, 4, 0.5)
    dims = octave_dims(640, H, 5)
    rng = np.random.default_rng(1)
    rows = []
    for o in range(5):
        y = rng.integers(1, dims[o][0] - 1, 200)
        rows.append(np.stack([np.full_like(y, o), np.ones_like(y), y, np.ones_like(y)], axis=1))
    org = np.concatenate(rows).astype(np.int32)
    owned = np.stack([_owned(org, lo, hi, r == len(plan.bands) - 1) for r, (lo, hi) in enumerate(plan.bands)])
    np.testing.assert_array_equal(owned.sum(axis=0), 1)


def _fake_truth(W, H, O, n=400, seed=0):
    """Whole-image keypoints with their candidate origins, reference order."""
    rng = np.random.default_rng(seed)
    dims = octave_dims(W, H, O)
    org = []
    for o in range(O):
        h, w = dims[o]
        m = n >> o
        org.append(np.stack([np.full(m, o), rng.integers(1, 4, m), rng.integers(1, h - 1, m),
                             rng.integers(1, w - 1, m)], axis=1))
    org = np.concatenate(org).astype(np.int32)
    org = org[np.lexsort((org[:, 3], org[:, 2], org[:, 1], org[:, 0]))]
    kp = np.zeros(org.shape[0], dtype=KEYPOINT_DTYPE)
    kp["octave"], kp["scale_level"], kp["local_y"], kp["local_x"] = org[:, 0], org[:, 1], org[:, 2], org[:, 3]
    kp["abs_x"] = np.arange(org.shape[0]) * 0.25
    return kp, org


class FakeCtx:
    """Stand-in for sift_amd.Context: 'detects' the truth restricted to what a
    crop (rows) / a tail run (octaves) would produce, and exports a base whose
    column 0 is the global row index, so the gathered base can be checked."""

    def __init__(self, W, H, O):
        self.W, self.H, self.O = W, H, O
        self.kp, self.org = _fake_truth(W, H, O)
        self.row0 = 0
        self.last = None

    def set_row_origin(self, r):
        self.row0 = r

    def detect(self, img, p):
        K = p.num_octaves - 1
        c0, c1 = self.row0, self.row0 + img.shape[0]
        o, y = self.org[:, 0], self.org[:, 2]
        lo = np.where(o == 0, 2 * c0, c0 >> np.maximum(o - 1, 0))
        hi = np.where(o == 0, 2 * c1, c1 >> np.maximum(o - 1, 0))
        sel = (o <= K) & (y >= lo) & (y < hi)
        self.last = sel
        self.K = K
        self.crop = (c0, c1)
        return self.kp[sel]

    def keypoint_origins(self):
        return self.org[self.last]

    def next_seed(self):
        c0, c1 = self.crop
        w = octave_dims(self.W, self.H, self.O)[self.K + 1][1]
        rows = -(-(c1 - c0) // 2 ** self.K)
        base = np.zeros((rows, w))
        base[:, 0] = (c0 >> self.K) + np.arange(rows)
        return base

    def detect_from_seed(self, base, o_first, W, H, p):
        np.testing.assert_array_equal(base[:, 0], np.arange(base.shape[0]))
        sel = self.org[:, 0] >= o_first
        self.last = sel
        return self.kp[sel]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, shape, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sift_amd.shard import detect_sharded
        W, H, O, S = shape
        ctx = FakeCtx(W, H, O)
        merged, plan = detect_sharded(ctx, np.zeros((H, W), np.float32), sift_amd.make_params(O, S))
        out_q.put((rank, merged.tobytes(), ctx.kp.tobytes(), plan.K))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shape", [(480, 360, 4, 3), (7680, 4320, 6, 5)])
def test_detect_sharded_gathers_world2(shape):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, merged, truth, K in res:
        assert merged == truth, "rank %d: merged shards differ from the whole image" % rank
        assert K < shape[2] - 1 or shape[2] == 1  # the tail path ran


def test_merge_orders_by_candidate():
    kp, org = _fake_truth(320, 240, 3, n=50, seed=2)
    perm = np.random.default_rng(0).permutation(kp.shape[0])
    a, b = perm[: len(perm) // 2], perm[len(perm) // 2:]
    m = merge([(kp[a], org[a]), (kp[b], org[b]), (kp[:0], org[:0])])
    assert m.tobytes() == kp.tobytes()


class FakeDeviceCtx(FakeCtx):
    """The device-resident interface of sift_amd.Context over CPU tensors:
    'device pointers' are host addresses of CPU tensors (ctypes.memmove)."""
    own = (-1, -1)

    def set_owned_rows(self, lo, hi=-1):
        self.own = (lo, hi)

    def _blocks(self, p):
        o, s = self.org[self.last, 0], self.org[self.last, 1]
        return np.bincount(o * p.scales_per_octave + s - 1,
                           minlength=p.num_octaves * p.scales_per_octave).astype(np.int64)

    def detect_device(self, ptr, W, h, p):
        self.detect(np.zeros((h, W), np.float32), p)
        lo, hi = self.own
        if lo >= 0:
            self.last &= _owned(self.org, lo, hi, hi < 0)
        self.blk = self._blocks(p)
        return int(self.last.sum())

    def block_counts(self):
        return self.blk

    def copy_keypoints_device(self, ptr, cap):
        import ctypes
        b = self.kp[self.last].tobytes()
        ctypes.memmove(ptr, b, len(b))
        return int(self.last.sum())

    def copy_keypoint_origins_device(self, ptr, cap):
        import ctypes
        b = np.ascontiguousarray(self.org[self.last], dtype=np.int32).tobytes()
        ctypes.memmove(ptr, b, len(b))
        return int(self.last.sum())

    def next_seed_dims(self):
        b = self.next_seed()
        return b.shape

    def copy_next_seed_device(self, ptr, cap, s0, s1):
        import ctypes
        b = np.ascontiguousarray(self.next_seed()[s0:s1]).tobytes()
        ctypes.memmove(ptr, b, len(b))

    def detect_from_seed_device(self, ptr, o_first, W, H, p):
        import ctypes
        h, w = octave_dims(W, H, self.O)[o_first]
        base = np.frombuffer((ctypes.c_double * (h * w)).from_address(ptr), dtype=np.float64).reshape(h, w)
        self.detect_from_seed(base.copy(), o_first, W, H, p)
        return int(self.last.sum())

    def detect_from_seed_range_device(self, ptr, o_first, o_scan, W, H, p):
        self.detect_from_seed_device(ptr, o_first, W, H, p)
        o = self.org[:, 0]
        self.last = (o >= o_scan) & (o < p.num_octaves)
        self.blk = self._blocks(p)
        return int(self.last.sum())

    def merge_keypoint_blocks_device(self, d_in, counts, d_out):
        import ctypes
        counts = np.asarray(counts, dtype=np.int64)
        n = int(np.abs(counts).sum())
        buf = np.frombuffer(ctypes.string_at(d_in, n * 48), dtype=np.uint8).reshape(n, 48)
        parts, off = [], 0
        for q in range(counts.shape[0]):
            blocks = []
            for b in range(counts.shape[1]):
                c = counts[q, b]
                blocks.append(buf[off:off + max(c, 0)])  # negative: skipped padding
                off += abs(c)
            parts.append(blocks)
        out = np.concatenate([parts[q][b] for b in range(counts.shape[1]) for q in range(counts.shape[0])])
        ctypes.memmove(d_out, out.tobytes(), out.nbytes)


@pytest.mark.parametrize("shape,n", [((480, 360, 4, 3), 3), ((7680, 4320, 6, 5), 8), ((640, 600, 5, 3), 1)])
def test_device_driver_local_with_stand_in(shape, n):
    """detect_sharded_device_local (torch ops for filtering and the ordered
    merge) reproduces the whole image with a stand-in context on CPU tensors."""
    import torch
    W, H, O, S = shape
    ctx = FakeDeviceCtx(W, H, O)
    from sift_amd.shard import detect_sharded_device_local
    merged, plan = detect_sharded_device_local(ctx, torch.zeros((H, W), dtype=torch.float32),
                                               sift_amd.make_params(O, S), n)
    assert merged.numpy().tobytes() == ctx.kp.tobytes()


def _worker_device(rank, world, port, shape, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from sift_amd.shard import detect_sharded_device
        W, H, O, S = shape
        ctx = FakeDeviceCtx(W, H, O)
        merged, plan = detect_sharded_device(ctx, torch.zeros((H, W), dtype=torch.float32),
                                             sift_amd.make_params(O, S))
        out_q.put((rank, merged.numpy().tobytes(), ctx.kp.tobytes(), plan.K))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("shape,world", [((480, 360, 4, 3), 2), ((7680, 4320, 6, 5), 2),
                                         ((7680, 4320, 6, 5), 3), ((1920, 1080, 5, 5), 3),
                                         ((7680, 4320, 6, 5), 8), ((480, 360, 4, 3), 8)])
def test_detect_sharded_device_gathers(shape, world):
    """The device-resident driver's gathers (all_gather_into_tensor of the
    padded base rows, counts, records and origins; the band keypoints on a
    second communicator) over gloo at world sizes 2, 3 and 8.  At 8K O6 on 8
    ranks three ranks own the tail octaves 3/4/5 and five own bands only, and
    the merge interleaves 8 parts block-major: patterns world size 2 cannot
    exercise."""
    from sift_amd.shard import plan_bands, tail_octaves
    W, H, O, S = shape
    plan = plan_bands(W, H, sift_amd.make_params(O, S), world, 0.5)
    owners = set(tail_octaves(plan, world).values()) if plan.has_tail else set()
    assert len(plan.bands) == world
    if world >= 3:
        assert len(owners) >= 2  # several tail owners
    if world == 8:
        assert len(owners) < world  # and band-only ranks
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_device, args=(r, world, port, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, merged, truth, K in res:
        assert merged == truth, "rank %d: merged shards differ from the whole image" % rank


def test_merge_device_equals_sort():
    """The sort-free block-major device merge (sift_merge_keypoint_blocks_device,
    stand-in context) equals a full sort by candidate on ragged parts that own
    disjoint row ranges per (octave, scale), plus tail octaves."""
    import torch
    from sift_amd.shard import merge_device
    kp, org = _fake_truth(640, 600, 5, n=300, seed=4)
    ctx = FakeDeviceCtx(640, 600, 5)
    # split octaves 0..2 into 3 row bands, octaves 3..4 = tail
    parts = []
    for lo, hi in ((0, 100), (100, 250), (250, 10 ** 6)):
        sel = (org[:, 0] <= 2) & (org[:, 2] >= lo) & (org[:, 2] < hi)
        parts.append(sel)
    parts.append(org[:, 0] > 2)
    kps = [torch.from_numpy(np.frombuffer(kp[m].tobytes(), np.uint8).reshape(-1, 48).copy()) for m in parts]
    orgs = [torch.from_numpy(org[m].copy()) for m in parts]
    kps.insert(1, kps[0][:0])
    orgs.insert(1, orgs[0][:0])
    counts = [np.bincount(o[:, 0].numpy() * 3 + o[:, 1].numpy() - 1, minlength=15) for o in orgs]
    out = merge_device(ctx, kps, counts, 5, 3)
    assert out.numpy().tobytes() == kp.tobytes()
