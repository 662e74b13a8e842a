"""Multi-GPU batch sharding: one process per GPU, RCCL keypoint all-gather.

SURVEY.md §8(e): independent images shard across ranks with no exchange
until the end; the only collective is the all-gather of the per-image
keypoint lists (ragged: counts first, then records padded to the largest
count).  torch.distributed with backend "nccl" is RCCL over xGMI on the GPU
box; the same code runs on "gloo" with CPU tensors in the tests.

Keypoint records are the 48-byte sift_keypoint (include/sift_hip.h), carried
as raw uint8 rows so no reinterpretation happens on the wire.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import KEYPOINT_DTYPE

REC = KEYPOINT_DTYPE.itemsize


def shard_images(n_images, world, rank):
    """Contiguous block of image indices for `rank` (weak scaling when
    n_images = world * per_rank)."""
    per, extra = divmod(n_images, world)
    start = rank * per + min(rank, extra)
    return list(range(start, start + per + (1 if rank < extra else 0)))


class KeypointGather:
    """Reusable all-gather of one ragged keypoint list per rank.

    `fill(buf, cap)` writes this rank's records into `buf` (uint8 tensor of
    cap*REC bytes, on `device`) and returns the count -- e.g. a device-to-
    device copy from the HIP context (sift_copy_keypoints_device)."""

    def __init__(self, device, group=None):
        self.device = torch.device(device)
        self.group = group
        self.world = dist.get_world_size(group)
        self.cap = 0
        self.send = None
        self.recv = None

    def _ensure(self, cap):
        if cap <= self.cap:
            return
        cap = max(cap, 1)
        cap += cap // 4
        self.send = torch.zeros(cap * REC, dtype=torch.uint8, device=self.device)
        self.recv = torch.zeros(self.world * cap * REC, dtype=torch.uint8, device=self.device)
        self.cap = cap

    def __call__(self, n_local, fill):
        cnt = torch.tensor([int(n_local)], dtype=torch.int64, device=self.device)
        cnts = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(cnts, cnt, group=self.group)
        counts = [int(c) for c in cnts.tolist()]
        self._ensure(max(counts))
        n = fill(self.send, self.cap)
        assert n == n_local, (n, n_local)
        dist.all_gather_into_tensor(self.recv, self.send, group=self.group)
        return counts

    def gathered(self, counts):
        """Host view: concatenation of every rank's records in rank order."""
        raw = self.recv.view(self.world, self.cap * REC).cpu().numpy()
        parts = [np.frombuffer(raw[r, :counts[r] * REC].tobytes(), dtype=KEYPOINT_DTYPE) for r in range(self.world)]
        return np.concatenate(parts) if parts else np.zeros(0, dtype=KEYPOINT_DTYPE)


class PipelinedKeypointGather:
    """The same all-gather, overlapped with the detections that follow.

    Per step the counts are all-gathered synchronously (8 B per rank), then
    the records all-gather is only enqueued (async_op) and this step's
    buffers are left to it; a ring of `depth` send / receive buffers keeps
    `depth - 1` record gathers in flight while the GPU keeps detecting.  A
    slot is reused only after its gather has completed on the device and the
    host has seen that (the next fill writes the send buffer from another HIP
    runtime's stream, which nothing else orders after RCCL's).  `drain()`
    completes every outstanding gather; `gathered(k)` is the host view of the
    step k slots back (after drain)."""

    def __init__(self, device, group=None, depth=3):
        self.device = torch.device(device)
        self.group = group
        self.world = dist.get_world_size(group)
        self.depth = max(1, int(depth))
        self.slots = [{"cap": 0, "send": None, "recv": None, "work": None, "counts": None, "m": 0}
                      for _ in range(self.depth)]
        self.k = 0

    def _settle(self, slot):
        if slot["work"] is not None:
            slot["work"].wait()
            if self.device.type == "cuda":
                torch.cuda.current_stream(self.device).synchronize()
            slot["work"] = None

    def __call__(self, n_local, fill):
        cnt = torch.tensor([int(n_local)], dtype=torch.int64, device=self.device)
        cnts = torch.zeros(self.world, dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(cnts, cnt, group=self.group)
        counts = [int(c) for c in cnts.tolist()]
        slot = self.slots[self.k % self.depth]
        self.k += 1
        self._settle(slot)
        need = max(max(counts), 1)
        if need > slot["cap"]:
            cap = need + need // 4
            slot["send"] = torch.zeros(cap * REC, dtype=torch.uint8, device=self.device)
            slot["recv"] = torch.zeros(self.world * cap * REC, dtype=torch.uint8, device=self.device)
            slot["cap"] = cap
        n = fill(slot["send"], slot["cap"])
        assert n == n_local, (n, n_local)
        # only the step's largest count goes on the wire (the buffers keep
        # 1/4 slack for growth; at N = 8 the slack alone would be 7 x 5 MB per
        # 4K step): every rank receives (N - 1) x need records
        m = need * REC
        slot["m"] = m
        slot["work"] = dist.all_gather_into_tensor(slot["recv"][:self.world * m], slot["send"][:m],
                                                   group=self.group, async_op=True)
        slot["counts"] = counts
        return counts

    def drain(self):
        for slot in self.slots:
            self._settle(slot)

    def gathered(self, back=1):
        """Host view of the step `back` steps ago (1 = the last), rank order.
        Only the last min(steps run, depth) steps are held: an older step's
        slot has been reused."""
        if not 1 <= back <= min(self.k, self.depth):
            raise ValueError("gathered(back=%d): only the last %d step(s) are held" % (back, min(self.k, self.depth)))
        slot = self.slots[(self.k - back) % self.depth]
        self._settle(slot)
        counts, m = slot["counts"], slot["m"]
        raw = slot["recv"][:self.world * m].view(self.world, m).cpu().numpy()
        parts = [np.frombuffer(raw[r, :counts[r] * REC].tobytes(), dtype=KEYPOINT_DTYPE) for r in range(self.world)]
        return np.concatenate(parts) if parts else np.zeros(0, dtype=KEYPOINT_DTYPE)


def host_fill(records):
    """fill() for host-side keypoint arrays (tests / CPU ranks)."""
    raw = np.ascontiguousarray(records, dtype=KEYPOINT_DTYPE).view(np.uint8)

    def fill(buf, cap):
        if raw.size:
            buf[:raw.size].copy_(torch.from_numpy(raw.copy()).to(buf.device))
        return records.shape[0]
    return fill
