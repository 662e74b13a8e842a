"""Multi-process (gloo, world size 2) checks of the batch-sharding path:
every rank detects on its own images, the ragged keypoint lists are
all-gathered, and the result equals the concatenation of the per-rank lists
in rank order."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sift_amd import KEYPOINT_DTYPE
from sift_amd.dist import KeypointGather, PipelinedKeypointGather, host_fill, shard_images


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def fake_keypoints(rank, n):
    k = np.zeros(n, dtype=KEYPOINT_DTYPE)
    k["octave"] = rank
    k["scale_level"] = 1 + np.arange(n) % 5
    k["local_x"] = np.arange(n)
    k["local_y"] = 7 * rank
    k["abs_x"] = np.arange(n) * 0.5 + rank
    k["abs_y"] = 1.25 * rank
    k["abs_sigma"] = 1.6
    k["interp_value"] = -0.01 * (rank + 1)
    return k


def _worker(rank, world, port, counts, out_q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = KeypointGather("cpu")
        res = []
        for step, per_rank in enumerate(counts):  # several steps: buffer reuse and growth
            mine = fake_keypoints(rank, per_rank[rank])
            c = g(mine.shape[0], host_fill(mine))
            res.append((c, g.gathered(c).tobytes()))
        # the pipelined form: gathers left in flight over a ring of 2 slots, read back a step later
        pg = PipelinedKeypointGather("cpu", depth=2)
        pres = []
        for step, per_rank in enumerate(counts):
            mine = fake_keypoints(rank, per_rank[rank])
            c = pg(mine.shape[0], host_fill(mine))
            if step:
                pres.append(pg.gathered(2).tobytes())
        pg.drain()
        pres.append(pg.gathered(1).tobytes())
        res.append(pres)
        out_q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_keypoint_all_gather_matches_concatenation(world):
    counts = [[3, 5], [0, 2], [11, 0], [0, 0]]
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, counts, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for step, per_rank in enumerate(counts):
        expect = np.concatenate([fake_keypoints(r, per_rank[r]) for r in range(world)])
        for r in range(world):
            c, blob = results[r][step]
            assert c == per_rank
            got = np.frombuffer(blob, dtype=KEYPOINT_DTYPE)
            assert got.tobytes() == expect.tobytes()
            assert results[r][len(counts)][step] == expect.tobytes()  # pipelined, one step later


def test_shard_images_covers_batch_once():
    for n, world in [(64, 8), (10, 4), (3, 8)]:
        seen = []
        for r in range(world):
            seen += shard_images(n, world, r)
        assert seen == list(range(n))


def _side_worker(rank, world, ports, out_q):
    from sift_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    res = []
    for port in ports:  # two process-group lifetimes in one process
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            g1 = shard.side_group()
            g2 = shard.side_group()
            t = torch.tensor([rank + 1.0])
            dist.all_reduce(t, group=g1)
            res.append((id(g1), g1 is g2, float(t.item())))
        finally:
            dist.destroy_process_group()
    out_q.put((rank, res))


def test_side_group_survives_process_group_reinit():
    """the side communicator cached for the default world is made
    again after destroy_process_group / init_process_group (a stale one would
    error or hang), and reused within one lifetime."""
    world = 2
    ports = [_free_port(), _free_port()]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_side_worker, args=(r, world, ports, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        (a_id, a_same, a_sum), (b_id, b_same, b_sum) = results[r]
        assert a_same and b_same            # cached within a lifetime
        assert a_sum == b_sum == 3.0        # the second lifetime's side group works
