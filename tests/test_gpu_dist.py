"""The collective paths on a real device under the `nccl` backend (RCCL),
world size 1 (the GPU box has one GPU; world-size-2 coverage of the same code
is gloo on the CPU, tests/test_dist.py and tests/test_shard.py).  What this
adds: RCCL collectives on buffers that torch's HIP runtime allocated and
libsift_hip.so wrote (sift_copy_keypoints_device into a torch tensor, the
row-band driver's all_gather_into_tensor of device keypoints and counts,
k_merge_blocks over the gathered list) -- the cross-runtime hand-off the
bench's N > 1 runs make."""
import socket

import numpy as np
import pytest

import sift_amd
from sift_amd.synth import blob_image

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_world1():
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1)
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_keypoint_gather_over_rccl_from_library_buffer(gpu_ctx, nccl_world1):
    import torch
    from sift_amd.dist import KeypointGather
    img = blob_image(640, 480, seed=31)
    p = sift_amd.make_params(4, 3)
    d_img = torch.from_numpy(img).to("cuda:0")
    want = gpu_ctx.detect(img, p).copy()
    g = KeypointGather("cuda:0")
    for _ in range(2):  # buffer reuse
        n = gpu_ctx.detect_device(d_img.data_ptr(), 640, 480, p)
        counts = g(n, lambda buf, cap: gpu_ctx.copy_keypoints_device(buf.data_ptr(), cap))
        assert counts == [want.shape[0]]
        assert g.gathered(counts).tobytes() == want.tobytes()


def test_pipelined_keypoint_gather_over_rccl(gpu_ctx, nccl_world1):
    """bench.py's gather: records all-gathers left in flight over a ring of
    slots while the next detections run, read back after drain()."""
    import torch
    from sift_amd.dist import PipelinedKeypointGather
    p = sift_amd.make_params(4, 3)
    imgs = [blob_image(480 + 32 * k, 360, seed=40 + k) for k in range(4)]
    want = [gpu_ctx.detect(im, p).copy() for im in imgs]
    g = PipelinedKeypointGather("cuda:0", depth=3)
    for im in imgs:
        d = torch.from_numpy(im).to("cuda:0")
        n = gpu_ctx.detect_device(d.data_ptr(), im.shape[1], im.shape[0], p)
        g(n, lambda buf, cap: gpu_ctx.copy_keypoints_device(buf.data_ptr(), cap))
    g.drain()
    for back in (1, 2, 3):
        assert g.gathered(back).tobytes() == want[len(imgs) - back].tobytes()


@pytest.mark.parametrize("W,H,O,S", [(1280, 720, 5, 4), (640, 480, 6, 3)])
def test_row_band_driver_over_rccl_equals_whole_image(gpu_ctx, nccl_world1, W, H, O, S):
    import torch
    from sift_amd.shard import detect_sharded_device
    img = blob_image(W, H, seed=32)
    p = sift_amd.make_params(O, S)
    whole = gpu_ctx.detect(img, p).copy()
    d_img = torch.from_numpy(img).to("cuda:0")
    out, plan = detect_sharded_device(gpu_ctx, d_img, p)
    got = out.cpu().numpy().view(sift_amd.KEYPOINT_DTYPE).reshape(-1)
    assert len(plan.bands) == 1
    assert got.tobytes() == whole.tobytes()
