"""Host time of one detection's enqueue (sift_detect_device_async) and wait
(sift_detect_wait) in the bench's pipelined loop, per image size: is the
pipelined rate bound by the host launching ~40 kernels per image?
usage: python tools/host_enqueue_probe.py [W H] ..."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, "sift-scale-space-extrema-detection_amd")
import sift_amd  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

sizes = [(int(a), int(b)) for a, b in zip(sys.argv[1::2], sys.argv[2::2])] or [(1920, 1080), (3840, 2160)]
for W, H in sizes:
    d = torch.from_numpy(blob_image(W, H, seed=42)).to("cuda")
    p = sift_amd.make_params(4, 5)
    ctxs = [sift_amd.Context(0) for _ in range(3)]
    for c in ctxs:
        c.detect_device_async(d.data_ptr(), W, H, p)
        c.detect_wait()
    enq, wait, n = [], [], 60
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n + 3):
        if i < n:
            a = time.perf_counter()
            ctxs[i % 3].detect_device_async(d.data_ptr(), W, H, p)
            enq.append(time.perf_counter() - a)
        if i >= 2 and i - 2 < n:
            a = time.perf_counter()
            ctxs[(i - 2) % 3].detect_wait()
            wait.append(time.perf_counter() - a)
    tot = time.perf_counter() - t0
    print("%dx%d: %.3f ms per image, enqueue median %.3f ms, wait median %.3f ms" %
          (W, H, 1e3 * tot / n, 1e3 * float(np.median(enq)), 1e3 * float(np.median(wait))))
