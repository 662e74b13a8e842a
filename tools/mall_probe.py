"""Does the extrema scan read DoG planes the Gaussian pass just wrote from the
256 MiB Infinity Cache?  Extrema-stage time right after the build vs after a
1 GiB write+read flush, per image size (octave-0 G+DoG 124 MB at 960x540,
500 MB at 1920x1080).  usage: python tools/mall_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

dev = torch.device("cuda:0")
flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
for (W, H) in [(480, 270), (960, 540), (1280, 720), (1920, 1080)]:
    img = torch.from_numpy(blob_image(W, H, seed=1)).to(dev)
    p = sift_amd.make_params(num_octaves=4, scales_per_octave=5)
    with sift_amd.Context(0) as ctx:
        res = {True: [], False: []}
        for rep in range(12):
            fl = bool(rep & 1)
            torch.cuda.synchronize()
            ctx.build_scale_space_device(img.data_ptr(), W, H, p)
            ctx.synchronize()
            if fl:
                flush.fill_(float(rep))
                s = float(flush.sum())
                torch.cuda.synchronize()
            ctx.find_extrema()
            if rep >= 2:
                res[fl].append(ctx.timings()["extrema_ms"])
        a, b = np.median(res[False]), np.median(res[True])
        dog = 7 * 4 * (2 * W) * (2 * H) / 1e6
        print("%4dx%-4d oct0 G+DoG %5.0f MB  extrema stage: right after build %.4f ms, after flush %.4f ms (%.2fx)"
              % (W, H, 15 / 7 * dog, a, b, b / a), flush=True)
