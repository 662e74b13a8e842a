"""Stage-API extrema timing probe (the reference's findCandidateKeypoints
surface: sift_find_extrema on a built pyramid, the stream idle when the stage
starts) against the same stage inside sift_detect (enqueued behind the
pass).  Prints, per image size, the HIP-event stage time of both paths and
the host wall time of the sift_find_extrema call; run it under
`rocprofv3 --kernel-trace --hip-runtime-trace` to see the gaps between the
stage's kernels.  usage: python tools/stage_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

dev = torch.device("cuda:0")
for (W, H, seed) in [(480, 270, 1), (1920, 1080, 1), (3840, 2160, 1), (3840, 2160, 42)]:
    img = torch.from_numpy(blob_image(W, H, seed=seed)).to(dev)
    p = sift_amd.make_params(num_octaves=4, scales_per_octave=5)
    with sift_amd.Context(0) as ctx:
        st, wall, det = [], [], []
        for rep in range(8):
            ctx.build_scale_space_device(img.data_ptr(), W, H, p)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.find_extrema()
            wall.append((time.perf_counter() - t0) * 1e3)
            st.append(ctx.timings()["extrema_ms"])
            ctx.detect_device(img.data_ptr(), W, H, p)
            det.append(ctx.timings()["extrema_ms"])
        c = ctx.counts()
        print("%4dx%-4d seed %2d stage API sift_find_extrema: events %.4f ms, host wall %.3f ms | inside sift_detect: "
              "events %.4f ms | %d candidates, %d ambiguous (exact fp64 re-decisions)"
              % (W, H, seed, np.median(st[2:]), np.median(wall[2:]), np.median(det[2:]), c["candidates"],
                 c["exact"]), flush=True)
