#!/usr/bin/env python3
"""Counts of the refinement's exact re-decisions and the output-precision
bound histogram (SIFT_DEBUG_REFINE prints them on stderr) for the
benchmark configurations.  usage: SIFT_DEBUG_REFINE=1 tools/refine_bounds.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

for (W, H, O, S, seed) in ((3840, 2160, 4, 5, 42), (7680, 4320, 6, 5, 8), (1920, 1080, 4, 5, 11)):
    img = blob_image(W, H, seed=seed)
    with sift_amd.Context(0) as c:
        for _ in range(2):
            t0 = time.perf_counter()
            kp = c.detect(img, sift_amd.make_params(O, S))
            t = time.perf_counter() - t0
        print("%dx%d O%d S%d: %d keypoints, counts %s, %.1f ms, timings %s" % (W, H, O, S, kp.shape[0], c.counts(),
                                                                             t * 1e3, c.timings()), flush=True)
