#!/usr/bin/env python3
"""Plane readback rate of the stage API (sift_get_plane) from Python: every
Gaussian and DoG plane of a 4K O4 S5 pyramid into fresh numpy arrays, into
pre-touched arrays, and as one timed loop per kind -- separates the library's
copy path from the JS layer's costs (tools/js_bench)."""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"))
import sift_amd  # noqa: E402
from sift_amd.synth import blob_image  # noqa: E402

W, H, O, S = 3840, 2160, 4, 5
img = blob_image(W, H, seed=42)
ctx = sift_amd.Context(0)
p = sift_amd.make_params(O, S)
ctx.build_scale_space(img, p)
kinds = [(sift_amd.PLANE_GAUSS, S + 3), (sift_amd.PLANE_DOG, S + 2)]
res = {}
for name, fresh in [("fresh", True), ("touched", False), ("touched_again", False), ("registered", False)]:
    bufs = {}
    if not fresh:
        for k, n in kinds:
            for o in range(O):
                h, w = ctx.dims(o)
                for s in range(n):
                    a = np.empty((h, w), dtype=np.float32)
                    a.fill(0)
                    if name == "registered":  # page-locked (sift_host_register, ABI 8): one DMA per plane
                        ctx._check(ctx._L.sift_host_register(a.ctypes.data_as(ctypes.c_void_p), a.nbytes),
                                   "sift_host_register")
                    bufs[(k, o, s)] = a
    t0 = time.perf_counter()
    tot = 0
    for k, n in kinds:
        for o in range(O):
            h, w = ctx.dims(o)
            for s in range(n):
                a = np.empty((h, w), dtype=np.float32) if fresh else bufs[(k, o, s)]
                ctx._check(ctx._L.sift_get_plane(ctx._h, k, o, s, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                 h * w), "sift_get_plane")
                tot += a.nbytes
    dt = time.perf_counter() - t0
    res[name] = {"bytes": tot, "ms": round(1e3 * dt, 1), "GB_s": round(tot / dt / 1e9, 2)}
    if name == "registered":
        for a in bufs.values():
            ctx._L.sift_host_unregister(a.ctypes.data_as(ctypes.c_void_p))
print(json.dumps({"what": "sift_get_plane of every Gaussian + DoG plane, 4K O4 S5, from Python", "results": res}))
