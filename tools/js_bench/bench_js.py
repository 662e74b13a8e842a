"""Writes the bench's synthetic image (sift_amd.synth.blob_image, seed 42) as
raw Float32 and times the JavaScript drop-in on it under Node
(tools/js_bench/bench_js.mjs).  usage:
  python tools/js_bench/bench_js.py [--width 3840 --height 2160 --octaves 4 --scales 5 --reps 10] --out X.json
"""
import argparse
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(R, "sift-scale-space-extrema-detection_amd"))
from sift_amd.synth import blob_image  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=3840)
ap.add_argument("--height", type=int, default=2160)
ap.add_argument("--octaves", type=int, default=4)
ap.add_argument("--scales", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--heap-mb", type=int, default=8192, help="node --max-old-space-size")
ap.add_argument("--out", required=True)
a = ap.parse_args()
img = blob_image(a.width, a.height, seed=42)
f32 = a.out + ".f32"
img.astype("<f4").tofile(f32)
try:
    # --expose-gc: each timed section starts from a collected heap; a larger
    # old space: Promise.all over 30 4K results holds ~13 M keypoint objects
    # (~1.3 GB), at which the default limit (~1.7 GB here) aborts the process
    sys.exit(subprocess.call(["node", "--expose-gc", "--max-old-space-size=%d" % a.heap_mb,
                              os.path.join(R, "tools", "js_bench", "bench_js.mjs"), f32, str(a.width),
                              str(a.height), str(a.octaves), str(a.scales), str(a.reps), a.out]))
finally:
    os.remove(f32)
