import sys, os
sys.path.insert(0, "/root/repo/sift-scale-space-extrema-detection_amd")
import sift_amd
from sift_amd.synth import blob_image
img = blob_image(3840, 2160, seed=42)
ctx = sift_amd.Context(0)
p = sift_amd.make_params(4, 5)
kp = ctx.detect(img, p)
print(ctx.counts(), len(kp))
