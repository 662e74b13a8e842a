"""Deterministic synthetic gray images for parity tests and the bench.

The reference ships no images or fixtures, so every input
is synthetic: a mid-gray field, 64 Gaussian blobs of random sign, and
uniform noise.  Values are quantised to k/4096 so the Float32 image the
C-ABI receives is bit-identical to the fp64 `Matrix2D` the reference
(`src/image-utils.js:27` produces values in [0,1]) would see.

The generator is a counter-based splitmix64 hash, so any pixel can be
drawn independently and the result does not depend on the numpy version.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def uniform(seed, stream, n):
    """n uniforms in [0,1) from (seed, stream); fp64 with 53 random bits."""
    base = (np.uint64(seed) << np.uint64(40)) ^ (np.uint64(stream) << np.uint64(32))
    idx = np.arange(n, dtype=np.uint64) + base
    with np.errstate(over="ignore"):
        r = _splitmix64(idx)
    return (r >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def blob_image(width, height, seed=42, n_blobs=64, noise=0.1, quant=4096):
    """Gray float32 image, row-major (height, width), values k/quant in [0,1]."""
    width, height = int(width), int(height)
    img = np.full((height, width), 0.5, dtype=np.float64)
    p = uniform(seed, 1, 4 * n_blobs).reshape(n_blobs, 4)
    smax = max(1.0, min(width, height) / 8.0)
    for cx_u, cy_u, a_u, s_u in p:
        cx, cy = cx_u * width, cy_u * height
        amp = 0.3 * (2.0 * a_u - 1.0)
        sig = 2.0 + s_u * smax
        rad = int(np.ceil(4.0 * sig))
        x0, x1 = max(0, int(cx) - rad), min(width, int(cx) + rad + 1)
        y0, y1 = max(0, int(cy) - rad), min(height, int(cy) + rad + 1)
        if x0 >= x1 or y0 >= y1:
            continue
        xs = (np.arange(x0, x1) - cx) ** 2
        ys = (np.arange(y0, y1) - cy) ** 2
        img[y0:y1, x0:x1] += amp * np.exp(-(ys[:, None] + xs[None, :]) / (2.0 * sig * sig))
    if noise > 0.0:
        u = uniform(seed, 2, width * height).reshape(height, width)
        img += noise * (2.0 * u - 1.0)
    k = np.clip(np.rint(img * quant), 0, quant)
    return (k / quant).astype(np.float32)


def constant_image(width, height, value=0.5):
    return np.full((int(height), int(width)), value, dtype=np.float32)
