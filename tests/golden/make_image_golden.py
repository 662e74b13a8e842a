#!/usr/bin/env python3
"""Golden fixtures for the image products.

Runs only in the build container (needs /root/reference and Node): drives
run_image_reference.mjs, which calls the reference's own
ImageUtils_convertImageDataToMatrix2D, Matrix2D_sigmoidNormalize,
Matrix2D_sampledNormalize and ImageUtils_convertMatrix2DToImageData, and
packs inputs and outputs into tests/golden/image_products.npz (data only).

Inputs: an RGBA image holding every byte value in every channel plus random
pixels, and an fp32 matrix with values in [-0.3, 1.3], exact k/255 and
(k+0.5)/255 grey levels (Math.round boundaries), huge magnitudes (clamping,
sigmoid saturation) and zeros; the same matrix without the saturating values
(the sampled normalisation then spreads over all levels); a constant matrix
pins the sampled normalisation's 0/0 case.

usage: python tests/golden/make_image_golden.py
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "image_products.npz")
W, H = 37, 23            # RGBA image (ragged width: not a multiple of 4)
MW, MH = 74, 46          # matrix = the octave-0 plane of a W x H input
COEF = 5.0               # background.js:303


def rgba_input():
    rng = np.random.default_rng(1234)
    a = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    v = np.arange(256, dtype=np.uint8)
    flat = a.reshape(-1, 4)
    for c in range(4):
        flat[:256, c] = np.roll(v, 37 * c)
    return a


def matrix_input(const=False, moderate=False):
    if const:
        return np.full((MH, MW), 0.25, dtype=np.float32)
    rng = np.random.default_rng(99)
    m = rng.uniform(-0.3, 1.3, size=(MH, MW)).astype(np.float32)
    flat = m.reshape(-1)
    k = np.arange(256)
    flat[:256] = (k / 255.0).astype(np.float32)
    flat[256:512] = ((k + 0.5) / 255.0).astype(np.float32)
    flat[512:520] = np.array([0.0, -0.0, 1e30, -1e30, 300.0, -300.0, 0.5 / 255, 254.5 / 255], dtype=np.float32)
    if moderate:  # no saturating values: the sampled normalisation spreads over all levels
        flat[514:518] = 0.5
    return m


def run(rgba, mat, tmp, tag):
    rp, mp = os.path.join(tmp, "rgba.u8"), os.path.join(tmp, "m.f32")
    od = os.path.join(tmp, tag)
    os.makedirs(od)
    rgba.tofile(rp)
    mat.tofile(mp)
    cmd = ["node", "--experimental-loader", os.path.join(HERE, "ref_loader.mjs"),
           os.path.join(HERE, "run_image_reference.mjs"), rp, str(W), str(H), mp, str(MW), str(MH), str(COEF), od]
    subprocess.run(cmd, check=True, cwd=HERE, stderr=subprocess.DEVNULL)
    rd = lambda n, t: np.fromfile(os.path.join(od, n), dtype=t)  # noqa: E731
    return {
        "gray": rd("gray.f64", np.float64).reshape(H, W),
        "alpha": rd("alpha.f64", np.float64).reshape(H, W),
        "plain": rd("plain.u8", np.uint8).reshape(MH, MW, 4),
        "sigmoid": rd("sigmoid.u8", np.uint8).reshape(MH, MW, 4),
        "sampled": rd("sampled.u8", np.uint8).reshape(MH, MW, 4),
    }


def main():
    rgba = rgba_input()
    m = matrix_input()
    mm = matrix_input(moderate=True)
    mc = matrix_input(const=True)
    with tempfile.TemporaryDirectory() as tmp:
        r = run(rgba, m, tmp, "a")
        rm = run(rgba, mm, tmp, "m")
        rc = run(rgba, mc, tmp, "c")
    np.savez_compressed(OUT, rgba=rgba, matrix=m, matrix_mod=mm, matrix_const=mc, coef=np.float64(COEF),
                        mod_plain=rm["plain"], mod_sigmoid=rm["sigmoid"], mod_sampled=rm["sampled"],
                        gray=r["gray"], alpha=r["alpha"], plain=r["plain"], sigmoid=r["sigmoid"],
                        sampled=r["sampled"], const_plain=rc["plain"], const_sampled=rc["sampled"],
                        const_sigmoid=rc["sigmoid"])
    print("wrote", OUT)


if __name__ == "__main__":
    main()
