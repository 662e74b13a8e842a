"""Image products either side of the path.

* RGBA ImageData -> gray (ImageUtils_convertImageDataToMatrix2D, perceptual,
  image-utils.js:27-152): bit-exact to fp32(the reference's fp64 gray), and
  alpha likewise;
* plane previews (ImageUtils_convertMatrix2DToImageData of the plain,
  Matrix2D_sigmoidNormalize and Matrix2D_sampledNormalize forms,
  image-utils.js:171-217, matrix2d.js:151-193): byte-exact.

Pinning: tests/golden/image_products.npz holds outputs of the reference's own
functions (tests/golden/make_image_golden.py).  The CPU tests pin the numpy
restatement (oracle/image_products.py); the GPU tests check the HIP kernels
(csrc/sift_image.hip) against the fixtures and, on real pyramids, against
the restatement applied to the same fp32 planes.
"""
import os

import numpy as np
import pytest

import image_products as ip

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "image_products.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


# ---- oracle pinning (CPU) --------------------------------------------------
def test_oracle_gray_matches_reference(gold):
    g, a = ip.rgba_to_gray(gold["rgba"])
    np.testing.assert_array_equal(g, gold["gray"])
    np.testing.assert_array_equal(a, gold["alpha"])


@pytest.mark.parametrize("prefix,mat", [("", "matrix"), ("mod_", "matrix_mod"), ("const_", "matrix_const")])
@pytest.mark.parametrize("mode,name", [(0, "plain"), (1, "sigmoid"), (2, "sampled")])
def test_oracle_plane_images_match_reference(gold, prefix, mat, mode, name):
    got = ip.plane_image(gold[mat], mode, float(gold["coef"]))
    np.testing.assert_array_equal(got, gold[prefix + name])


# ---- HIP kernels (GPU) -----------------------------------------------------
def _load_matrix_as_plane(ctx, m):
    """Put matrix m (2H x 2W) into Gaussian plane (0, 0) of a 1-octave pyramid."""
    import sift_amd
    MH, MW = m.shape
    p = sift_amd.make_params(1, 1)
    planes = np.zeros((p.scales_per_octave + 3, MH, MW), dtype=np.float32)
    planes[0] = m
    planes[1:] = m[None] * 0.5
    ctx.load_scale_space(planes.ravel(), MW // 2, MH // 2, p)


@pytest.mark.gpu
def test_gpu_rgba_to_gray_bit_exact(gpu_ctx, gold):
    g, a = gpu_ctx.rgba_to_gray(gold["rgba"], alpha=True)
    np.testing.assert_array_equal(g, gold["gray"].astype(np.float32))
    np.testing.assert_array_equal(a, gold["alpha"].astype(np.float32))
    g2 = gpu_ctx.rgba_to_gray(gold["rgba"])
    np.testing.assert_array_equal(g2, g)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H", [(1, 1), (3, 5), (64, 16), (1283, 7)])
def test_gpu_rgba_to_gray_sizes(gpu_ctx, W, H):
    rng = np.random.default_rng(W * 131 + H)
    rgba = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    g, a = gpu_ctx.rgba_to_gray(rgba, alpha=True)
    rg, ra = ip.rgba_to_gray(rgba)
    np.testing.assert_array_equal(g, rg.astype(np.float32))
    np.testing.assert_array_equal(a, ra.astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("prefix,mat", [("", "matrix"), ("mod_", "matrix_mod"), ("const_", "matrix_const")])
@pytest.mark.parametrize("mode,name", [(0, "plain"), (1, "sigmoid"), (2, "sampled")])
def test_gpu_plane_images_match_reference(gpu_ctx, gold, prefix, mat, mode, name):
    import sift_amd
    _load_matrix_as_plane(gpu_ctx, gold[mat])
    got = gpu_ctx.plane_image(sift_amd.PLANE_GAUSS, 0, 0, mode, float(gold["coef"]))
    np.testing.assert_array_equal(got, gold[prefix + name])


@pytest.mark.gpu
def test_gpu_plane_images_of_a_pyramid(gpu_ctx):
    """Every display form of every plane of a real pyramid (ragged widths,
    unaligned plane offsets) against the restatement on the same fp32 planes."""
    import sift_amd
    from sift_amd.synth import blob_image
    img = blob_image(203, 97, seed=11)
    p = sift_amd.make_params(3, 3)
    gpu_ctx.build_scale_space(img, p)
    for o in range(3):
        for kind, n in ((sift_amd.PLANE_GAUSS, 6), (sift_amd.PLANE_DOG, 5)):
            for s in range(n):
                v = gpu_ctx.plane(kind, o, s)
                for mode, c in ((0, 1.0), (1, 5.0), (2, 1.0)):
                    got = gpu_ctx.plane_image(kind, o, s, mode, c)
                    np.testing.assert_array_equal(got, ip.plane_image(v, mode, c), err_msg=str((kind, o, s, mode)))


@pytest.mark.gpu
def test_gpu_detect_rgba_equals_gray_path(gpu_ctx):
    """sift_detect_rgba == sift_detect on the fp32 gray the reference formula
    gives, and the stage path from RGBA gives the same planes."""
    import sift_amd
    rng = np.random.default_rng(5)
    H, W = 120, 161
    yy, xx = np.mgrid[0:H, 0:W]
    base = 128 + 90 * np.sin(xx / 7.0) * np.cos(yy / 5.0) + rng.integers(-20, 21, size=(H, W))
    rgba = np.empty((H, W, 4), dtype=np.uint8)
    for c, k in enumerate((1.0, 0.8, 1.2)):
        rgba[..., c] = np.clip(base * k, 0, 255).astype(np.uint8)
    rgba[..., 3] = 255
    gray = ip.rgba_to_gray(rgba)[0].astype(np.float32)
    p = sift_amd.make_params(4, 3)
    k1 = gpu_ctx.detect_rgba(rgba, p)
    k2 = gpu_ctx.detect(gray, p)
    assert k1.shape[0] == k2.shape[0] > 0
    np.testing.assert_array_equal(k1, k2)
    gpu_ctx.build_scale_space_rgba(rgba, p)
    d1 = gpu_ctx.plane(sift_amd.PLANE_DOG, 1, 2)
    gpu_ctx.build_scale_space(gray, p)
    np.testing.assert_array_equal(d1, gpu_ctx.plane(sift_amd.PLANE_DOG, 1, 2))


@pytest.mark.gpu
def test_gpu_image_products_reject_bad_arguments(gpu_ctx):
    import ctypes
    import sift_amd
    L = sift_amd.lib()
    buf = np.zeros(64, dtype=np.uint8)
    g = np.zeros(16, dtype=np.float32)
    fp = g.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    assert L.sift_rgba_to_gray(gpu_ctx._h, buf.ctypes.data_as(ctypes.c_void_p), 4, 4, 15, fp, None) == \
        sift_amd.SIFT_E_ARG
    assert L.sift_rgba_to_gray(gpu_ctx._h, None, 4, 4, 16, fp, None) == sift_amd.SIFT_E_ARG
    gpu_ctx.build_scale_space(np.full((8, 8), 0.5, np.float32), sift_amd.make_params(1, 1))
    assert L.sift_plane_image(gpu_ctx._h, 0, 0, 0, 7, 1.0, buf.ctypes.data_as(ctypes.c_void_p), 1 << 20) == \
        sift_amd.SIFT_E_ARG
    assert L.sift_plane_image(gpu_ctx._h, 0, 0, 0, 0, 1.0, buf.ctypes.data_as(ctypes.c_void_p), 64) == \
        sift_amd.SIFT_E_CAPACITY
