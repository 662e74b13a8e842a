"""numpy restatement of the reference's image products -- TEST INFRASTRUCTURE ONLY.

SURVEY.md §8f rows 2-3: the conversions either side of the hot path.  Only
tests/ use this, as the checker of sift_image.hip; it is pinned against
tests/golden/image_products.npz, produced by the reference's own functions
(tests/golden/make_image_golden.py).
"""
import numpy as np


def rgba_to_gray(rgba):
    """ImageUtils_convertImageDataToMatrix2D({convertToGrayscale: true,
    usePerceptualGrayscale: true}) (image-utils.js:27-152): fp64 gray and alpha.
    Operation order of image-utils.js:107 / :114 and :87."""
    a = np.asarray(rgba, dtype=np.uint8).astype(np.float64)
    v = (a[..., 0] * 0.299) + (a[..., 1] * 0.587) + (a[..., 2] * 0.114)
    return v / 255.0, a[..., 3] / 255.0


def js_round(x):
    """Math.round: ties toward +inf, exact for |x| < 2^52."""
    f = np.floor(x)
    return np.where(x - f >= 0.5, f + 1.0, f)


def to_uint8_clamped(p):
    """Uint8ClampedArray store of an integral double: NaN / <= 0 -> 0, >= 255 -> 255."""
    out = np.where(p > 0.0, np.minimum(p, 255.0), 0.0)
    out = np.where(np.isnan(p), 0.0, out)
    return out.astype(np.uint8)


def sigmoid_normalize(m, coefficient=1.0):
    """Matrix2D_sigmoidNormalize (matrix2d.js:151-158)."""
    x = np.asarray(m, dtype=np.float64)
    with np.errstate(over="ignore"):
        return 1.0 / (1.0 + np.exp(coefficient * (-1.0 * x)))


def sampled_normalize(m):
    """Matrix2D_sampledNormalize (matrix2d.js:169-193): min/max scan with
    `value < min` / `value > max` (NaNs never win), then (v-min)/(max-min)."""
    x = np.asarray(m, dtype=np.float64)
    finite = x[~np.isnan(x)]
    mn = finite.min() if finite.size else float(2 ** 53 - 1)
    mx = finite.max() if finite.size else -float(2 ** 53 - 1)
    with np.errstate(invalid="ignore", divide="ignore"):
        return (x - mn) / (mx - mn)


def gray_image_data(g):
    """ImageUtils_convertMatrix2DToImageData(w, h, {grayChannelMatrix}) (image-utils.js:171-217):
    (p, p, p, 255) with p = Math.round(g * 255), rows x cols x 4 uint8."""
    with np.errstate(invalid="ignore"):
        p = to_uint8_clamped(js_round(np.asarray(g, dtype=np.float64) * 255.0))
    out = np.empty(p.shape + (4,), dtype=np.uint8)
    out[..., 0] = out[..., 1] = out[..., 2] = p
    out[..., 3] = 255
    return out


def plane_image(m, mode, coefficient=1.0):
    """Preview image of a plane: mode 0 plain, 1 sigmoid(coefficient), 2 sampled."""
    if mode == 1:
        return gray_image_data(sigmoid_normalize(m, coefficient))
    if mode == 2:
        return gray_image_data(sampled_normalize(m))
    return gray_image_data(m)
