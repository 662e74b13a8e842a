"""Comparison helpers shared by the GPU parity tests.

Tolerances: keypoint (x, y, sigma) within 1e-4 (BASELINE.json north_star),
identical candidate / keypoint sets and order, plane values within fp32
rounding of the reference's fp64 values.
"""
import os

import numpy as np

import oracle as orc
import sift_amd

XY_SIGMA_TOL = 1e-4


def host_threads():
    """CPU threads for the oracle (the GPU box's share is 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def oracle_params(p):
    return orc.make_params(p.num_octaves, p.scales_per_octave, p.min_blur, p.assumed_blur,
                           p.min_interpixel_distance)


def check_candidates(c, ref, value_rtol=2 ** -23):
    """c: EXTREMUM_DTYPE array; ref: (N,5) [o, s, x, y, value]."""
    assert c.shape[0] == ref.shape[0], (c.shape[0], ref.shape[0])
    got = np.stack([c["octave"], c["scale"], c["x"], c["y"]], axis=1)
    np.testing.assert_array_equal(got, ref[:, :4].astype(np.int64))
    np.testing.assert_allclose(c["value"], ref[:, 4], rtol=value_rtol, atol=1e-15)


def check_keypoints(k, ref):
    """k: KEYPOINT_DTYPE array; ref: (M,8) reference order."""
    assert k.shape[0] == ref.shape[0], (k.shape[0], ref.shape[0])
    ints = np.stack([k["octave"], k["scale_level"], k["local_x"], k["local_y"]], axis=1)
    np.testing.assert_array_equal(ints, ref[:, :4].astype(np.int64))
    np.testing.assert_allclose(k["abs_sigma"], ref[:, 4], rtol=0, atol=XY_SIGMA_TOL)
    np.testing.assert_allclose(k["abs_x"], ref[:, 5], rtol=0, atol=XY_SIGMA_TOL)
    np.testing.assert_allclose(k["abs_y"], ref[:, 6], rtol=0, atol=XY_SIGMA_TOL)
    np.testing.assert_allclose(k["interp_value"], ref[:, 7], rtol=0, atol=1e-6)


def as_keypoints(buf):
    """uint8 [n, 48] (device or host tensor / array) -> KEYPOINT_DTYPE array."""
    if hasattr(buf, "cpu"):
        buf = buf.cpu().numpy()
    return np.frombuffer(np.ascontiguousarray(buf).tobytes(), dtype=sift_amd.KEYPOINT_DTYPE)
