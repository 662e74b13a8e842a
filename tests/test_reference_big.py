"""Parity at headline scale against the reference ITSELF.

tests/golden/big holds the unmodified reference's outputs (background.js
under Node, make_golden_big.py) for BASELINE cfg 2 (1920x1080, O=4, S=5)
and cfg 3 (3840x2160, O=4, S=5, bench.py's image): candidate lists in the
reference's order, per-(octave, scale) low-contrast counts, refined
keypoints in order.  The HIP path (C ABI) is compared with them directly --
no oracle in between -- and the CPU oracle is pinned to the 1080p case
(CPU suite).

Tolerances: identical candidate and keypoint sets and order; candidate
values within fp32 rounding (the fixture stores them as fp32); keypoint (x,
y, sigma) within 1e-4 (BASELINE.json north_star); interpolated values within
1e-6.
"""
import numpy as np
import pytest

import oracle as orc
import sift_amd
from golden_util import BigGolden, big_case_names
from parity_util import check_candidates, check_keypoints, host_threads

FP32_RTOL = 2 ** -23


def _params(g, flags=0):
    P = g.params
    return sift_amd.make_params(P["num_octaves"], P["scales_per_octave"], P["min_blur"], P["assumed_blur"],
                                P["min_interpixel_distance"], flags)


def _low_counts(low, O, S):
    n = np.zeros(O * S, dtype=np.int64)
    np.add.at(n, low["octave"].astype(np.int64) * S + low["scale"].astype(np.int64) - 1, 1)
    return n


def test_big_fixtures_consistent():
    names = big_case_names()
    assert {"ref1080p_o4_s5", "ref4k_o4_s5"} <= set(names)
    for n in names:
        g = BigGolden(n)
        assert g.candidates.shape[0] == g.meta["n_candidates"]
        assert g.refined.shape[0] == g.meta["n_refined"]
        assert int(g.low_contrast_counts.sum()) == g.meta["n_low_contrast"]
        assert g.meta["refine_error"] is None


@pytest.mark.timeout(300)
def test_oracle_matches_reference_1080p():
    """The CPU oracle (separable fp64, the GPU path's numerics) against the
    reference's own 1080p outputs."""
    g = BigGolden("ref1080p_o4_s5")
    P = g.params
    op = orc.make_params(P["num_octaves"], P["scales_per_octave"], P["min_blur"], P["assumed_blur"],
                         P["min_interpixel_distance"])
    r = orc.OracleRun(g.img, op, orc.CONV_SEPARABLE, threads=host_threads(), keep_gauss=False)
    ref_c = g.candidates
    c = r.candidates()
    np.testing.assert_array_equal(c[:, :4], ref_c[:, :4])
    np.testing.assert_allclose(c[:, 4], ref_c[:, 4], rtol=FP32_RTOL, atol=1e-15)
    k, ref_k = r.refined, g.refined
    np.testing.assert_array_equal(k[:, :4], ref_k[:, :4])
    np.testing.assert_allclose(k[:, 4:7], ref_k[:, 4:7], rtol=0, atol=1e-4)
    assert r.n_low == int(g.low_contrast_counts.sum())


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", big_case_names())
def test_gpu_matches_reference_itself(gpu_ctx, name):
    g = BigGolden(name)
    P = g.params
    O, S = P["num_octaves"], P["scales_per_octave"]
    kp = gpu_ctx.detect(g.img, _params(g, sift_amd.F_LOW_CONTRAST_LIST)).copy()
    check_candidates(gpu_ctx.candidates(), g.candidates, value_rtol=FP32_RTOL)
    check_keypoints(kp, g.refined)
    np.testing.assert_array_equal(_low_counts(gpu_ctx.low_contrast(), O, S), g.low_contrast_counts)
    print("\n%s: %d candidates, %d keypoints, %d low-contrast: identical to the reference"
          % (name, g.candidates.shape[0], kp.shape[0], int(g.low_contrast_counts.sum())))
