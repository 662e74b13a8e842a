"""The CPU oracle (oracle/sift_oracle.c) against the golden vectors that the
reference itself produced (tests/golden/make_golden.py).  This pins the
oracle before it is used as the checker of the HIP path."""
import numpy as np
import pytest

import oracle as orc
from golden_util import Golden, case_names


def _params(g):
    P = g.params
    return orc.make_params(P["num_octaves"], P["scales_per_octave"], P["min_blur"], P["assumed_blur"],
                           P["min_interpixel_distance"])


@pytest.mark.parametrize("mode", [orc.CONV_2D, orc.CONV_SEPARABLE], ids=["2d", "separable"])
@pytest.mark.parametrize("name", case_names())
def test_oracle_matches_reference(name, mode):
    g = Golden(name)
    if mode == orc.CONV_2D and g.img.size > 300 * 300:
        pytest.skip("2D mode is covered on the smaller cases (seconds budget)")
    p = _params(g)
    r = orc.OracleRun(g.img, p, mode)
    z = g.z
    # schedule: blur levels of every Gaussian / DoG plane (background.js:207-210, :326-329).
    # V8's Math.pow (fdlibm) and glibc pow differ by 1 ulp on some inputs, so
    # the C schedule agrees to 1 ulp; the JS host passes its own Math.pow
    # schedule through the ABI when bit-identical metadata matters.
    blur, _ = orc.schedule(p)
    np.testing.assert_allclose(blur, z["gauss_blur"], rtol=3e-16, atol=0)
    np.testing.assert_allclose(blur[:, :-1], z["dog_blur"], rtol=3e-16, atol=0)
    tol = 1e-15 if mode == orc.CONV_2D else 5e-14
    for o, (h, w) in enumerate(r.dims):
        assert (h, w) == tuple(z["dims"][o])
        pos = z["sample_pos"][o]
        np.testing.assert_allclose(r.gauss[o][:, pos[:, 0], pos[:, 1]], z["gauss_samples"][o], rtol=0, atol=tol * 4)
        np.testing.assert_allclose(r.dog[o][:, pos[:, 0], pos[:, 1]], z["dog_samples"][o], rtol=0, atol=tol * 4)
        gs = r.gauss[o].reshape(r.gauss[o].shape[0], -1).sum(axis=1)
        np.testing.assert_allclose(gs, z["gauss_stats"][o][:, 0], rtol=1e-12)
    c = r.candidates()
    zc = g.candidates
    assert c.shape == zc.shape
    np.testing.assert_array_equal(c[:, :4], zc[:, :4])          # same set, same order
    np.testing.assert_allclose(c[:, 4], zc[:, 4], rtol=0, atol=1e-13)
    assert r.n_low == int(z["low_contrast_counts"].sum())
    k = r.refined
    zk = g.refined
    assert g.meta["refine_error"] is None and r.n_singular == 0
    assert k.shape == zk.shape
    np.testing.assert_array_equal(k[:, :4], zk[:, :4])
    np.testing.assert_allclose(k[:, 4:], zk[:, 4:], rtol=0, atol=1e-9)


def test_oracle_refine_singular_is_flagged():
    """A candidate on a flat DoG has det(H) = 0: the reference throws
    (matrix2d.js:482 -> 455); the oracle counts it as singular."""
    p = orc.make_params(1, 3)
    img = np.full((8, 8), 0.5, dtype=np.float32)
    r = orc.OracleRun(img, p, orc.CONV_SEPARABLE)
    rec = np.array([[0, 1, 5, 5]], dtype=np.int32)
    out, sing = r.refine(rec, np.array([0.0]))
    assert out.shape[0] == 0 and sing == 1


def test_oracle_thread_count_and_orders():
    """The threaded oracle (blur loops and extrema scan over OpenMP rows) gives
    the single-thread lists bit for bit; the three summation orders give the
    same candidates here and planes within a few fp64 ulps."""
    import numpy as np
    from sift_amd.synth import blob_image
    img = blob_image(200, 150, seed=9)
    p = orc.make_params(4, 4)
    a = orc.OracleRun(img, p, orc.CONV_SEPARABLE, threads=1)
    b = orc.OracleRun(img, p, orc.CONV_SEPARABLE, threads=4)
    for f in ("cand_rec", "cand_val", "low_rec", "low_val", "refined", "dog_flat"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert a.low_rec.shape[0] == a.n_low > 0
    for mode in (orc.CONV_2D, orc.CONV_SEPARABLE_FMA_VH):
        c = orc.OracleRun(img, p, mode, threads=4)
        assert np.array_equal(c.cand_rec, a.cand_rec)
        assert np.abs(c.dog_flat - a.dog_flat).max() < 1e-14
