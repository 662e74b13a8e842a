"""Parity of the HIP path (through the C ABI) with the reference.

* golden cases: against vectors the reference itself produced
  (tests/golden), for the one-call path and the stage-by-stage path;
* larger sizes: against the pinned CPU oracle (fp64 C restatement);
* caller-supplied pyramids (sift_load_dog / sift_load_scale_space): exact
  against the oracle run on the same fp32 planes;
* quirks and edge cases the reference has (singular Hessian, flat images,
  tiny octaves), determinism.

Tolerances: keypoint (x, y, sigma) within 1e-4 (BASELINE.json north_star),
identical candidate / keypoint sets and order, plane values within fp32
rounding of the reference's fp64 values.
"""
import numpy as np
import pytest

import oracle as orc
import sift_amd
from golden_util import Golden, case_names
from parity_util import check_candidates, check_keypoints, oracle_params as _oracle_params
from sift_amd.synth import blob_image

pytestmark = pytest.mark.gpu


def params_of(g, flags=0):
    P = g.params
    return sift_amd.make_params(P["num_octaves"], P["scales_per_octave"], P["min_blur"], P["assumed_blur"],
                                P["min_interpixel_distance"], flags)


@pytest.mark.parametrize("name", case_names())
def test_detect_matches_reference(gpu_ctx, name):
    g = Golden(name)
    kp = gpu_ctx.detect(g.img, params_of(g, sift_amd.F_LOW_CONTRAST_LIST))
    check_candidates(gpu_ctx.candidates(), g.candidates)
    check_keypoints(kp, g.refined)
    cnt = gpu_ctx.counts()
    assert cnt["low_contrast"] == int(g.z["low_contrast_counts"].sum())
    assert cnt["singular"] == 0
    # per (octave, scale) low-contrast counts of the reference (background.js:408-413 markers)
    low = gpu_ctx.low_contrast()
    per = np.zeros_like(np.asarray(g.z["low_contrast_counts"]).ravel())
    S = g.params["scales_per_octave"]
    np.add.at(per, low["octave"] * S + low["scale"] - 1, 1)
    np.testing.assert_array_equal(per, np.asarray(g.z["low_contrast_counts"]).ravel())


@pytest.mark.parametrize("name", case_names())
def test_stage_api_matches_reference(gpu_ctx, name):
    """computeGaussianScaleSpace -> computeDifferenceOfGaussians ->
    findCandidateKeypoints -> refineCandidateKeypoints, stage by stage."""
    g = Golden(name)
    p = params_of(g)
    gpu_ctx.build_scale_space(g.img, p)
    z = g.z
    O, S = p.num_octaves, p.scales_per_octave
    for o in range(O):
        assert gpu_ctx.dims(o) == tuple(z["dims"][o])
        pos = z["sample_pos"][o]
        for s in range(S + 3):
            L = gpu_ctx.plane(sift_amd.PLANE_GAUSS, o, s).astype(np.float64)
            ref = z["gauss_samples"][o][s]
            np.testing.assert_allclose(L[pos[:, 0], pos[:, 1]], ref, rtol=2 ** -24, atol=1e-13)
            assert gpu_ctx.blur_level(sift_amd.PLANE_GAUSS, o, s) == pytest.approx(z["gauss_blur"][o][s], rel=1e-15)
        for s in range(S + 2):
            D = gpu_ctx.plane(sift_amd.PLANE_DOG, o, s).astype(np.float64)
            ref = z["dog_samples"][o][s]
            np.testing.assert_allclose(D[pos[:, 0], pos[:, 1]], ref, rtol=2 ** -24, atol=1e-13)
    cand, low = gpu_ctx.find_extrema()
    check_candidates(cand, g.candidates)
    assert low == int(z["low_contrast_counts"].sum())
    kp, sing = gpu_ctx.refine()
    check_keypoints(kp, g.refined)
    assert sing == 0


@pytest.mark.parametrize("W,H,O,S,seed", [(1920, 1080, 4, 5, 11), (640, 480, 5, 3, 12), (333, 517, 4, 4, 13)])
def test_detect_matches_oracle_large(gpu_ctx, W, H, O, S, seed):
    img = blob_image(W, H, seed=seed)
    p = sift_amd.make_params(O, S, flags=sift_amd.F_LOW_CONTRAST_LIST)
    kp = gpu_ctx.detect(img, p)
    r = orc.OracleRun(img, _oracle_params(p), orc.CONV_SEPARABLE)
    check_candidates(gpu_ctx.candidates(), r.candidates())
    check_keypoints(kp, r.refined)
    assert gpu_ctx.counts()["low_contrast"] == r.n_low
    # the reference's lowContrastKeypoints (sift.js:293-306), in its order
    check_candidates(gpu_ctx.low_contrast(), r.low_contrast())


def test_low_contrast_list_stage_api_and_flags(gpu_ctx):
    """The low-contrast list through the stage API (sift_set_flags before
    sift_find_extrema on a built pyramid) and on a caller-supplied DoG
    (exact planes), against the oracle; without the flag it is refused."""
    img = blob_image(300, 220, seed=27)
    p = sift_amd.make_params(4, 4)
    r = orc.OracleRun(img, _oracle_params(p), orc.CONV_SEPARABLE)
    gpu_ctx.build_scale_space(img, p)
    gpu_ctx.find_extrema()
    with pytest.raises(sift_amd.SiftError):
        gpu_ctx.low_contrast()
    gpu_ctx.set_flags(sift_amd.F_LOW_CONTRAST_LIST)
    cand, low = gpu_ctx.find_extrema()
    check_candidates(cand, r.candidates())
    lc = gpu_ctx.low_contrast()
    assert lc.shape[0] == low == r.n_low
    check_candidates(lc, r.low_contrast())
    # caller-supplied fp32 DoG planes: every decision is on those planes
    dog32 = r.dog_flat.astype(np.float32)
    gpu_ctx.load_dog(dog32, 300, 220, sift_amd.make_params(4, 4, flags=sift_amd.F_LOW_CONTRAST_LIST))
    cand2, low2 = gpu_ctx.find_extrema()
    (crec, cval), (lrec, lval) = orc.extrema_lists(_oracle_params(p), 300, 220, dog32.astype(np.float64))
    check_candidates(cand2, orc.as_records(crec, cval))
    lc2 = gpu_ctx.low_contrast()
    assert lc2.shape[0] == low2 == lrec.shape[0]
    check_candidates(lc2, orc.as_records(lrec, lval))


def test_plane_reads_through_staging_round_trip(gpu_ctx):
    """sift_get_plane copies through double-buffered pinned staging in 8 MB
    chunks: a loaded DoG pyramid reads back bit-exact, for a plane of 3.15
    chunks (ragged last chunk) and for sub-megabyte planes (direct copy)."""
    W, H = 1500, 1100
    p = sift_amd.make_params(4, 3)
    px = [a * b for a, b in orc.octave_dims(W, H, 4)]
    rng = np.random.default_rng(5)
    dog = rng.standard_normal(sum(px) * 5).astype(np.float32)
    gpu_ctx.load_dog(dog, W, H, p)
    assert px[0] * 4 > 3 * (8 << 20)
    off = 0
    for o in range(4):
        h, w = gpu_ctx.dims(o)
        assert h * w == px[o]
        for s in range(5):
            np.testing.assert_array_equal(gpu_ctx.plane(sift_amd.PLANE_DOG, o, s).ravel(), dog[off:off + h * w])
            off += h * w


def test_foreign_dog_is_exact(gpu_ctx):
    """findCandidateKeypoints / refineCandidateKeypoints on a DoG pyramid the
    context did not build: the fp32 planes are the data, results are exact."""
    img = blob_image(200, 150, seed=21)
    p = sift_amd.make_params(4, 3)
    op = _oracle_params(p)
    r = orc.OracleRun(img, op, orc.CONV_SEPARABLE)
    dog32 = r.dog_flat.astype(np.float32)
    gpu_ctx.load_dog(dog32, 200, 150, p)
    cand, low = gpu_ctx.find_extrema()
    # oracle on the same fp32 values
    r.dog_flat = dog32.astype(np.float64)
    import ctypes
    lowc = ctypes.c_long(0)
    L = orc.lib()
    n = L.oracle_find_extrema(ctypes.byref(op), 200, 150, r.dog_flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                              None, None, 0, ctypes.byref(lowc))
    rec = np.zeros((max(n, 1), 4), dtype=np.int32)
    val = np.zeros(max(n, 1))
    L.oracle_find_extrema(ctypes.byref(op), 200, 150, r.dog_flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                          rec.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          val.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n, ctypes.byref(lowc))
    ref = np.concatenate([rec[:n], val[:n, None]], axis=1).astype(np.float64)
    check_candidates(cand, ref, value_rtol=0)
    assert low == lowc.value
    kp, sing = gpu_ctx.refine()
    out, osing = r.refine(rec[:n], val[:n])
    assert sing == osing
    assert kp.shape[0] == out.shape[0]
    got = np.stack([kp["abs_sigma"], kp["abs_x"], kp["abs_y"], kp["interp_value"]], axis=1)
    np.testing.assert_allclose(got, out[:, 4:], rtol=1e-14, atol=1e-15)


def test_foreign_dog_with_nonfinite_values(gpu_ctx):
    """A caller DoG holding NaN, +Inf and -Inf (sift_load_dog): the
    reference's strict comparisons (sift.js:227-256) are false for a NaN
    centre or neighbour and true for an infinite centre above / below finite
    neighbours; candidates, low-contrast count and refined keypoints (NaN /
    Inf propagated by the refinement arithmetic, background.js:468-675) equal
    the oracle's on the same values."""
    img = blob_image(200, 150, seed=23)
    p = sift_amd.make_params(4, 3)
    op = _oracle_params(p)
    r = orc.OracleRun(img, op, orc.CONV_SEPARABLE)
    dog32 = r.dog_flat.astype(np.float32)
    rng = np.random.default_rng(5)
    for v, frac in ((np.nan, 0.004), (np.inf, 0.001), (-np.inf, 0.001)):
        idx = rng.choice(dog32.size, int(frac * dog32.size), replace=False)
        dog32[idx] = v
    gpu_ctx.load_dog(dog32, 200, 150, p)
    cand, low = gpu_ctx.find_extrema()
    r.dog_flat = dog32.astype(np.float64)
    import ctypes
    lowc = ctypes.c_long(0)
    L = orc.lib()
    n = L.oracle_find_extrema(ctypes.byref(op), 200, 150, r.dog_flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                              None, None, 0, ctypes.byref(lowc))
    rec = np.zeros((max(n, 1), 4), dtype=np.int32)
    val = np.zeros(max(n, 1))
    L.oracle_find_extrema(ctypes.byref(op), 200, 150, r.dog_flat.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                          rec.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                          val.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), n, ctypes.byref(lowc))
    assert np.isinf(val[:n]).any(), "the injected infinities make candidates"
    ref = np.concatenate([rec[:n], val[:n, None]], axis=1).astype(np.float64)
    check_candidates(cand, ref, value_rtol=0)
    assert low == lowc.value
    kp, sing = gpu_ctx.refine()
    out, osing = r.refine(rec[:n], val[:n])
    assert sing == osing
    assert kp.shape[0] == out.shape[0]
    got = np.stack([kp["abs_sigma"], kp["abs_x"], kp["abs_y"], kp["interp_value"]], axis=1)
    np.testing.assert_allclose(got, out[:, 4:], rtol=1e-14, atol=1e-15)  # NaN == NaN


def test_keypoint_field_arrays_equal_records(gpu_ctx):
    """sift_copy_keypoints_soa (pinned staging, the JS typed format) carries
    the 48-byte records' fields in order; a host image goes through the
    context's pinned staging (parallel row copies) and gives the device
    image's keypoints."""
    img = blob_image(1024, 600, seed=31)
    p = sift_amd.make_params(4, 3)
    gpu_ctx.detect(np.ascontiguousarray(img), p)
    kp = gpu_ctx.keypoints()
    ints, reals = gpu_ctx.keypoints_soa()
    assert ints.shape[0] == kp.shape[0] > 100
    np.testing.assert_array_equal(ints, np.stack([kp["octave"], kp["scale_level"], kp["local_x"], kp["local_y"]], 1))
    np.testing.assert_array_equal(reals, np.stack([kp["abs_sigma"], kp["abs_x"], kp["abs_y"], kp["interp_value"]], 1))
    import torch
    d_img = torch.from_numpy(np.ascontiguousarray(img)).to("cuda")
    gpu_ctx.detect_device(d_img.data_ptr(), 1024, 600, p)
    assert gpu_ctx.keypoints().tobytes() == kp.tobytes()


def test_page_locked_image_and_field_arrays(gpu_ctx):
    """Page-locked host memory (sift_host_register): the image goes up by one
    DMA straight from it, and sift_copy_keypoints_soa splits the records on
    the device and DMAs the fields straight into page-locked destinations --
    the same keypoints and fields as the staged paths (a pageable image, and
    destinations through the pinned staging)."""
    import ctypes
    import mmap
    W, H = 1024, 600
    img = blob_image(W, H, seed=31)
    p = sift_amd.make_params(4, 3)
    gpu_ctx.detect(np.ascontiguousarray(img), p)
    ref = gpu_ctx.keypoints()
    ints0, reals0 = gpu_ctx.keypoints_soa()
    n = ref.shape[0]
    assert n > 100
    L = gpu_ctx._L
    bufs = [mmap.mmap(-1, W * H * 4), mmap.mmap(-1, n * 16), mmap.mmap(-1, n * 32)]  # page-aligned
    a = np.frombuffer(bufs[0], dtype=np.float32).reshape(H, W)
    a[:] = img
    ints = np.frombuffer(bufs[1], dtype=np.int32).reshape(n, 4)
    reals = np.frombuffer(bufs[2], dtype=np.float64).reshape(n, 4)
    ptrs = [a.ctypes.data, ints.ctypes.data, reals.ctypes.data]
    for q, b in zip(ptrs, bufs):
        assert L.sift_host_register(ctypes.c_void_p(q), len(b)) == 0
    try:
        gpu_ctx.detect(a, p)
        assert gpu_ctx.keypoints().tobytes() == ref.tobytes()
        got = ctypes.c_size_t()
        assert L.sift_copy_keypoints_soa(gpu_ctx._h, ctypes.c_void_p(ptrs[1]), ctypes.c_void_p(ptrs[2]), n,
                                         ctypes.byref(got)) == 0
        assert got.value == n
        np.testing.assert_array_equal(ints, ints0)
        np.testing.assert_array_equal(reals, reals0)
    finally:
        for q in ptrs:
            L.sift_host_unregister(ctypes.c_void_p(q))
        del a, ints, reals


def test_foreign_scale_space_dog(gpu_ctx):
    """computeDifferenceOfGaussians on a caller scale space: D = L[s-1]-L[s]."""
    img = blob_image(96, 80, seed=22)
    p = sift_amd.make_params(3, 3)
    r = orc.OracleRun(img, _oracle_params(p), orc.CONV_SEPARABLE)
    g32 = r.gauss_flat.astype(np.float32)
    gpu_ctx.load_scale_space(g32, 96, 80, p)
    off = 0
    for o, (h, w) in enumerate(r.dims):
        G = g32[off:off + 6 * h * w].reshape(6, h, w).astype(np.float64)
        off += 6 * h * w
        for s in range(5):
            D = gpu_ctx.plane(sift_amd.PLANE_DOG, o, s)
            np.testing.assert_array_equal(D, (G[s] - G[s + 1]).astype(np.float32))


def test_singular_hessian_is_reported(gpu_ctx):
    """Flat DoG around a candidate: det(H) = 0 -> the reference throws a
    TypeError (matrix2d.js:482 -> :455); the ABI returns SIFT_E_SINGULAR."""
    p = sift_amd.make_params(2, 3)
    dims = sift_amd.octave_dims(16, 16, 2)
    total = sum(h * w for h, w in dims) * 5
    gpu_ctx.load_dog(np.zeros(total, dtype=np.float32), 16, 16, p)
    cand = np.zeros(1, dtype=sift_amd.EXTREMUM_DTYPE)
    cand[0] = (0, 1, 5, 5, 0.0)
    gpu_ctx.set_candidates(cand)
    with pytest.raises(sift_amd.SiftSingularError):
        gpu_ctx.refine(raise_singular=True)
    kp, sing = gpu_ctx.refine()
    assert kp.shape[0] == 0 and sing == 1


def test_flat_image_has_no_keypoints(gpu_ctx):
    img = np.full((64, 48), 0.25, dtype=np.float32)
    kp = gpu_ctx.detect(img, sift_amd.make_params(4, 3))
    assert kp.shape[0] == 0 and gpu_ctx.counts()["candidates"] == 0


@pytest.mark.parametrize("W,H,O,S", [(1, 1, 1, 3), (3, 2, 2, 3), (7, 1, 3, 2), (1, 9, 4, 3), (5, 5, 5, 5),
                                     (2, 64, 3, 3), (4, 300, 3, 3), (300, 3, 3, 3), (6, 6, 2, 3)])
def test_degenerate_sizes_match_oracle(gpu_ctx, W, H, O, S):
    """Images down to 1 x 1 and one-pixel-wide strips, octaves down to 1 x 1:
    every Gaussian / DoG plane within fp32 rounding of the oracle, and the
    same (here: empty or tiny) candidate and keypoint lists."""
    rng = np.random.default_rng(W * 31 + H)
    img = (rng.integers(0, 4097, size=(H, W)) / 4096.0).astype(np.float32)
    p = sift_amd.make_params(O, S)
    kp = gpu_ctx.detect(img, p)
    r = orc.OracleRun(img, orc.make_params(O, S), orc.CONV_SEPARABLE)
    for o, (h, w) in enumerate(r.dims):
        assert gpu_ctx.dims(o) == (h, w)
        for s in range(S + 3):
            np.testing.assert_allclose(gpu_ctx.plane(sift_amd.PLANE_GAUSS, o, s), r.gauss[o][s], rtol=2 ** -23,
                                       atol=1e-12)
    check_candidates(gpu_ctx.candidates(), r.candidates())
    check_keypoints(kp, r.refined)


def test_empty_image_is_rejected(gpu_ctx):
    with pytest.raises(sift_amd.SiftError) as e:
        gpu_ctx.detect(np.zeros((0, 5), np.float32), sift_amd.make_params(2, 3))
    assert e.value.code == sift_amd.SIFT_E_ARG


def test_detect_is_deterministic(gpu_ctx):
    img = blob_image(512, 384, seed=23)
    p = sift_amd.make_params(4, 5)
    a = gpu_ctx.detect(img, p)
    b = gpu_ctx.detect(img, p)
    assert a.tobytes() == b.tobytes()


def test_schedule_taps_reused_across_depths_and_schedules(gpu_ctx):
    """The context keeps the deepest schedule's taps (setup_geometry) and a
    schedule whose sigmas are its prefix reuses them: detections alternating
    octave counts, scale counts and blurs on one context equal the same
    detections on fresh contexts, byte for byte."""
    img = blob_image(200, 150, seed=41)
    seq = [(5, 4, 0.8), (3, 4, 0.8), (5, 4, 0.8), (4, 3, 0.8), (2, 4, 0.8), (5, 4, 1.1), (3, 4, 1.1), (4, 4, 0.8)]
    ctx = sift_amd.Context(0)
    try:
        for O, S, mb in seq:
            p = sift_amd.make_params(O, S, min_blur=mb)
            fresh = sift_amd.Context(0)
            try:
                want = fresh.detect(img, p).tobytes()
            finally:
                fresh.close()
            assert ctx.detect(img, p).tobytes() == want, (O, S, mb)
    finally:
        ctx.close()


def test_skip_gauss_planes_same_keypoints(gpu_ctx):
    img = blob_image(300, 200, seed=24)
    a = gpu_ctx.detect(img, sift_amd.make_params(4, 4))
    b = gpu_ctx.detect(img, sift_amd.make_params(4, 4, flags=sift_amd.F_SKIP_GAUSS_PLANES))
    assert a.tobytes() == b.tobytes()
    with pytest.raises(sift_amd.SiftError):
        gpu_ctx.plane(sift_amd.PLANE_GAUSS, 0, 0)


def test_large_radii_paths_match_oracle(gpu_ctx):
    """min_blur 2.5: octave-0 radii above the unrolled range (materialised
    fp64 upsample + generic-radius path) and radii up to ~45 in octave 1."""
    img = blob_image(160, 120, seed=31)
    p = sift_amd.make_params(3, 3, min_blur=2.5)
    kp = gpu_ctx.detect(img, p)
    r = orc.OracleRun(img, _oracle_params(p), orc.CONV_SEPARABLE)
    check_candidates(gpu_ctx.candidates(), r.candidates())
    check_keypoints(kp, r.refined)
    assert gpu_ctx.counts()["low_contrast"] == r.n_low


@pytest.mark.parametrize("W,H", [(257, 131), (64, 48)])
def test_unaligned_widths_match_oracle(gpu_ctx, W, H):
    """Widths not a multiple of 4 (scalar plane stores, ragged right tiles)."""
    img = blob_image(W, H, seed=W + H)
    p = sift_amd.make_params(4, 4)
    kp = gpu_ctx.detect(img, p)
    r = orc.OracleRun(img, _oracle_params(p), orc.CONV_SEPARABLE)
    check_candidates(gpu_ctx.candidates(), r.candidates())
    check_keypoints(kp, r.refined)


def _device_copy(img):
    """hipMalloc + upload through the HIP runtime libsift_hip.so uses (torch may
    bundle a different one, which must not share the process's device state)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    ptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(img.nbytes)) == 0
    assert hip.hipMemcpy(ptr, img.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(img.nbytes), 1) == 0  # H2D
    return hip, ptr


def test_async_detect_matches_sync():
    """sift_detect_device_async / sift_detect_wait on two contexts in flight
    give the same keypoints as the synchronous call."""
    img = np.ascontiguousarray(blob_image(640, 360, seed=41), dtype=np.float32)
    p = sift_amd.make_params(4, 4)
    hip, d = _device_copy(img)
    try:
        with sift_amd.Context(0) as a, sift_amd.Context(0, share=a) as b, sift_amd.Context(0) as c:
            n_ref = c.detect_device(d.value, 640, 360, p)
            ref = c.keypoints().tobytes()
            a.detect_device_async(d.value, 640, 360, p)
            b.detect_device_async(d.value, 640, 360, p)
            with pytest.raises(sift_amd.SiftError):
                a.detect_device_async(d.value, 640, 360, p)  # one in flight per context
            assert a.detect_wait() == n_ref and b.detect_wait() == n_ref
            assert a.keypoints().tobytes() == ref and b.keypoints().tobytes() == ref
    finally:
        hip.hipFree(d)


def test_phased_detect_matches_sync():
    """The two-phase API (sift_detect_begin_async / _end_async) in the bench's
    phased schedule on three contexts with their own streams: each image's
    extrema stage ordered after the next image's octave 0, each octave 0 after
    the refinement two images back -- the same keypoints as the synchronous
    call, for every image."""
    img = np.ascontiguousarray(blob_image(640, 360, seed=43), dtype=np.float32)
    p = sift_amd.make_params(4, 4)
    hip, d = _device_copy(img)
    try:
        with sift_amd.Context(0) as r:
            n_ref = r.detect_device(d.value, 640, 360, p)
            ref = r.keypoints().tobytes()
        ctxs = [sift_amd.Context(0) for _ in range(3)]
        try:
            with pytest.raises(sift_amd.SiftError):
                ctxs[0].detect_end_async()  # nothing begun
            pend = None
            done = []
            for i in range(7):
                c = ctxs[i % 3]
                if i >= 3:
                    done.append((c.detect_wait(), c.keypoints().tobytes()))
                if i >= 2:
                    c.order_after(ctxs[(i - 2) % 3], sift_amd.AFTER_REFINEMENT)
                c.detect_begin_async(d.value, 640, 360, p)
                with pytest.raises(sift_amd.SiftError):
                    c.detect_device_async(d.value, 640, 360, p)  # phase 1 in flight
                if pend is not None:
                    q = ctxs[pend % 3]
                    q.order_after(c, sift_amd.AFTER_OCTAVE0)
                    q.detect_end_async()
                pend = i
            ctxs[pend % 3].detect_end_async()
            for i in range(4, 7):
                c = ctxs[i % 3]
                done.append((c.detect_wait(), c.keypoints().tobytes()))
            assert len(done) == 7
            for n, k in done:
                assert n == n_ref and k == ref
        finally:
            for c in ctxs:
                c.close()
    finally:
        hip.hipFree(d)


# ---------------------------------------------------------------------------
# Row-band shards of one image (SURVEY.md §8e cfg 5): crops of whole rows for
# the leading octaves, the gathered fp64 base for the trailing ones.  The
# merged keypoints must be the whole-image keypoints bit for bit.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("W,H,O,S,n,overhead", [
    (480, 360, 4, 3, 2, 0.5),
    (480, 360, 4, 3, 3, 0.5),
    (640, 600, 5, 3, 4, 0.5),
    (640, 600, 5, 3, 4, 4.0),    # deeper split octave, more halo
    (512, 520, 4, 5, 5, 0.05),   # K = 0: octave 0 only on crops
])
def test_row_band_shards_match_whole_image(gpu_ctx, W, H, O, S, n, overhead):
    from sift_amd.shard import detect_sharded_local
    img = blob_image(W, H, seed=7 + n)
    p = sift_amd.make_params(O, S)
    whole = gpu_ctx.detect(img, p).copy()
    merged, plan = detect_sharded_local(gpu_ctx, img, p, n, max_overhead=overhead)
    assert len(plan.bands) == n
    assert merged.shape == whole.shape, (merged.shape, whole.shape, plan)
    for f in whole.dtype.names:
        np.testing.assert_array_equal(merged[f], whole[f], err_msg=f)


@pytest.mark.parametrize("W,H,O,S,n,overhead", [
    (480, 360, 4, 3, 3, 0.5),
    (640, 600, 5, 3, 4, 4.0),
    (512, 520, 4, 5, 5, 0.05),
    (1920, 1080, 5, 5, 8, 0.5),
])
def test_row_band_shards_device_resident(gpu_ctx, W, H, O, S, n, overhead):
    """The device-resident driver (crops as pointer offsets, on-device origin
    decoding, owned-row filtering, base-row copies and ordered merge) gives
    the whole-image keypoints bit for bit, and the decoded device origins
    equal the host-decoded ones."""
    import torch
    from sift_amd.shard import detect_sharded_device_local
    img = blob_image(W, H, seed=11 + n)
    p = sift_amd.make_params(O, S)
    whole = gpu_ctx.detect(img, p).copy()
    d_img = torch.from_numpy(img).to("cuda:0")
    merged, plan = detect_sharded_device_local(gpu_ctx, d_img, p, n, max_overhead=overhead)
    got = np.frombuffer(merged.cpu().numpy().tobytes(), dtype=sift_amd.KEYPOINT_DTYPE)
    assert len(plan.bands) == n
    assert got.shape == whole.shape, (got.shape, whole.shape, plan)
    assert got.tobytes() == whole.tobytes()
    pk = sift_amd.make_params(O, S, flags=sift_amd.F_KEYPOINT_ORIGINS)
    gpu_ctx.set_row_origin(2 ** (O - 1) * 3)
    try:
        n_kp = gpu_ctx.detect_device(d_img.data_ptr(), W, H, pk)
        host = gpu_ctx.keypoint_origins()
        dev = torch.empty((max(n_kp, 1), 4), dtype=torch.int32, device="cuda:0")
        assert gpu_ctx.copy_keypoint_origins_device(dev.data_ptr(), 4 * n_kp) == n_kp
    finally:
        gpu_ctx.set_row_origin(0)
    np.testing.assert_array_equal(dev[:n_kp].cpu().numpy(), host)


def test_keypoint_origins_and_next_seed(gpu_ctx):
    """Origins are the candidates of the keypoints; the exported base equals
    the base a deeper run builds (its octave-O Gaussian scale 0)."""
    img = blob_image(320, 240, seed=3)
    p = sift_amd.make_params(3, 3, flags=sift_amd.F_KEYPOINT_ORIGINS | sift_amd.F_EXPORT_NEXT_SEED)
    kp = gpu_ctx.detect(img, p).copy()
    org = gpu_ctx.keypoint_origins()
    assert org.shape == (kp.shape[0], 4)
    np.testing.assert_array_equal(org[:, 0], kp["octave"])
    cand = gpu_ctx.candidates()
    ckeys = set(zip(cand["octave"], cand["scale"], cand["y"], cand["x"]))
    assert all(tuple(r) in ckeys for r in org.tolist())
    seed = gpu_ctx.next_seed()
    p4 = sift_amd.make_params(4, 3)
    gpu_ctx.build_scale_space(img, p4)
    np.testing.assert_array_equal(seed.astype(np.float32), gpu_ctx.plane(sift_amd.PLANE_GAUSS, 3, 0))


def test_block_counts_of_caller_candidates_in_any_order(gpu_ctx):
    """Per-block counts come from the block starts of a key-ordered list; a
    caller list out of key order (sift_set_candidates) takes the histogram
    path and still counts every kept keypoint in its block."""
    img = blob_image(320, 240, seed=19)
    O, S = 4, 3
    p = sift_amd.make_params(O, S, flags=sift_amd.F_KEYPOINT_ORIGINS)
    gpu_ctx.build_scale_space(img, p)
    cand, _ = gpu_ctx.find_extrema()
    kp_sorted, _ = gpu_ctx.refine()
    org = gpu_ctx.keypoint_origins()  # blocks are by candidate (octave, scale)
    want = np.bincount(org[:, 0] * S + org[:, 1] - 1, minlength=O * S)
    assert want.sum() == kp_sorted.shape[0] > 0
    np.testing.assert_array_equal(gpu_ctx.block_counts(), want)
    rev = cand[::-1].copy()
    gpu_ctx.set_candidates(rev)
    kp_rev, _ = gpu_ctx.refine()
    assert kp_rev.shape == kp_sorted.shape
    np.testing.assert_array_equal(gpu_ctx.block_counts(), want)
    gpu_ctx.set_candidates(cand[:1].copy())
    kp1, _ = gpu_ctx.refine()
    got = gpu_ctx.block_counts()
    assert got.sum() == kp1.shape[0] <= 1


def test_owned_rows_and_block_counts(gpu_ctx):
    """sift_set_owned_rows keeps exactly the keypoints whose candidate row lies
    in the band (octave rows 2 r at octave 0, r >> (o-1) above); the per-block
    counts are the list's (octave, scale) boundaries."""
    from sift_amd.shard import _owned
    img = blob_image(400, 300, seed=17)
    O, S = 4, 4
    p = sift_amd.make_params(O, S, flags=sift_amd.F_KEYPOINT_ORIGINS)
    whole = gpu_ctx.detect(img, p).copy()
    org = gpu_ctx.keypoint_origins()
    blk = gpu_ctx.block_counts()
    np.testing.assert_array_equal(blk, np.bincount(org[:, 0] * S + org[:, 1] - 1, minlength=O * S))
    for lo, hi in ((0, 96), (96, 200), (200, -1)):
        gpu_ctx.set_owned_rows(lo, hi)
        try:
            kp = gpu_ctx.detect(img, p).copy()
            counts = gpu_ctx.block_counts()
        finally:
            gpu_ctx.set_owned_rows(-1)
        keep = _owned(org, lo, hi, hi < 0)
        assert kp.tobytes() == whole[keep].tobytes()
        np.testing.assert_array_equal(counts, np.bincount(org[keep, 0] * S + org[keep, 1] - 1, minlength=O * S))


def test_compaction_after_a_larger_detection_and_empty_band(gpu_ctx):
    """The keypoint compaction works only on the slot tiles up to the device
    candidate count (launch_keep_compact): a small detection right after a
    large one on the same context (stale flags and positions past its count)
    gives the fresh context's records, origins and block counts, and a band
    that owns no rows keeps nothing."""
    p = sift_amd.make_params(4, 4, flags=sift_amd.F_KEYPOINT_ORIGINS)
    small = blob_image(200, 150, seed=5)
    with sift_amd.Context(0) as fresh:
        want = fresh.detect(small, p).copy()
        want_org = fresh.keypoint_origins().copy()
        want_blk = fresh.block_counts().copy()
    assert len(want) > 0
    gpu_ctx.detect(blob_image(1024, 768, seed=3), p)
    got = gpu_ctx.detect(small, p).copy()
    assert got.tobytes() == want.tobytes()
    np.testing.assert_array_equal(gpu_ctx.keypoint_origins(), want_org)
    np.testing.assert_array_equal(gpu_ctx.block_counts(), want_blk)
    gpu_ctx.set_owned_rows(10 ** 6, -1)
    try:
        none = gpu_ctx.detect(small, p).copy()
        blk = gpu_ctx.block_counts().copy()
    finally:
        gpu_ctx.set_owned_rows(-1)
    assert len(none) == 0
    assert not blk.any()


@pytest.mark.parametrize("t", [3, 5])
def test_range_detection_seed_only_octaves_bit_identical(gpu_ctx, t):
    """sift_detect_from_seed_range_device evaluates the octaves below its scan
    octave for their successor's base only (launch_seed_only: L[S] at even
    rows and columns).  The scanned octave's planes and keypoints equal those
    of the full build from the same fp64 base, bit for bit; the seed-only
    octaves have no planes.  960x540 O6 S5: octave-4/5 radii 94 / 188 exceed
    their planes (clamped chains)."""
    import torch
    W, H, O, S = 960, 540, 6, 5
    img = blob_image(W, H, seed=23)
    gpu_ctx.detect(img, sift_amd.make_params(1, S, flags=sift_amd.F_EXPORT_NEXT_SEED))
    d_seed = torch.tensor(gpu_ctx.next_seed(), dtype=torch.float64, device="cuda:0").contiguous()
    torch.cuda.synchronize()
    p = sift_amd.make_params(t + 1, S, flags=sift_amd.F_KEYPOINT_ORIGINS)
    gpu_ctx.detect_from_seed_device(d_seed.data_ptr(), 1, W, H, p)
    full = gpu_ctx.keypoints().copy()
    full_org = gpu_ctx.keypoint_origins()
    planes = [gpu_ctx.plane(k, t, s) for k, n in ((sift_amd.PLANE_GAUSS, S + 3), (sift_amd.PLANE_DOG, S + 2))
              for s in range(n)]
    gpu_ctx.detect_from_seed_range_device(d_seed.data_ptr(), 1, t, W, H, p)
    got = gpu_ctx.keypoints().copy()
    assert got.tobytes() == full[full_org[:, 0] == t].tobytes()
    again = [gpu_ctx.plane(k, t, s) for k, n in ((sift_amd.PLANE_GAUSS, S + 3), (sift_amd.PLANE_DOG, S + 2))
             for s in range(n)]
    for a, b in zip(planes, again):
        assert a.tobytes() == b.tobytes()
    with pytest.raises(sift_amd.SiftError):
        gpu_ctx.plane(sift_amd.PLANE_DOG, t - 1, 0)


def test_loaded_dog_after_range_detection_scans_every_octave(gpu_ctx):
    """A context that ran sift_detect_from_seed_range_device (which scans only
    octaves >= its octave_scan_first) and then loads a caller DoG pyramid
    scans every octave of the loaded pyramid, as a fresh context does (ADVICE
    r2: the load paths reset the scan range)."""
    import torch
    W, H, O, S = 256, 192, 4, 3
    img = blob_image(W, H, seed=11)
    p = sift_amd.make_params(O, S)
    gpu_ctx.build_scale_space(img, p)
    planes = np.concatenate([gpu_ctx.plane(sift_amd.PLANE_DOG, o, s).ravel()
                             for o in range(O) for s in range(S + 2)])
    h1, w1 = gpu_ctx.dims(1)
    seed = torch.tensor(gpu_ctx.plane(sift_amd.PLANE_GAUSS, 1, 0).astype(np.float64), device="cuda:0")
    gpu_ctx.detect_from_seed_range_device(seed.data_ptr(), 1, 3, W, H, p)
    torch.cuda.synchronize()
    gpu_ctx.load_dog(planes, W, H, p)
    cand, low = gpu_ctx.find_extrema()
    with sift_amd.Context() as fresh:
        fresh.load_dog(planes, W, H, p)
        cref, lref = fresh.find_extrema()
    assert set(np.unique(cref["octave"]).tolist()) >= {0, 1}
    np.testing.assert_array_equal(cand, cref)
    assert low == lref


@pytest.mark.timeout(300)
def test_bench_octave0_schedule_4k_matches_sync():
    """bench.py's timed schedule at its own configuration (3840x2160, O=4,
    S=5): three contexts with their own streams, image i+1 ordered after
    image i's octave-0 pass (sift_order_after AFTER_OCTAVE0), image i settled
    only after image i+2 is enqueued.  Two different inputs alternate, so a
    context that mixed up another's planes or lists would show: every image's
    keypoint records equal a synchronous detection of its input."""
    W, H = 3840, 2160
    p = sift_amd.make_params(4, 5)
    imgs = [np.ascontiguousarray(blob_image(W, H, seed=s), dtype=np.float32) for s in (42, 43)]
    bufs = [_device_copy(im) for im in imgs]
    try:
        ref = []
        with sift_amd.Context(0) as c:
            for hip, d in bufs:
                c.detect_device(d.value, W, H, p)
                ref.append(c.keypoints().tobytes())
        assert ref[0] != ref[1]
        ctxs = [sift_amd.Context(0) for _ in range(3)]
        try:
            n_img = 8
            for i in range(n_img + 2):
                if i < n_img:
                    c = ctxs[i % 3]
                    if i > 0:
                        c.order_after(ctxs[(i - 1) % 3], sift_amd.AFTER_OCTAVE0)
                    c.detect_device_async(bufs[i % 2][1].value, W, H, p)
                j = i - 2
                if j >= 0:
                    ctxs[j % 3].detect_wait()
                    assert ctxs[j % 3].keypoints().tobytes() == ref[j % 2], "image %d" % j
        finally:
            for c in ctxs:
                c.close()
    finally:
        for hip, d in bufs:
            hip.hipFree(d)


# ---------------------------------------------------------------------------
# Batches of independent images (BASELINE cfg 4's images per GPU): one launch
# per stage over the batch must give every image exactly its own detection.
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("W,H,O,S,n", [
    (1920, 1080, 4, 5, 8),   # cfg 4's per-GPU share, eight distinct images
    (333, 517, 4, 3, 3),     # odd sizes (scalar plane stores, edge tiles)
    (960, 540, 6, 5, 2),     # octaves 4, 5 with radii 94 / 188: split pass and kept fp64 planes per image
])
def test_batch_equals_single_detections(gpu_ctx, W, H, O, S, n):
    import torch
    p = sift_amd.make_params(O, S)
    imgs = np.stack([blob_image(W, H, seed=100 + i) for i in range(n)])
    d = torch.from_numpy(imgs).to("cuda:0")
    singles, counts = [], []
    for i in range(n):
        gpu_ctx.detect_device(d[i].data_ptr(), W, H, p)
        singles.append(gpu_ctx.keypoints().copy())
        counts.append(singles[-1].shape[0])
    total = gpu_ctx.detect_batch_device(d.data_ptr(), n, W, H, p)
    got = gpu_ctx.keypoints()
    assert total == sum(counts) and got.shape[0] == total
    np.testing.assert_array_equal(gpu_ctx.batch_counts(n), counts)
    assert got.tobytes() == np.concatenate(singles).tobytes()
    assert len({s.tobytes() for s in singles}) == n  # distinct images, distinct lists
    # a single image through the batch entry point is the plain detection
    assert gpu_ctx.detect_batch_device(d[n - 1].data_ptr(), 1, W, H, p) == counts[-1]
    assert gpu_ctx.keypoints().tobytes() == singles[-1].tobytes()


@pytest.mark.timeout(300)
def test_batch_mixing_saturated_and_blob_images(gpu_ctx):
    """Saturated images (whole rows of tied fp32 DoG values: many listed
    ambiguous words, re-decided by k_exact_words with image-aware keys and
    row offsets) at batch positions 1 and 3 between blob images: the batch
    equals the per-image detections byte for byte, and the ambiguous work
    of images >= 1 is the sum of theirs."""
    import torch
    W, H, O, S = 640, 480, 4, 3
    p = sift_amd.make_params(O, S)
    imgs = []
    for i in range(4):
        img = blob_image(W, H, seed=300 + i)
        if i % 2:
            img = (np.clip(np.rint((img - 0.5) * 3.0 * 4096 + 2048), 0, 4096) / 4096).astype(np.float32)
            assert (img == 0).mean() + (img == 1).mean() > 0.02
        imgs.append(img)
    d = torch.from_numpy(np.stack(imgs)).to("cuda:0")
    singles, exact = [], []
    for i in range(4):
        gpu_ctx.detect_device(d[i].data_ptr(), W, H, p)
        singles.append(gpu_ctx.keypoints().copy())
        exact.append(gpu_ctx.counts()["exact"])
    assert exact[1] > 1000 and exact[3] > 1000, exact
    total = gpu_ctx.detect_batch_device(d.data_ptr(), 4, W, H, p)
    assert total == sum(s.shape[0] for s in singles)
    np.testing.assert_array_equal(gpu_ctx.batch_counts(4), [s.shape[0] for s in singles])
    assert gpu_ctx.keypoints().tobytes() == np.concatenate(singles).tobytes()
    assert gpu_ctx.counts()["exact"] == sum(exact)
    # saturated image first: image 0 owns the ambiguous words, then a blob
    total = gpu_ctx.detect_batch_device(d[1:3].data_ptr(), 2, W, H, p)
    assert gpu_ctx.keypoints().tobytes() == np.concatenate(singles[1:3]).tobytes()


def test_batch_async_and_padded_image_stride(gpu_ctx):
    """The asynchronous batch entry point, images not back to back (a row
    stride and an image stride with padding), and the unsupported options."""
    import torch
    W, H, n = 640, 480, 4
    p = sift_amd.make_params(4, 3)
    stride, istride = W + 32, (H + 5) * (W + 32)
    buf = torch.zeros(n * istride, dtype=torch.float32, device="cuda:0")
    singles = []
    for i in range(n):
        img = torch.from_numpy(blob_image(W, H, seed=200 + i)).to("cuda:0")
        buf[i * istride:i * istride + H * stride].view(H, stride)[:, :W] = img
        gpu_ctx.detect_device(img.data_ptr(), W, H, p)
        singles.append(gpu_ctx.keypoints().copy())
    torch.cuda.synchronize()
    gpu_ctx.detect_batch_device_async(buf.data_ptr(), n, W, H, p, image_stride=istride, stride=stride)
    gpu_ctx.detect_wait()
    assert gpu_ctx.keypoints().tobytes() == np.concatenate(singles).tobytes()
    with pytest.raises(sift_amd.SiftError):
        gpu_ctx.detect_batch_device(buf.data_ptr(), n, W, H, sift_amd.make_params(4, 3, flags=sift_amd.F_LOW_CONTRAST_LIST),
                                    image_stride=istride, stride=stride)
    with pytest.raises(sift_amd.SiftError):  # overlapping images
        gpu_ctx.detect_batch_device(buf.data_ptr(), n, W, H, p, image_stride=W, stride=stride)
