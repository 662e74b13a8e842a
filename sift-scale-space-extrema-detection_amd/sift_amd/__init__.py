"""Python binding of libsift_hip.so (the C ABI in include/sift_hip.h).

This is host plumbing for tests, the bench and Python callers; the Node
N-API addon (../napi) binds the same symbols for the JS drop-in.  There is
no CPU fallback: if the HIP library is missing, import of the binding fails
loudly (SiftLibraryError) -- the CPU oracle lives in /oracle and is test
infrastructure only.
"""
import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("SIFT_HIP_LIB") or os.path.join(PKG_DIR, "libsift_hip.so")  # override: A/B builds

SIFT_OK = 0
SIFT_E_ARG = -1
SIFT_E_HIP = -2
SIFT_E_CAPACITY = -3
SIFT_E_STATE = -4
SIFT_E_SINGULAR = -5
SIFT_E_UNSUPPORTED = -6

PLANE_GAUSS = 0
PLANE_DOG = 1

F_SKIP_GAUSS_PLANES = 1
F_EXPORT_NEXT_SEED = 4
F_KEYPOINT_ORIGINS = 8
F_FUSED_EXTREMA = 16
F_LOW_CONTRAST_LIST = 32

AFTER_OCTAVE0 = 0
AFTER_GAUSSIAN = 1
AFTER_REFINEMENT = 2

DISPLAY_PLAIN = 0
DISPLAY_SIGMOID = 1
DISPLAY_SAMPLED = 2

# Exported symbols, exactly those include/sift_hip.h declares.
ABI_SYMBOLS = (
    "sift_abi_version", "sift_params_default", "sift_ctx_create", "sift_ctx_destroy",
    "sift_last_error", "sift_schedule", "sift_octave_dims", "sift_build_scale_space",
    "sift_build_scale_space_device", "sift_get_dims", "sift_get_blur_level", "sift_get_plane",
    "sift_load_dog", "sift_load_scale_space", "sift_find_extrema", "sift_refine",
    "sift_set_candidates", "sift_refine_params", "sift_copy_candidates", "sift_copy_keypoints", "sift_copy_keypoints_soa", "sift_host_register", "sift_host_unregister",
    "sift_copy_keypoints_device", "sift_detect", "sift_detect_device", "sift_last_counts",
    "sift_last_timings", "sift_device_keypoints", "sift_stream", "sift_synchronize",
    "sift_detect_device_async", "sift_detect_wait", "sift_ctx_create_shared",
    "sift_next_seed", "sift_device_next_seed", "sift_detect_from_seed", "sift_detect_from_seed_device",
    "sift_keypoint_origins", "sift_set_row_origin", "sift_order_after",
    "sift_rgba_to_gray", "sift_rgba_to_gray_device", "sift_build_scale_space_rgba", "sift_detect_rgba",
    "sift_plane_image", "sift_plane_image_device", "sift_detect_begin_async", "sift_detect_end_async",
    "sift_copy_keypoint_origins_device", "sift_copy_next_seed_device", "sift_last_octave_timings",
    "sift_last_pass_kernels",
    "sift_detect_from_seed_range_device", "sift_merge_keypoint_blocks_device", "sift_set_owned_rows",
    "sift_last_block_counts", "sift_copy_low_contrast", "sift_set_flags",
    "sift_detect_batch_device", "sift_detect_batch_device_async", "sift_detect_batch",
)


class SiftLibraryError(RuntimeError):
    pass


class SiftError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("sift error %d: %s" % (code, msg))
        self.code = code


class SiftSingularError(SiftError):
    """The reference throws a TypeError here (matrix2d.js:482 -> :455)."""


class Params(ctypes.Structure):
    _fields_ = [("num_octaves", ctypes.c_int), ("scales_per_octave", ctypes.c_int),
                ("min_blur", ctypes.c_double), ("assumed_blur", ctypes.c_double),
                ("min_interpixel_distance", ctypes.c_double), ("flags", ctypes.c_int)]


class Extremum(ctypes.Structure):
    _fields_ = [("octave", ctypes.c_int32), ("scale", ctypes.c_int32), ("x", ctypes.c_int32),
                ("y", ctypes.c_int32), ("value", ctypes.c_double)]


class Keypoint(ctypes.Structure):
    _fields_ = [("octave", ctypes.c_int32), ("scale_level", ctypes.c_int32),
                ("local_x", ctypes.c_int32), ("local_y", ctypes.c_int32),
                ("abs_x", ctypes.c_double), ("abs_y", ctypes.c_double),
                ("abs_sigma", ctypes.c_double), ("interp_value", ctypes.c_double)]


class Timings(ctypes.Structure):
    _fields_ = [("gauss_dog_ms", ctypes.c_double), ("extrema_ms", ctypes.c_double),
                ("refine_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("gauss_oct0_ms", ctypes.c_double)]


EXTREMUM_DTYPE = np.dtype([("octave", "<i4"), ("scale", "<i4"), ("x", "<i4"), ("y", "<i4"),
                           ("value", "<f8")])
KEYPOINT_DTYPE = np.dtype([("octave", "<i4"), ("scale_level", "<i4"), ("local_x", "<i4"),
                           ("local_y", "<i4"), ("abs_x", "<f8"), ("abs_y", "<f8"),
                           ("abs_sigma", "<f8"), ("interp_value", "<f8")])

_lib = None


def lib():
    """Load libsift_hip.so (raises SiftLibraryError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SiftLibraryError("libsift_hip.so not built: run `make lib` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    szp = ctypes.POINTER(ctypes.c_size_t)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int)
    fp = ctypes.POINTER(ctypes.c_float)
    pp = ctypes.POINTER(Params)
    sig = {
        "sift_abi_version": (ctypes.c_int, []),
        "sift_params_default": (ctypes.c_int, [pp]),
        "sift_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
        "sift_ctx_destroy": (ctypes.c_int, [vp]),
        "sift_last_error": (ctypes.c_char_p, [vp]),
        "sift_schedule": (ctypes.c_int, [pp, dp, dp]),
        "sift_octave_dims": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip]),
        "sift_build_scale_space": (ctypes.c_int, [vp, fp, ctypes.c_int, ctypes.c_int, sz, pp, dp]),
        "sift_build_scale_space_device": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp, dp]),
        "sift_get_dims": (ctypes.c_int, [vp, ctypes.c_int, ip, ip]),
        "sift_get_blur_level": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp]),
        "sift_get_plane": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp, sz]),
        "sift_load_dog": (ctypes.c_int, [vp, fp, ctypes.c_int, ctypes.c_int, pp]),
        "sift_load_scale_space": (ctypes.c_int, [vp, fp, ctypes.c_int, ctypes.c_int, pp]),
        "sift_find_extrema": (ctypes.c_int, [vp, vp, sz, szp, szp]),
        "sift_refine": (ctypes.c_int, [vp, vp, sz, szp, szp]),
        "sift_set_candidates": (ctypes.c_int, [vp, vp, sz]),
        "sift_refine_params": (ctypes.c_int, [vp, ctypes.c_double, ctypes.c_double]),
        "sift_copy_candidates": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_copy_low_contrast": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_set_flags": (ctypes.c_int, [vp, ctypes.c_int]),
        "sift_copy_keypoints": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_copy_keypoints_soa": (ctypes.c_int, [vp, vp, vp, sz, szp]),
        "sift_host_register": (ctypes.c_int, [vp, sz]),
        "sift_host_unregister": (ctypes.c_int, [vp]),
        "sift_copy_keypoints_device": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_detect": (ctypes.c_int, [vp, fp, ctypes.c_int, ctypes.c_int, sz, pp, vp, sz, szp]),
        "sift_detect_device": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp, vp, sz, szp]),
        "sift_detect_device_async": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp]),
        "sift_detect_wait": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_detect_batch_device": (ctypes.c_int, [vp, vp, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int, sz, pp, vp,
                                                    sz, szp]),
        "sift_detect_batch": (ctypes.c_int, [vp, vp, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int, sz, pp, vp, sz, szp]),
        "sift_detect_batch_device_async": (ctypes.c_int, [vp, vp, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int, sz,
                                                          pp]),
        "sift_detect_begin_async": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp]),
        "sift_detect_end_async": (ctypes.c_int, [vp]),
        "sift_copy_keypoint_origins_device": (ctypes.c_int, [vp, vp, sz, szp]),
        "sift_copy_next_seed_device": (ctypes.c_int, [vp, vp, sz, ctypes.c_int, ctypes.c_int]),
        "sift_ctx_create_shared": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        "sift_last_counts": (ctypes.c_int, [vp, szp, szp, szp, szp, szp]),
        "sift_last_timings": (ctypes.c_int, [vp, ctypes.POINTER(Timings)]),
        "sift_last_octave_timings": (ctypes.c_int, [vp, dp, ctypes.c_int, ip]),
        "sift_last_pass_kernels": (ctypes.c_int, [vp, ctypes.c_char_p, sz, szp]),
        "sift_detect_from_seed_range_device": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int,
                                                              ctypes.c_int, pp, vp, sz, szp]),
        "sift_merge_keypoint_blocks_device": (ctypes.c_int, [vp, vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                                             ctypes.c_int, vp]),
        "sift_set_owned_rows": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int]),
        "sift_last_block_counts": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int, ip]),
        "sift_device_keypoints": (ctypes.c_int, [vp, ctypes.POINTER(vp), szp]),
        "sift_stream": (vp, [vp]),
        "sift_synchronize": (ctypes.c_int, [vp]),
        "sift_next_seed": (ctypes.c_int, [vp, dp, sz, ip, ip]),
        "sift_device_next_seed": (ctypes.c_int, [vp, ctypes.POINTER(vp), ip, ip]),
        "sift_detect_from_seed": (ctypes.c_int, [vp, ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, pp, vp, sz,
                                                 szp]),
        "sift_detect_from_seed_device": (ctypes.c_int, [vp, ctypes.c_int, vp, ctypes.c_int, ctypes.c_int, pp, vp,
                                                        sz, szp]),
        "sift_keypoint_origins": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_int32), sz, szp]),
        "sift_set_row_origin": (ctypes.c_int, [vp, ctypes.c_int]),
        "sift_order_after": (ctypes.c_int, [vp, vp, ctypes.c_int]),
        "sift_rgba_to_gray": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, fp, fp]),
        "sift_rgba_to_gray_device": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, vp, vp]),
        "sift_build_scale_space_rgba": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp, dp]),
        "sift_detect_rgba": (ctypes.c_int, [vp, vp, ctypes.c_int, ctypes.c_int, sz, pp, vp, sz, szp]),
        "sift_plane_image": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_double, vp, sz]),
        "sift_plane_image_device": (ctypes.c_int, [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_double, vp, sz]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def make_params(num_octaves=5, scales_per_octave=3, min_blur=0.8, assumed_blur=0.5,
                min_interpixel_distance=0.5, flags=0):
    """Defaults follow src/worker.js:29-98."""
    return Params(int(num_octaves), int(scales_per_octave), float(min_blur), float(assumed_blur),
                  float(min_interpixel_distance), int(flags))


def schedule(params):
    O, NS = params.num_octaves, params.scales_per_octave + 3
    blur = np.zeros(O * NS)
    sig = np.zeros(O * NS)
    rc = lib().sift_schedule(ctypes.byref(params), blur.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             sig.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    if rc:
        raise SiftError(rc, "sift_schedule")
    return blur.reshape(O, NS), sig.reshape(O, NS)


def octave_dims(width, height, num_octaves):
    d = np.zeros(2 * num_octaves, dtype=np.int32)
    rc = lib().sift_octave_dims(int(width), int(height), int(num_octaves),
                                d.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    if rc:
        raise SiftError(rc, "sift_octave_dims")
    return [(int(d[2 * o]), int(d[2 * o + 1])) for o in range(num_octaves)]


class Context:
    """One sift_ctx: a HIP stream plus device-resident pyramids on `device`."""

    def __init__(self, device=0, share=None):
        """share: another Context whose HIP stream this one uses (its work is
        ordered after the other's; keep `share` open longer than this one)."""
        self._L = lib()
        h = ctypes.c_void_p()
        if share is not None:
            rc = self._L.sift_ctx_create_shared(share._h, ctypes.byref(h))
        else:
            rc = self._L.sift_ctx_create(int(device), ctypes.byref(h))
        if rc:
            raise SiftError(rc, "sift_ctx_create(device=%d) failed (no HIP device?)" % device)
        self._share = share  # keeps the stream owner alive
        self._h = h
        self.params = None
        self.width = self.height = 0

    def close(self):
        if self._h:
            self._L.sift_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        if rc == SIFT_OK:
            return
        msg = "%s: %s" % (what, self._L.sift_last_error(self._h).decode())
        if rc == SIFT_E_SINGULAR:
            raise SiftSingularError(rc, msg)
        raise SiftError(rc, msg)

    # -- stages -----------------------------------------------------------
    def build_scale_space(self, img, params, offset_sigmas=None):
        img = np.ascontiguousarray(img, dtype=np.float32)
        H, W = img.shape
        sig = None
        if offset_sigmas is not None:
            sig = np.ascontiguousarray(offset_sigmas, dtype=np.float64).ravel()
            sig = sig.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        rc = self._L.sift_build_scale_space(self._h, img.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                            W, H, W, ctypes.byref(params), sig)
        self._check(rc, "sift_build_scale_space")
        self.params, self.width, self.height = params, W, H

    def build_scale_space_device(self, d_ptr, width, height, params, stride=None):
        rc = self._L.sift_build_scale_space_device(self._h, ctypes.c_void_p(int(d_ptr)), int(width),
                                                   int(height), int(stride or width),
                                                   ctypes.byref(params), None)
        self._check(rc, "sift_build_scale_space_device")
        self.params, self.width, self.height = params, width, height

    def dims(self, octave):
        r, c = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.sift_get_dims(self._h, octave, ctypes.byref(r), ctypes.byref(c)), "sift_get_dims")
        return r.value, c.value

    def blur_level(self, kind, octave, scale):
        b = ctypes.c_double()
        self._check(self._L.sift_get_blur_level(self._h, kind, octave, scale, ctypes.byref(b)),
                    "sift_get_blur_level")
        return b.value

    def plane(self, kind, octave, scale):
        h, w = self.dims(octave)
        out = np.empty((h, w), dtype=np.float32)
        self._check(self._L.sift_get_plane(self._h, kind, octave, scale,
                                           out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), h * w),
                    "sift_get_plane")
        return out

    def load_dog(self, planes_flat, width, height, params):
        a = np.ascontiguousarray(planes_flat, dtype=np.float32)
        self._check(self._L.sift_load_dog(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                          int(width), int(height), ctypes.byref(params)), "sift_load_dog")
        self.params, self.width, self.height = params, width, height

    def load_scale_space(self, planes_flat, width, height, params):
        a = np.ascontiguousarray(planes_flat, dtype=np.float32)
        self._check(self._L.sift_load_scale_space(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                  int(width), int(height), ctypes.byref(params)),
                    "sift_load_scale_space")
        self.params, self.width, self.height = params, width, height

    def find_extrema(self):
        n, low = ctypes.c_size_t(), ctypes.c_size_t()
        self._check(self._L.sift_find_extrema(self._h, None, 0, ctypes.byref(n), ctypes.byref(low)),
                    "sift_find_extrema")
        return self.candidates(), int(low.value)

    def candidates(self):
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_candidates(self._h, None, 0, ctypes.byref(n)), "sift_copy_candidates")
        out = np.zeros(max(n.value, 1), dtype=EXTREMUM_DTYPE)
        self._check(self._L.sift_copy_candidates(self._h, out.ctypes.data_as(ctypes.c_void_p), out.shape[0],
                                                 ctypes.byref(n)), "sift_copy_candidates")
        return out[:n.value]

    def set_flags(self, flags):
        """Replace the current pyramid's sift_params.flags for the following stages."""
        self._check(self._L.sift_set_flags(self._h, int(flags)), "sift_set_flags")

    def low_contrast(self):
        """Low-contrast extrema of the last extrema stage (params with F_LOW_CONTRAST_LIST), reference order."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_low_contrast(self._h, None, 0, ctypes.byref(n)), "sift_copy_low_contrast")
        out = np.zeros(max(n.value, 1), dtype=EXTREMUM_DTYPE)
        self._check(self._L.sift_copy_low_contrast(self._h, out.ctypes.data_as(ctypes.c_void_p), out.shape[0],
                                                   ctypes.byref(n)), "sift_copy_low_contrast")
        return out[:n.value]

    def keypoints(self):
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_keypoints(self._h, None, 0, ctypes.byref(n)), "sift_copy_keypoints")
        out = np.zeros(max(n.value, 1), dtype=KEYPOINT_DTYPE)
        self._check(self._L.sift_copy_keypoints(self._h, out.ctypes.data_as(ctypes.c_void_p), out.shape[0],
                                                ctypes.byref(n)), "sift_copy_keypoints")
        return out[:n.value]

    def keypoints_soa(self):
        """The last keypoints as (ints int32 [n, 4]: octave, scale_level,
        local_x, local_y; reals float64 [n, 4]: abs_sigma, abs_x, abs_y,
        interp_value) -- sift_copy_keypoints_soa, the JS typed format."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_keypoints_soa(self._h, None, None, 0, ctypes.byref(n)), "sift_copy_keypoints_soa")
        ints = np.zeros((max(n.value, 1), 4), dtype=np.int32)
        reals = np.zeros((max(n.value, 1), 4), dtype=np.float64)
        self._check(self._L.sift_copy_keypoints_soa(self._h, ints.ctypes.data_as(ctypes.c_void_p),
                                                    reals.ctypes.data_as(ctypes.c_void_p), ints.shape[0],
                                                    ctypes.byref(n)), "sift_copy_keypoints_soa")
        return ints[:n.value], reals[:n.value]

    def refine_params(self, min_blur_level, min_interpixel_distance=0.5):
        self._check(self._L.sift_refine_params(self._h, float(min_blur_level), float(min_interpixel_distance)),
                    "sift_refine_params")

    def set_candidates(self, cand):
        c = np.ascontiguousarray(cand, dtype=EXTREMUM_DTYPE)
        self._check(self._L.sift_set_candidates(self._h, c.ctypes.data_as(ctypes.c_void_p), c.shape[0]),
                    "sift_set_candidates")

    def refine(self, raise_singular=False):
        n, ns = ctypes.c_size_t(), ctypes.c_size_t()
        rc = self._L.sift_refine(self._h, None, 0, ctypes.byref(n), ctypes.byref(ns))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_refine")
        return self.keypoints(), int(ns.value)

    def detect(self, img, params, raise_singular=False):
        img = np.ascontiguousarray(img, dtype=np.float32)
        H, W = img.shape
        n = ctypes.c_size_t()
        rc = self._L.sift_detect(self._h, img.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), W, H, W,
                                 ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect")
        self.params, self.width, self.height = params, W, H
        return self.keypoints()

    # -- image products (ImageData in / preview ImageData out) ---------------
    def rgba_to_gray(self, rgba, alpha=False):
        """rgba: uint8 (H, W, 4) ImageData.data -> fp32 gray (H, W) [, alpha]
        (image-utils.js:27-152 with the perceptual weights)."""
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        H, W = a.shape[0], a.shape[1]
        g = np.empty((H, W), dtype=np.float32)
        al = np.empty((H, W), dtype=np.float32) if alpha else None
        self._check(self._L.sift_rgba_to_gray(self._h, a.ctypes.data_as(ctypes.c_void_p), W, H, W * 4,
                                              g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                              al.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if alpha else None),
                    "sift_rgba_to_gray")
        return (g, al) if alpha else g

    def build_scale_space_rgba(self, rgba, params):
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        H, W = a.shape[0], a.shape[1]
        self._check(self._L.sift_build_scale_space_rgba(self._h, a.ctypes.data_as(ctypes.c_void_p), W, H, W * 4,
                                                        ctypes.byref(params), None), "sift_build_scale_space_rgba")
        self.params, self.width, self.height = params, W, H

    def detect_rgba(self, rgba, params, raise_singular=False):
        a = np.ascontiguousarray(rgba, dtype=np.uint8)
        H, W = a.shape[0], a.shape[1]
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_rgba(self._h, a.ctypes.data_as(ctypes.c_void_p), W, H, W * 4,
                                      ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_rgba")
        self.params, self.width, self.height = params, W, H
        return self.keypoints()

    def plane_image(self, kind, octave, scale, mode=DISPLAY_PLAIN, coefficient=1.0):
        """Preview ImageData (H, W, 4) uint8 of one plane (image-utils.js:171-217)."""
        h, w = self.dims(octave)
        out = np.empty((h, w, 4), dtype=np.uint8)
        self._check(self._L.sift_plane_image(self._h, kind, octave, scale, mode, float(coefficient),
                                             out.ctypes.data_as(ctypes.c_void_p), out.nbytes), "sift_plane_image")
        return out

    def detect_device(self, d_ptr, width, height, params, stride=None, raise_singular=False):
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_device(self._h, ctypes.c_void_p(int(d_ptr)), int(width), int(height),
                                        int(stride or width), ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_device")
        self.params, self.width, self.height = params, width, height
        return n.value

    def detect_device_async(self, d_ptr, width, height, params, stride=None):
        """Enqueue one detection and return (sift_detect_device_async); finish
        with detect_wait().  One in flight per context."""
        self._check(self._L.sift_detect_device_async(self._h, ctypes.c_void_p(int(d_ptr)), int(width), int(height),
                                                     int(stride or width), ctypes.byref(params)),
                    "sift_detect_device_async")
        self.params, self.width, self.height = params, width, height

    def detect_batch_device_async(self, d_ptr, n_images, width, height, params, image_stride=None, stride=None):
        """Enqueue one detection of a batch of n_images device images (image b
        at d_ptr + 4 * b * image_stride bytes; default height * width): ONE
        launch per stage over the batch (sift_detect_batch_device_async);
        finish with detect_wait(), split with batch_counts()."""
        st = int(stride or width)
        self._check(self._L.sift_detect_batch_device_async(self._h, ctypes.c_void_p(int(d_ptr)), int(n_images),
                                                           int(image_stride or height * st), int(width),
                                                           int(height), st, ctypes.byref(params)),
                    "sift_detect_batch_device_async")
        self.params, self.width, self.height = params, width, height

    def detect_batch_device(self, d_ptr, n_images, width, height, params, image_stride=None, stride=None,
                            raise_singular=False):
        """Synchronous batch detection; returns the total keypoint count."""
        self.detect_batch_device_async(d_ptr, n_images, width, height, params, image_stride, stride)
        return self.detect_wait(raise_singular=raise_singular)

    def detect_batch(self, imgs, params, raise_singular=False):
        """Host batch (imgs: (n, H, W) float32): one batched detection;
        returns the keypoints of all images (image-major, split with
        batch_counts)."""
        a = np.ascontiguousarray(imgs, dtype=np.float32)
        n_img, H, W = a.shape
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_batch(self._h, a.ctypes.data_as(ctypes.c_void_p), int(n_img), int(H * W), int(W),
                                       int(H), int(W), ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_batch")
        self.params, self.width, self.height = params, W, H
        return self.keypoints()

    def batch_counts(self, n_images):
        """Keypoints per image of the last batch detection (sums of its
        image-major block counts)."""
        return self.block_counts().reshape(int(n_images), -1).sum(axis=1)

    def detect_begin_async(self, d_ptr, width, height, params, stride=None):
        """Phase 1 of an asynchronous detection: the Gaussian+DoG pass."""
        rc = self._L.sift_detect_begin_async(self._h, ctypes.c_void_p(int(d_ptr)), int(width), int(height),
                                             int(stride or width), ctypes.byref(params))
        self._check(rc, "sift_detect_begin_async")
        self.params, self.width, self.height = params, width, height

    def detect_end_async(self):
        """Phase 2: extrema scan and refinement (complete with detect_wait)."""
        self._check(self._L.sift_detect_end_async(self._h), "sift_detect_end_async")

    def copy_keypoint_origins_device(self, d_dst, cap):
        """Decoded origins (4 int32 per keypoint) into device memory; returns the count."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_keypoint_origins_device(self._h, ctypes.c_void_p(int(d_dst)), int(cap),
                                                               ctypes.byref(n)), "sift_copy_keypoint_origins_device")
        return int(n.value)

    def copy_next_seed_device(self, d_dst, cap, row_begin, row_end):
        self._check(self._L.sift_copy_next_seed_device(self._h, ctypes.c_void_p(int(d_dst)), int(cap),
                                                        int(row_begin), int(row_end)), "sift_copy_next_seed_device")

    def next_seed_dims(self):
        r, c = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.sift_next_seed(self._h, None, 0, ctypes.byref(r), ctypes.byref(c)), "sift_next_seed")
        return r.value, c.value

    def order_after(self, prev, after=0):
        """Next work on this context waits until prev's last detection has
        passed `after` (AFTER_OCTAVE0 / AFTER_GAUSSIAN / AFTER_REFINEMENT,
        sift_order_after): software pipelining of consecutive images."""
        self._check(self._L.sift_order_after(self._h, prev._h, int(after)), "sift_order_after")

    def detect_wait(self, raise_singular=False):
        """Complete the detection in flight; returns the keypoint count."""
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_wait(self._h, None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_wait")
        return n.value

    # -- row-band shards (include/sift_hip.h, ABI >= 3) ---------------------
    def next_seed(self):
        """fp64 base of octave num_octaves from the last build with F_EXPORT_NEXT_SEED."""
        r, c = ctypes.c_int(), ctypes.c_int()
        self._check(self._L.sift_next_seed(self._h, None, 0, ctypes.byref(r), ctypes.byref(c)), "sift_next_seed")
        out = np.empty((r.value, c.value), dtype=np.float64)
        self._check(self._L.sift_next_seed(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), out.size,
                                           ctypes.byref(r), ctypes.byref(c)), "sift_next_seed")
        return out

    def detect_from_seed(self, seed, octave_first, width, height, params, raise_singular=False):
        """Octaves octave_first.. of a width x height input from that octave's fp64 base."""
        seed = np.ascontiguousarray(seed, dtype=np.float64)
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_from_seed(self._h, int(octave_first),
                                           seed.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), int(width),
                                           int(height), ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_from_seed")
        self.params, self.width, self.height = params, width, height
        return self.keypoints()

    def detect_from_seed_device(self, d_seed, octave_first, width, height, params, raise_singular=False):
        """detect_from_seed with the fp64 base in device memory; keypoints stay
        on device (returns the count)."""
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_from_seed_device(self._h, int(octave_first), ctypes.c_void_p(int(d_seed)),
                                                  int(width), int(height), ctypes.byref(params), None, 0,
                                                  ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_from_seed_device")
        self.params, self.width, self.height = params, width, height
        return n.value

    def detect_from_seed_range_device(self, d_seed, octave_first, octave_scan_first, width, height, params,
                                      raise_singular=False):
        """Build octaves octave_first.. from the device fp64 base, detect only
        octaves octave_scan_first..params.num_octaves-1 (keypoints stay on
        device; returns the count)."""
        n = ctypes.c_size_t()
        rc = self._L.sift_detect_from_seed_range_device(self._h, int(octave_first), int(octave_scan_first),
                                                        ctypes.c_void_p(int(d_seed)), int(width), int(height),
                                                        ctypes.byref(params), None, 0, ctypes.byref(n))
        if rc == SIFT_E_SINGULAR and not raise_singular:
            rc = SIFT_OK
        self._check(rc, "sift_detect_from_seed_range_device")
        self.params, self.width, self.height = params, width, height
        return n.value

    def merge_keypoint_blocks_device(self, d_in, counts, d_out):
        """Block-major merge of keypoint lists on the device; counts: int64
        (n_parts, n_blocks) host array."""
        c = np.ascontiguousarray(counts, dtype=np.int64)
        self._check(self._L.sift_merge_keypoint_blocks_device(self._h, ctypes.c_void_p(int(d_in)),
                                                              c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                              c.shape[0], c.shape[1], ctypes.c_void_p(int(d_out))),
                    "sift_merge_keypoint_blocks_device")

    def set_owned_rows(self, row_begin, row_end=-1):
        """Keep only keypoints whose candidate lies in input rows [row_begin,
        row_end) (row_end < 0: to the bottom; row_begin < 0: all)."""
        self._check(self._L.sift_set_owned_rows(self._h, int(row_begin), int(row_end)), "sift_set_owned_rows")

    def block_counts(self):
        """Kept keypoints per (octave, scale) of the last refinement: int64 [O * S]."""
        n = ctypes.c_int()
        self._check(self._L.sift_last_block_counts(self._h, None, 0, ctypes.byref(n)), "sift_last_block_counts")
        out = np.zeros(max(n.value, 1), dtype=np.int64)
        self._check(self._L.sift_last_block_counts(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                                   out.shape[0], ctypes.byref(n)), "sift_last_block_counts")
        return out[:n.value]

    def set_row_origin(self, input_row0):
        """Input row of the first row of the following images (a row-band crop)."""
        self._check(self._L.sift_set_row_origin(self._h, int(input_row0)), "sift_set_row_origin")

    def keypoint_origins(self):
        """(n, 4) int32: candidate (octave, scale, y, x) of each keypoint (F_KEYPOINT_ORIGINS)."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_keypoint_origins(self._h, None, 0, ctypes.byref(n)), "sift_keypoint_origins")
        out = np.zeros((max(n.value, 1), 4), dtype=np.int32)
        self._check(self._L.sift_keypoint_origins(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                  out.size, ctypes.byref(n)), "sift_keypoint_origins")
        return out[:n.value]

    def device_keypoints(self):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self._L.sift_device_keypoints(self._h, ctypes.byref(p), ctypes.byref(n)),
                    "sift_device_keypoints")
        return p.value or 0, n.value

    def copy_keypoints_device(self, d_dst, cap):
        """D2D copy of the last keypoints into device memory at d_dst (cap records)."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_copy_keypoints_device(self._h, ctypes.c_void_p(int(d_dst)), int(cap),
                                                       ctypes.byref(n)), "sift_copy_keypoints_device")
        return n.value

    def counts(self):
        v = [ctypes.c_size_t() for _ in range(5)]
        self._check(self._L.sift_last_counts(self._h, *[ctypes.byref(x) for x in v]), "sift_last_counts")
        keys = ("candidates", "low_contrast", "keypoints", "singular", "exact")
        return dict(zip(keys, (x.value for x in v)))

    def timings(self):
        t = Timings()
        self._check(self._L.sift_last_timings(self._h, ctypes.byref(t)), "sift_last_timings")
        return dict(gauss_dog_ms=t.gauss_dog_ms, extrema_ms=t.extrema_ms, refine_ms=t.refine_ms,
                    h2d_ms=t.h2d_ms, gauss_oct0_ms=t.gauss_oct0_ms)

    def octave_timings(self):
        """Per-octave Gaussian+DoG launch ms of the last build / detection."""
        n = ctypes.c_int()
        self._check(self._L.sift_last_octave_timings(self._h, None, 0, ctypes.byref(n)), "sift_last_octave_timings")
        out = np.zeros(max(n.value, 1))
        self._check(self._L.sift_last_octave_timings(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                     out.shape[0], ctypes.byref(n)), "sift_last_octave_timings")
        return [float(v) for v in out[:n.value]]

    def pass_kernels(self):
        """The Gaussian+DoG kernels of the last build / detection, per octave
        ("o0: k_gauss_dog<octave0>; o1: ...")."""
        n = ctypes.c_size_t()
        self._check(self._L.sift_last_pass_kernels(self._h, None, 0, ctypes.byref(n)), "sift_last_pass_kernels")
        buf = ctypes.create_string_buffer(n.value + 1)
        self._check(self._L.sift_last_pass_kernels(self._h, buf, n.value + 1, ctypes.byref(n)), "sift_last_pass_kernels")
        return buf.value.decode()

    def stream(self):
        return self._L.sift_stream(self._h)

    def synchronize(self):
        self._check(self._L.sift_synchronize(self._h), "sift_synchronize")


def flatten_pyramid(planes):
    """[[2D arrays per scale] per octave] -> flat fp32 octave-major buffer."""
    return np.concatenate([np.asarray(p, dtype=np.float32).ravel() for octv in planes for p in octv])
