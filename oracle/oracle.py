"""ctypes wrapper of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

The oracle (sift_oracle.c) is an fp64 C restatement of the reference's
algorithm, pinned against golden vectors produced by the reference itself
(tests/golden).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may use it, as the checker / CPU baseline -- the product
path (libsift_hip.so) never links or calls it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

CONV_2D = 0                 # the reference's 2D kernel and summation order
CONV_SEPARABLE = 1          # the same operator, rows then columns
CONV_SEPARABLE_FMA_VH = 2   # columns then rows, fma chains: the HIP path's own order (bit-exact pin)


class OracleParams(ctypes.Structure):
    _fields_ = [("num_octaves", ctypes.c_int), ("scales_per_octave", ctypes.c_int),
                ("min_blur", ctypes.c_double), ("assumed_blur", ctypes.c_double),
                ("min_interpixel_distance", ctypes.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        lp = ctypes.POINTER(ctypes.c_long)
        pp = ctypes.POINTER(OracleParams)
        L.oracle_octave_dims.restype = ctypes.c_long
        L.oracle_octave_dims.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ip]
        L.oracle_schedule.argtypes = [pp, dp, dp]
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_set_threads.restype = None
        L.oracle_scale_space.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int,
                                         pp, ctypes.c_int, dp]
        L.oracle_dog.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, dp]
        L.oracle_find_extrema.restype = ctypes.c_long
        L.oracle_find_extrema.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, ip, dp, ctypes.c_long, lp]
        L.oracle_find_extrema_ex.restype = ctypes.c_long
        L.oracle_find_extrema_ex.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, ip, dp, ctypes.c_long, ip, dp,
                                             ctypes.c_long, lp]
        L.oracle_refine.restype = ctypes.c_long
        L.oracle_refine.argtypes = [pp, ctypes.c_int, ctypes.c_int, dp, ip, dp, ctypes.c_long, dp,
                                    ctypes.c_long, lp]
        L.oracle_detect_count.restype = ctypes.c_long
        L.oracle_detect_count.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int,
                                          pp, ctypes.c_int, lp]
        _lib = L
    return _lib


def _ptr(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def make_params(num_octaves, scales_per_octave, min_blur=0.8, assumed_blur=0.5,
                min_interpixel_distance=0.5):
    return OracleParams(int(num_octaves), int(scales_per_octave), float(min_blur),
                        float(assumed_blur), float(min_interpixel_distance))


def octave_dims(W, H, O):
    d = np.zeros(2 * O, dtype=np.int32)
    lib().oracle_octave_dims(W, H, O, _ptr(d, ctypes.c_int32))
    return [(int(d[2 * o]), int(d[2 * o + 1])) for o in range(O)]


def schedule(p):
    NS = p.scales_per_octave + 3
    blur = np.zeros(p.num_octaves * NS)
    sig = np.zeros(p.num_octaves * NS)
    lib().oracle_schedule(ctypes.byref(p), _ptr(blur, ctypes.c_double), _ptr(sig, ctypes.c_double))
    return blur.reshape(-1, NS), sig.reshape(-1, NS)


def split_pyramid(flat, dims, per_octave):
    out, off = [], 0
    for (h, w) in dims:
        n = h * w * per_octave
        out.append(flat[off:off + n].reshape(per_octave, h, w))
        off += n
    return out


def extrema_lists(p, W, H, dog_flat):
    """Candidate and low-contrast extrema of a flat fp64 DoG pyramid (any
    source: computed here or the fp32 planes a caller loads), reference order:
    ((rec (N,4) int32, value (N,)), (low_rec, low_value))."""
    L = lib()
    dog_flat = np.ascontiguousarray(dog_flat, dtype=np.float64)
    low = ctypes.c_long(0)
    dogp = _ptr(dog_flat, ctypes.c_double)
    n = L.oracle_find_extrema_ex(ctypes.byref(p), W, H, dogp, None, None, 0, None, None, 0, ctypes.byref(low))
    nl = int(low.value)
    rec = np.zeros((max(n, 1), 4), dtype=np.int32)
    val = np.zeros(max(n, 1))
    low_rec = np.zeros((max(nl, 1), 4), dtype=np.int32)
    low_val = np.zeros(max(nl, 1))
    L.oracle_find_extrema_ex(ctypes.byref(p), W, H, dogp, _ptr(rec, ctypes.c_int32), _ptr(val, ctypes.c_double), n,
                             _ptr(low_rec, ctypes.c_int32), _ptr(low_val, ctypes.c_double), nl, ctypes.byref(low))
    return (rec[:n], val[:n]), (low_rec[:nl], low_val[:nl])


def as_records(rec, val):
    """(N,5) [octave, scale, x, y, value] rows of an extrema list."""
    c = np.zeros((rec.shape[0], 5))
    c[:, :4] = rec
    c[:, 4] = val
    return c


class OracleRun:
    """Full oracle pipeline on one image; keeps flat fp64 pyramids."""

    def __init__(self, img, p, mode=CONV_SEPARABLE, threads=1, keep_gauss=True):
        """threads: OpenMP threads of the blur loops and the extrema scan
        (identical results for any count).  keep_gauss=False frees the
        Gaussian pyramid once the DoG is formed (large images)."""
        img = np.ascontiguousarray(img, dtype=np.float32)
        H, W = img.shape
        self.W, self.H, self.p = W, H, p
        O, S = p.num_octaves, p.scales_per_octave
        self.dims = octave_dims(W, H, O)
        P = sum(h * w for h, w in self.dims)
        L = lib()
        set_threads(threads)
        try:
            gauss_flat = np.zeros(P * (S + 3))
            L.oracle_scale_space(_ptr(img, ctypes.c_float), W, H, ctypes.byref(p), mode,
                                 _ptr(gauss_flat, ctypes.c_double))
            self.dog_flat = np.zeros(P * (S + 2))
            L.oracle_dog(ctypes.byref(p), W, H, _ptr(gauss_flat, ctypes.c_double),
                         _ptr(self.dog_flat, ctypes.c_double))
            if keep_gauss:
                self.gauss_flat = gauss_flat
                self.gauss = split_pyramid(self.gauss_flat, self.dims, S + 3)
            del gauss_flat
            self.dog = split_pyramid(self.dog_flat, self.dims, S + 2)
            (self.cand_rec, self.cand_val), (self.low_rec, self.low_val) = extrema_lists(p, W, H, self.dog_flat)
        finally:
            set_threads(1)
        self.n_low = self.low_rec.shape[0]
        self.refined, self.n_singular = self.refine(self.cand_rec, self.cand_val)

    def low_contrast(self):
        """(N,5) [octave, scale, x, y, value] of the low-contrast extrema, reference order."""
        return as_records(self.low_rec, self.low_val)

    def refine(self, rec, val):
        rec = np.ascontiguousarray(rec, dtype=np.int32)
        val = np.ascontiguousarray(val, dtype=np.float64)
        n = rec.shape[0]
        out = np.zeros((max(n, 1), 8))
        sing = ctypes.c_long(0)
        k = lib().oracle_refine(ctypes.byref(self.p), self.W, self.H,
                                _ptr(self.dog_flat, ctypes.c_double), _ptr(rec, ctypes.c_int32),
                                _ptr(val, ctypes.c_double), n, _ptr(out, ctypes.c_double), n,
                                ctypes.byref(sing))
        return out[:k], int(sing.value)

    def candidates(self):
        """(N,5) [octave, scale, x, y, value] in reference order."""
        return as_records(self.cand_rec, self.cand_val)


def detect_count(img, p, mode=CONV_2D):
    img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = img.shape
    nc = ctypes.c_long(0)
    nk = lib().oracle_detect_count(_ptr(img, ctypes.c_float), W, H, ctypes.byref(p), mode,
                                   ctypes.byref(nc))
    return int(nk), int(nc.value)


def set_threads(n):
    """Threads of the oracle's blur loops (results are identical for any n)."""
    lib().oracle_set_threads(int(n))
