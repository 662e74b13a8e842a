"""CPU-side checks of the C ABI: the library loads, exports exactly what
include/sift_hip.h declares, and its host-only math matches the oracle.
No compute calls here (no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle as orc
import sift_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sift_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sift_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = sift_amd.lib()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(sift_amd.ABI_SYMBOLS) == declared
    out = subprocess.run(["nm", "-D", "--defined-only", sift_amd.LIB_PATH], capture_output=True, text=True).stdout
    exported = sorted(set(re.findall(r" T (sift_[a-z_0-9]+)", out)))
    assert exported == declared


def test_abi_version_and_defaults():
    L = sift_amd.lib()
    assert L.sift_abi_version() == 9
    p = sift_amd.Params()
    assert L.sift_params_default(ctypes.byref(p)) == 0
    # src/worker.js:33-37,88
    assert (p.num_octaves, p.scales_per_octave, p.min_blur, p.assumed_blur, p.min_interpixel_distance, p.flags) == \
        (5, 3, 0.8, 0.5, 0.5, 0)


@pytest.mark.parametrize("O,S,mb,ab", [(5, 3, 0.8, 0.5), (4, 5, 0.8, 0.5), (3, 4, 1.0, 0.4), (6, 2, 0.8, 0.5)])
def test_schedule_matches_oracle(O, S, mb, ab):
    p = sift_amd.make_params(O, S, mb, ab)
    blur, sig = sift_amd.schedule(p)
    ob, osig = orc.schedule(orc.make_params(O, S, mb, ab))
    np.testing.assert_array_equal(blur, ob)
    np.testing.assert_array_equal(sig, osig)


@pytest.mark.parametrize("W,H,O", [(3840, 2160, 4), (77, 51, 4), (16, 12, 5), (1, 1, 3)])
def test_octave_dims_match_oracle(W, H, O):
    assert sift_amd.octave_dims(W, H, O) == orc.octave_dims(W, H, O)


def test_bad_arguments_are_rejected():
    L = sift_amd.lib()
    d = np.zeros(8, dtype=np.int32)
    assert L.sift_octave_dims(0, 5, 2, d.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == sift_amd.SIFT_E_ARG
    p = sift_amd.make_params(0, 3)
    b = np.zeros(16)
    assert L.sift_schedule(ctypes.byref(p), b.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                           b.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) == sift_amd.SIFT_E_UNSUPPORTED
    assert L.sift_ctx_destroy(None) == sift_amd.SIFT_E_ARG
    assert L.sift_last_error(None) == b"null context"
