"""Cost of page-locking host memory (sift_host_register = hipHostRegister)
for touched anonymous buffers, with and without transparent huge pages --
the N-API result pool registers a recycled buffer on its first reuse.
usage: python tools/register_probe.py"""
import ctypes
import mmap
import sys
import time

sys.path.insert(0, "sift-scale-space-extrema-detection_amd")
import sift_amd  # noqa: E402

L = sift_amd.lib()
ctx = sift_amd.Context(0)  # initialises the device
for huge in (False, True):
    for mb in (1, 4, 16, 64):
        n = mb << 20
        m = mmap.mmap(-1, n)
        if huge and hasattr(mmap, "MADV_HUGEPAGE"):
            m.madvise(mmap.MADV_HUGEPAGE)
        m.write(b"\1" * n)  # touch every page
        p = ctypes.c_void_p(ctypes.addressof(ctypes.c_char.from_buffer(m)))
        t0 = time.perf_counter()
        rc = L.sift_host_register(p, n)
        t1 = time.perf_counter()
        rc2 = L.sift_host_unregister(p)
        t2 = time.perf_counter()
        print("huge=%d %3d MB: register %.2f ms (%.0f MB/s) rc %d, unregister %.2f ms rc %d" %
              (huge, mb, 1e3 * (t1 - t0), mb / max(t1 - t0, 1e-9), rc, 1e3 * (t2 - t1), rc2))
        del p
        m.close()
