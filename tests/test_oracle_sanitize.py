"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer.

`make -C oracle asan selftest` builds oracle/oracle_selftest.c against
sift_oracle.c twice: instrumented (-fsanitize=address,undefined,
-fno-sanitize-recover=all, so any finding aborts) and plain.  The driver runs
every oracle entry point over tiny / odd / deep-octave shapes, all three
convolution orders, serial and threaded scans and capacity-limited calls; the
two builds' output checksums must agree line for line.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None and shutil.which("cc") is None, reason="no C compiler")
def test_oracle_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "asan", "selftest"], capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and "asan" in r.stderr.lower() and "cannot find" in r.stderr.lower():
        pytest.skip("libasan not installed: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    a = subprocess.run([os.path.join(ORACLE, "oracle_selftest_asan")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert a.returncode == 0, a.stdout[-2000:] + a.stderr[-4000:]
    assert "runtime error" not in a.stderr and "ERROR: AddressSanitizer" not in a.stderr, a.stderr[-4000:]
    p = subprocess.run([os.path.join(ORACLE, "oracle_selftest")], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-2000:]
    assert a.stdout == p.stdout
    lines = a.stdout.splitlines()
    assert lines[-1] == "OK" and len(lines) == 33
    assert sum(int(l.split(" kp ")[1].split()[0]) for l in lines[:-1]) > 100
