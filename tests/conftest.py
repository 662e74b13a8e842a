import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "sift-scale-space-extrema-detection_amd"), os.path.join(ROOT, "oracle"),
          os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def gpu_ctx():
    # torch (its own bundled HIP runtime) must initialise the device before
    # libsift_hip.so's runtime does, as bench.py does: the other order leaves
    # torch with "No HIP GPUs are available" for the tests that hand torch
    # device tensors to the library.
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except ImportError:
        pass
    import sift_amd
    ctx = sift_amd.Context(0)
    yield ctx
    ctx.close()
