import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library on cuda:0)")
    config.addinivalue_line("markers", "slow: full-size configurations")


@pytest.fixture(scope="session")
def oracle():
    import scenes
    return scenes.OracleFactory()


@pytest.fixture(scope="session")
def gpu():
    """The HIP library through its Pybind mirror.  Fails (never skips) when no
    device is usable: the GPU tests must not pass on a fallback."""
    import scenes
    # torch's HIP runtime first (the tests that hand the library torch tensors
    # need torch's device view; with the library's runtime loaded first, torch
    # found no device when such a test ran before any other torch use)
    import torch
    torch.cuda.init()
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    if R.device_count() <= 0:
        pytest.fail("no HIP device visible: GPU tests need an MI355X")
    return scenes.GpuFactory()


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "scenes.npz")))
