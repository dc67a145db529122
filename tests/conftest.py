import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libsrpde_hip.so")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def conv_math():
    """Restores the conv kernel family (h3 / f32) a test switched."""
    from superresolution_for_pdes_amd import hipops as H
    before = H.conv_math()
    yield before
    H.set_conv_math(before)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    d = os.path.join(ROOT, "tests", "golden")
    return {k: np.load(os.path.join(d, f"{k}_fixture.npz")) for k in ("unet", "poisson", "datagen", "cascade",
                                                                             "unet_b1024", "cascade640")}
