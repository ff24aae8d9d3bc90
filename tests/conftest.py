import os
import sys

import numpy as np
import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(REPO, "pnp-pds_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_ops():
    return load_golden("ops.npz")


@pytest.fixture(scope="session")
def golden_denoiser():
    return load_golden("denoiser.npz")


@pytest.fixture(scope="session")
def gpu_ctx():
    """One device context for the whole GPU session (tests run in one process)."""
    from pnppds import _lib
    ctx = _lib.Context(0)
    ctx.set_precision("fp16")   # the denoiser tests on this context target the fp16 path unless they set another
    yield ctx
    ctx.close()
