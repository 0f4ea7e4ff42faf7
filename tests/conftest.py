import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
import s2v_import  # noqa: E402,F401  (registers the ``s2v_amd`` package)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libs2v.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, f"{name}.npz"))
    return load


@pytest.fixture(params=["f32", "bf16x3", "f16x3"])
def prec(request):
    """Run a test once per conv arithmetic mode (s2v_amd.ops.set_precision): exact fp32 MFMA and
    the split-fp32 forms on the bf16 and f16 MFMAs (f16x3 is the default)."""
    from s2v_amd import ops
    prev = ops.set_precision(request.param)
    yield request.param
    ops.set_precision(prev)
