"""pytest config: registers the `gpu` marker and puts the repo root on sys.path.

`-m "not gpu"` runs here on CPU (oracle vs golden vectors, host logic, ABI
exports, gloo multi-process).  `-m gpu` is the parity suite proper: it calls
the HIP path through the C ABI and fails -- never skips -- without a GPU.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")


# The property tests (tests/test_properties.py, tests/test_gpu_properties.py)
# run derandomised by default -- the same generated cases every run, so the
# suite is repeatable -- and explore new cases with
# GEV_HYPOTHESIS_PROFILE=explore (plus --hypothesis-seed=N to pin a sweep).
try:
    from hypothesis import settings as _hsettings

    _hsettings.register_profile("ci", derandomize=True)
    _hsettings.register_profile("explore", derandomize=False)
    _hsettings.load_profile(os.environ.get("GEV_HYPOTHESIS_PROFILE", "ci"))
except ImportError:  # hypothesis is in the image; the property tests need it
    pass


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    d = np.load(os.path.join(ROOT, "tests", "golden", "ws_golden.npz"))
    cases = sorted({k.split("/")[0] for k in d.files})
    return {c: {k.split("/")[1]: d[k] for k in d.files if k.startswith(c + "/")} for c in cases}


@pytest.fixture(scope="session")
def engine():
    import gev_amd
    if gev_amd.device_count() < 1:
        pytest.fail("gpu test without a HIP device: the decode path has no CPU fallback")
    e = gev_amd.Engine(0)
    yield e
    e.close()
