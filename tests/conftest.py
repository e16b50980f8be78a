import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "neo-dsp_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libneo_hip.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # test infrastructure (CPU restatement)

    O.build()
    return O


@pytest.fixture(scope="session")
def neo_gpu():
    import neo

    neo._native.require_gpu()
    return neo


def peak_err(y, ref):
    import numpy as np

    y = np.asarray(y)
    ref = np.asarray(ref)
    scale = max(float(np.abs(ref).max()), 1e-30)
    return float(np.abs(y.astype(np.complex128) - ref.astype(np.complex128)).max()) / scale
