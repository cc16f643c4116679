import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "isl-signlanguage-translation_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    # GPU tests run one process on the box; never silently skip them there.
    pass


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    class G:
        def __getattr__(self, name):
            return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return G()
