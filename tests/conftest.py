import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


_GOLDEN_CACHE = {}


def golden(name):
    """A committed fixture, fully materialised (NpzFile re-inflates on every access)."""
    import numpy as np
    if name not in _GOLDEN_CACHE:
        with np.load(os.path.join(GOLDEN, name)) as z:
            _GOLDEN_CACHE[name] = {k: z[k] for k in z.files}
    return _GOLDEN_CACHE[name]


@pytest.fixture(scope="session")
def pkg():
    """The product package (hyphenated directory, loaded as ``nfsp_amd``)."""
    import __graft_entry__
    return __graft_entry__.load_package()


@pytest.fixture(scope="session")
def lib(pkg):
    """The HIP C-ABI library, loaded; GPU tests only."""
    return pkg.native.lib()
