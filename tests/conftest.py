import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "riemannian-interior-point-trust-region-method_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def fixture_n50():
    import numpy as np
    d = os.path.join(GOLDEN, "nonnegpca_1")
    return (np.loadtxt(os.path.join(d, "Z.csv")), np.loadtxt(os.path.join(d, "initx_a.csv")),
            np.loadtxt(os.path.join(d, "initineqLagmult.csv")))


@pytest.fixture(scope="session")
def built_lib():
    import __graft_entry__ as g
    g.build()
    import riptrm_native
    return riptrm_native.load()
