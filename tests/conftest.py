import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "fccf-pcr_amd")
for p in (PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run with -m gpu")


@pytest.fixture(scope="session")
def fccf():
    import fccf_amd
    return fccf_amd


@pytest.fixture(scope="session")
def oracle():
    import oracle_py
    return oracle_py


@pytest.fixture(scope="session")
def ctx(fccf):
    c = fccf.Ctx(0, debug=True)
    yield c
    c.close()
