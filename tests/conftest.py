"""Shared test setup.  GPU tests are marked ``@pytest.mark.gpu`` and run on a
real MI355X; everything else runs on CPU.  The CPU oracle (oracle/) is the
checker only; the product package never imports it."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures")
GOLD = os.path.join(ROOT, "tests", "golden")
REF = "/root/reference"

for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) and libpacgpu.so")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def ctx():
    import pac_amd
    from pac_amd import _lib
    c = _lib.Context(0)
    yield c
    c.close()


def fixture(name):
    """A committed reference fixture (tests/fixtures/MANIFEST.json): inputs/*.wav
    are the reference's inputs/*.wav, coded/ its verified .pac/.wak files."""
    for d in (FIX, os.path.join(FIX, "inputs"), os.path.join(FIX, "coded")):
        if os.path.exists(os.path.join(d, name)):
            return os.path.join(d, name)
    return os.path.join(FIX, name)
