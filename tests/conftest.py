import os
import sys

import pytest

# Descriptor pointer fields take tensors (held by the descriptor) or None, never raw addresses
# (hiseg._lib.Desc): the suite runs in strict mode, rank processes it spawns inherit it.
os.environ.setdefault("HISEG_STRICT_PTRS", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "human-instance-segmentation_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhiseg on cuda:0)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
