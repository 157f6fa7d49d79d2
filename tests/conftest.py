"""pytest setup: the `gpu` marker, import paths, shared fixtures.

CPU suite:  python -m pytest tests -m "not gpu"   (oracle vs golden vectors, host logic, ABI load)
GPU suite:  python -m pytest tests -m gpu          (HIP path vs oracle + goldens, through the C ABI)
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "storage-engines_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs the HIP library)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def seb():
    import seb_bloom
    if not os.path.exists(seb_bloom.LIB_PATH):
        seb_bloom.build_library()
    return seb_bloom
