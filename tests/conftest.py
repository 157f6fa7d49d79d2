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


@pytest.fixture(scope="session", autouse=True)
def _hip_path_only():
    """On a GPU, no Go-API-mirror call may have fallen back to the host copy (seb_fallback_count):
    the parity the GPU tests show is the HIP path's.  tests/test_fallback.py forces fallbacks in
    child processes only."""
    yield
    mod = sys.modules.get("seb_bloom")
    if mod is None or mod._lib is None:
        return
    import torch

    if torch.cuda.is_available():
        assert mod.fallback_count() == 0, f"{mod.fallback_count()} CPU fallbacks on a GPU run"
