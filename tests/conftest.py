import os
import sys
import tempfile

import pytest

# Run-time specialised modules go to a fresh on-disk cache per test session
# (RSE_OPT_JIT_DISK_CACHE), so build counters mean builds and no run reuses
# another's modules; tests of the cache itself set their own directories.
os.environ.setdefault("RSE_JIT_CACHE_DIR", tempfile.mkdtemp(prefix="rse_jit_cache_"))

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "reed-solomon-erasure_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
