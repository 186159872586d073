import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# Run-time specialised modules go to a fresh on-disk cache per test session
# (RSE_OPT_JIT_DISK_CACHE), so no run reuses another run's modules; tests of
# the cache itself set their own directories.  It starts as a copy of the
# tree's prebuilt cache (tools/prebuild_all.sh: code objects of this source,
# keyed by a hash of the whole module source, so a stale one is never hit),
# which spares the GPU box minutes of hiprtc; build counters in the tests
# count built + cached modules where a codec may be among them.
# The suite A/Bs the library's tuning switches against the oracle
# (include/rse_hip_tune.h): rse_set_option takes them only under RSE_TUNE=1.
os.environ.setdefault("RSE_TUNE", "1")

if "RSE_JIT_CACHE_DIR" not in os.environ:
    import shutil
    _cache = tempfile.mkdtemp(prefix="rse_jit_cache_")
    _pre = os.path.join(ROOT, "jitcache")
    if os.path.isdir(_pre):
        for _f in os.listdir(_pre):
            if _f.endswith(".co"):
                shutil.copy(os.path.join(_pre, _f), _cache)
    os.environ["RSE_JIT_CACHE_DIR"] = _cache

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


# Run-time modules the suite's largest codecs need (GF(2^16) 1000+24: 8 chain
# modules of 149 inputs) take ~20-45 minutes of hiprtc on a cold cache; with
# the tree's jitcache/ (tools/prebuild_all.sh) they load in milliseconds.
# Tests of such codecs wait at most JIT_BUDGET_S and then skip with that
# reason, so a cold cache cannot hold the GPU suite past its step limit.
JIT_BUDGET_S = float(os.environ.get("RSE_TEST_JIT_BUDGET_S", "60"))
_jit_timed_out = set()  # codecs whose build already outlasted the budget in this session


def kernels_or_skip(r, what, budget_s=None):
    """r.kernel_kind(wait=True) if the build finishes within the budget, else
    pytest.skip (the build goes on in the background; its helper processes
    stop when the library unloads)."""
    import threading
    budget_s = JIT_BUDGET_S if budget_s is None else budget_s
    if what in _jit_timed_out:  # one wait per session: its build is still running
        pytest.skip(f"{what}: run-time modules not in the JIT cache (cold cache; an earlier "
                    f"test waited {budget_s:.0f} s; tools/prebuild_all.sh builds them)")
    out = []
    th = threading.Thread(target=lambda: out.append(r.kernel_kind(wait=True)), daemon=True)
    th.start()
    th.join(budget_s)
    if not out:
        _jit_timed_out.add(what)
        pytest.skip(f"{what}: run-time modules not in the JIT cache and not built within "
                    f"{budget_s:.0f} s (cold cache; tools/prebuild_all.sh builds them)")
    return out[0]
