"""Builds run-time specialised modules on the host CPU into a JIT disk cache
(rse_jit.cpp: hiprtc needs no GPU), so a GPU session loads them in
milliseconds instead of spending box time in hiprtc.

    RSE_JIT_CACHE_DIR=jitcache python3 tools/prebuild_jit.py \
        --codec 8:50:20 --codec 16:40:12 --set 26=1,26=2,26=3
Each --set entry is a comma list of KEY=VALUE options applied before the
codecs are created.  A process registers each codec once (modules are keyed by
rows, not options), so run one process per option set.

--pattern field:k:p:shard_bytes:e0,e1,... builds the decode-pattern module of
those erased shards (what a repeated reconstruct of that pattern runs,
rse_codec.cpp pattern_kernel): a reconstruct call on host buffers under
RSE_OPT_JIT 2 builds it, and then fails for want of a GPU, which is expected
here."""
import argparse
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "reed-solomon-erasure_amd"))
import reed_solomon_erasure as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--codec", action="append", default=[], help="field:k:p")
ap.add_argument("--set", action="append", default=[], help="KEY=VALUE,KEY=VALUE")
ap.add_argument("--pattern", action="append", default=[], help="field:k:p:shard_bytes:e0,e1,...")
args = ap.parse_args()
assert os.environ.get("RSE_JIT_CACHE_DIR"), "set RSE_JIT_CACHE_DIR"
lib = R._lib.load()
for opts in args.set or [""]:
    kv = [tuple(int(x) for x in o.split("=")) for o in opts.split(",") if o]
    for key, val in kv:
        assert lib.rse_set_option(key, val) == 0, key
    for spec in args.codec:
        f, k, p = (int(x) for x in spec.split(":"))
        r = R.core.ReedSolomon(k, p, f)
        print(opts or "defaults", spec, r.kernel_kind(wait=True), flush=True)
if args.pattern:
    import ctypes
    import numpy as np
    old = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)
    for spec in args.pattern:
        f, k, p, nb, er = spec.split(":")
        f, k, p, nb = int(f), int(k), int(p), int(nb)
        erased = [int(x) for x in er.split(",")]
        T = k + p
        r = R.core.ReedSolomon(k, p, f)
        bufs = [np.zeros(nb, np.uint8) for _ in range(T)]
        ptrs = (ctypes.c_void_p * T)(*[b.ctypes.data for b in bufs])
        lens = (ctypes.c_size_t * T)(*([nb // (f // 8)] * T))
        pres = (ctypes.c_uint8 * T)(*[0 if i in erased else 1 for i in range(T)])
        before = lib.rse_get_option(10) + lib.rse_get_option(16)
        lib.rse_reconstruct(r._h, ptrs, lens, pres, T, None)  # fails after the build
        print("pattern", spec, "modules", lib.rse_get_option(10) + lib.rse_get_option(16) - before,
              flush=True)
    lib.rse_set_option(9, old)
print("built", lib.rse_get_option(10), "cache hits", lib.rse_get_option(16))
