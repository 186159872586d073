"""Builds run-time specialised modules on the host CPU into a JIT disk cache
(rse_jit.cpp: hiprtc needs no GPU), so a GPU session loads them in
milliseconds instead of spending box time in hiprtc.

    RSE_JIT_CACHE_DIR=jitcache python3 tools/prebuild_jit.py \
        --codec 8:50:20 --codec 16:40:12 --set 26=1,26=2,26=3
Each --set entry is a comma list of KEY=VALUE options applied before the
codecs are created.  A process registers each codec once (modules are keyed by
rows, not options), so run one process per option set."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "reed-solomon-erasure_amd"))
import reed_solomon_erasure as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--codec", action="append", default=[], help="field:k:p")
ap.add_argument("--set", action="append", default=[], help="KEY=VALUE,KEY=VALUE")
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
print("built", lib.rse_get_option(10), "cache hits", lib.rse_get_option(16))
