#!/usr/bin/env python3
"""Where a Python verify call's time goes (10+4 x 16 MiB, one stripe per call):
the whole call, its argument marshalling (_arrays), the stream lookup, and the
C ABI call alone with prepared arguments.  Prints one JSON line (us per call)."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "reed-solomon-erasure_amd"))
import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure import core  # noqa: E402


def per_call(fn, n=400):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


def main():
    k, p, L = 10, 4, 16 << 20
    r = R.galois_8.ReedSolomon(k, p)
    v = torch.randint(0, 256, (k + p, L), dtype=torch.uint8, device="cuda")
    sh = [v[i] for i in range(k + p)]
    r.encode(sh)
    assert r.verify(sh)
    lib = R._lib.load()
    ptrs, lens = core._arrays(sh, 8)
    ok = ctypes.c_int(0)
    st = core._stream(sh[0])
    out = {
        "verify": per_call(lambda: r.verify(sh)),
        "arrays": per_call(lambda: core._arrays(sh, 8), 4000),
        "stream": per_call(lambda: core._stream(sh[0]), 4000),
        "capi_prepared": per_call(lambda: lib.rse_verify(r._h, ptrs, lens, k + p, ctypes.byref(ok), st)),
    }
    out["verify_again"] = per_call(lambda: r.verify(sh))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
