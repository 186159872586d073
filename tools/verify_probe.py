#!/usr/bin/env python3
"""Per-call verify / encode of one 10+4 x 16 MiB stripe: wall time per call,
to set beside the kernel durations of a rocprofv3 kernel trace of this script
(how much of a synchronous call is kernel, how much launch and wake-up)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
import torch  # noqa: E402

import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402

MiB = 1 << 20
k, p, L, S = 10, 4, 16 * MiB, 16
v = torch.empty((S, k + p, L), dtype=torch.uint8, device="cuda")
fill_splitmix(v.view(-1), 1, 0)
r = R.galois_8.ReedSolomon(k, p)
r.encode_flat(v.view(-1), L, S)
torch.cuda.synchronize()
shards = [[v[s, i] for i in range(k + p)] for s in range(S)]
for name, fn in (("verify", lambda s: r.verify(shards[s])), ("encode", lambda s: r.encode(shards[s]))):
    for s in range(S):
        fn(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for rep in range(4):
        for s in range(S):
            fn(s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (4 * S)
    print(f"{name}: {dt * 1e6:7.1f} us per call, {(k + p) * L / dt / 1e9:6.1f} GB/s", flush=True)
