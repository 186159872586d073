#!/usr/bin/env python3
"""Why the bench's pinned-host encode pipeline is slower than tools/host_e2e.py:
the same measurement (8 stripes 10+4 x 16 MiB, rse_encode_host_flat) at
points of a bench-like process (debugging aid)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402

MiB = 1 << 20
k, p, L, S = 10, 4, 16 * MiB, int(os.environ.get("PROBE_STRIPES", "512"))
v = torch.empty((S, k + p, L), dtype=torch.uint8, device="cuda")
for s in range(8):
    for i in range(k):
        fill_splitmix(v[s, i], bench.SEED, bench.shard_id(s, i))
r = R.galois_8.ReedSolomon(k, p)
r.encode_flat(v.view(-1), L, S)
torch.cuda.synchronize()
ns = 8
hflat = v[:ns].reshape(-1).cpu().pin_memory()


def e2e(tag):
    r.encode_host_flat(hflat, L, ns)
    t0 = time.perf_counter()
    for _ in range(3):
        r.encode_host_flat(hflat, L, ns)
    dt = (time.perf_counter() - t0) / 3
    print(f"{tag:40s} {ns * (k + p) * L / dt / 1e9:6.1f} GB/s data+parity", flush=True)


e2e("first")
e2e("again")
h2 = torch.empty(hflat.numel(), dtype=torch.uint8, pin_memory=True)
h2.copy_(hflat)
hsave, hflat = hflat, h2
e2e("fresh torch.empty(pin_memory) buffer")
hflat = hsave
if os.environ.get("PROBE_SHORT"):
    sys.exit(0)
stream = torch.cuda.current_stream()
legs = bench.extra_legs(r, v, k, p, L, 256, stream)
print("bench legs e2e flat:", legs["end_to_end_pinned_host_flat"]["MB_per_s"] * MiB / 1e9, flush=True)
e2e("after extra_legs")
time.sleep(5)
e2e("after 5 s")
