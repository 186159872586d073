#!/usr/bin/env python3
"""Why bench.py's pinned-host flat encode leg (extra_legs) reads about half of
the same call in host_leg: the same measurement -- 8 stripes
of 10+4 x 16 MiB through rse_encode_host_flat -- repeated after each step of
a bench-like process, with the library's per-call resource sets counted, and
variants at the point where it is slow (debugging aid, GPU box only)."""
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402

MiB = 1 << 20
k, p, L = 10, 4, 16 * MiB
S = int(os.environ.get("PROBE_STRIPES", "64"))
lib = R._lib.load()
ns = 8


def live():
    return lib.rse_get_option(24)  # RSE_OPT_SCRATCH_LIVE


def e2e(tag, r, hflat, reps=3):
    r.encode_host_flat(hflat, L, ns)
    t0 = time.perf_counter()
    for _ in range(reps):
        r.encode_host_flat(hflat, L, ns)
    dt = (time.perf_counter() - t0) / reps
    print(f"{tag:58s} {ns * (k + p) * L / dt / 1e9:6.1f} GB/s data+parity  "
          f"(H2D {ns * k * L / dt / 1e9:5.1f})  scratch sets {live()}", flush=True)


def main():
    v = torch.empty((S, k + p, L), dtype=torch.uint8, device="cuda")
    for s in range(S):
        for i in range(k):
            fill_splitmix(v[s, i], bench.SEED, bench.shard_id(s, i))
    r = R.galois_8.ReedSolomon(k, p)
    r.encode_flat(v.view(-1), L, S)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    h1 = v[:ns].reshape(-1).cpu().pin_memory()
    e2e("host_leg's buffer, first calls", r, h1)
    e2e("again", r, h1)
    del h1
    ids = list(range(S))
    n = min(S, 64)
    lib.rse_set_option(11, 0)
    bench.reconstruct_leg(r, v, k, [0, 1], L, n, stream, fill_splitmix, ids[:n], None)
    lib.rse_set_option(11, 1)
    h2 = v[:ns].reshape(-1).cpu().pin_memory()
    e2e("new pinned buffer, after a syndrome reconstruct leg", r, h2)
    old = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)
    bench.reconstruct_leg(r, v, k, [0, 1], L, n, stream, fill_splitmix, ids[:n], None, reps=5)
    lib.rse_set_option(9, old)
    e2e("after the cached-pattern reconstruct leg", r, h2)
    bench.verify_leg(r, v, k, p, L, min(n, 64), reps=5)
    e2e("after the verify legs", r, h2)
    hs = [v[0, i].cpu().pin_memory() for i in range(k)] + \
         [torch.empty(L, dtype=torch.uint8).pin_memory() for _ in range(p)]
    for _ in range(6):
        r.encode_host(hs)
    e2e("after 6 one-stripe encode_host calls", r, h2)
    h3 = v[:ns].reshape(-1).cpu().pin_memory()
    h3.view(ns, k + p, L)[:, k:].zero_()
    e2e("bench's flat buffer (made after the one-stripe calls)", r, h3)
    ok = torch.equal(h3.view(ns, k + p, L)[:, k:], v[:ns, k:].cpu())
    print("parity ok:", ok, flush=True)
    for nh in (1, 2, 3, 4):
        lib.rse_set_option(8, nh)  # new pipeline streams for this (nh, ring)
        e2e(f"  RSE_OPT_HOST_H2D_STREAMS {nh}", r, h3)
    lib.rse_set_option(8, 2)
    lib.rse_set_option(21, 0)
    e2e("  no 2D copies", r, h3)
    lib.rse_set_option(21, 1)
    for kib in (1024, 2048, 8192):
        lib.rse_set_option(7, kib)
        e2e(f"  chunk {kib} KiB", r, h3)
    lib.rse_set_option(7, 4096)
    e2e("  defaults again", r, h3)
    e2e("  old buffer h2 again", r, h2)
    # plain copies of the same bytes in this process (the PCIe ceiling)
    d = torch.empty_like(h3, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        d.copy_(h3, non_blocking=True)
    torch.cuda.synchronize()
    print(f"plain pinned H2D copy of the flat buffer {3 * h3.numel() / (time.perf_counter() - t0) / 1e9:.1f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
