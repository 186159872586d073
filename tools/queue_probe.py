#!/usr/bin/env python3
"""The pinned-host pipeline (rse_encode_host_flat, 8 stripes of 10+4 x 16 MiB)
against the hardware queues its streams land on: with 0..6
other streams in the process (each used once, so it holds a queue), the same
call under RSE_OPT_HOST_QUEUES 0 (plain streams: HIP maps them least-used onto
GPU_MAX_HW_QUEUES queues per priority) and 1 (the D2H stream at high
priority; session r06/s4 also had a CU-masked stream per pipeline stream,
a queue each, which measured the same).  Every mode change re-creates the
pipeline's streams.  GPU box only."""
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
k, p, L, ns = 10, 4, 16 * MiB, 8
QUEUES = 52
lib = R._lib.load()


def rate(r, h, reps=3):
    r.encode_host_flat(h, L, ns)
    t0 = time.perf_counter()
    for _ in range(reps):
        r.encode_host_flat(h, L, ns)
    return ns * (k + p) * L / ((time.perf_counter() - t0) / reps) / 1e9


def main():
    v = torch.empty((ns, k + p, L), dtype=torch.uint8, device="cuda")
    for s in range(ns):
        for i in range(k):
            fill_splitmix(v[s, i], bench.SEED, bench.shard_id(s, i))
    r = R.galois_8.ReedSolomon(k, p)
    r.encode_flat(v.view(-1), L, ns)
    torch.cuda.synchronize()
    h = v.reshape(-1).cpu().pin_memory()
    h.view(ns, k + p, L)[:, k:].zero_()
    others = []
    print("other streams | GB/s data+parity by RSE_OPT_HOST_QUEUES (0 / 1), twice", flush=True)
    for n_other in (0, 1, 2, 3, 4, 6):
        while len(others) < n_other:
            s_ = torch.cuda.Stream()
            with torch.cuda.stream(s_):
                torch.zeros(1, device="cuda").add_(1)  # the stream takes its queue
            others.append(s_)
        torch.cuda.synchronize()
        row = []
        for mode in (0, 1, 0, 1):
            assert lib.rse_set_option(QUEUES, mode) == 0
            row.append(f"{rate(r, h):6.1f}")
        print(f"{n_other:13d} | " + " ".join(row), flush=True)
    ok = torch.equal(h.view(ns, k + p, L)[:, k:], v[:, k:].cpu())
    print("parity ok:", ok, flush=True)
    d = torch.empty_like(h, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    print(f"plain pinned H2D copy {3 * h.numel() / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
