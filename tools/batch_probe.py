#!/usr/bin/env python3
"""Per-call timing of rse_reconstruct_batch (each call on its own: host wall
time and HIP events), to see the spread tools/tune.py's median hides.

    python3 tools/batch_probe.py --field 16 --k 20 --p 8 --shard-kib 4 \
        --stripes 65536 --erasures 4 --calls 20 [--set KEY=VALUE ...]
"""
import argparse
import os
import statistics
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "reed-solomon-erasure_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--field", type=int, default=16)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--shard-kib", type=int, default=4)
    ap.add_argument("--stripes", type=int, default=65536)
    ap.add_argument("--erasures", type=int, default=4)
    ap.add_argument("--calls", type=int, default=20)
    ap.add_argument("--set", action="append", default=[])
    ap.add_argument("--device-flags", action="store_true", help="flags in HBM (read in place)")
    a = ap.parse_args()
    lib = R._lib.load()
    for kv in a.set:
        key, val = (int(x) for x in kv.split("="))
        assert lib.rse_set_option(key, val) == 0
    k, p, S, L = a.k, a.p, a.stripes, a.shard_kib * 1024
    T = k + p
    buf = torch.empty(S * T * L, dtype=torch.uint8, device="cuda")
    fill_splitmix(buf, 1, 0)
    r = R.core.ReedSolomon(k, p, a.field)
    elems = L // (a.field // 8)
    rng = np.random.default_rng(5)
    pres = np.ones((S, T), bool)
    for s in range(S):
        pres[s, rng.choice(T, a.erasures, replace=False)] = False
    miss = (~pres[:, :k]).sum(axis=1)
    if a.device_flags:
        pres = torch.from_numpy(pres).cuda()
    nbytes = int((miss > 0).sum() * k + miss.sum()) * L
    r.reconstruct_batch(buf, elems, S, pres, data_only=True)
    torch.cuda.synchronize()
    ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    wall, gpu = [], []
    for _ in range(a.calls):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev[0].record()
        r.reconstruct_batch(buf, elems, S, pres, data_only=True)
        ev[1].record()
        torch.cuda.synchronize()
        wall.append(time.perf_counter() - t0)
        gpu.append(ev[0].elapsed_time(ev[1]) * 1e-3)
    print(f"reconstruct_batch GF(2^{a.field}) {k}+{p} x {a.shard_kib} KiB x {S}, "
          f"{a.erasures} erasures per stripe, {nbytes / 1e9:.2f} GB per call, flags in "
          f"{'HBM' if a.device_flags else 'host memory'}")
    for w, g in zip(wall, gpu):
        print(f"  wall {w * 1e3:7.3f} ms ({nbytes / w / 1e9:7.1f} GB/s)   events "
              f"{g * 1e3:7.3f} ms ({nbytes / g / 1e9:7.1f} GB/s)")
    print(f"median wall {statistics.median(wall) * 1e3:.3f} ms = "
          f"{nbytes / statistics.median(wall) / 1e9:.1f} GB/s; median events "
          f"{statistics.median(gpu) * 1e3:.3f} ms = {nbytes / statistics.median(gpu) / 1e9:.1f} GB/s")


if __name__ == "__main__":
    main()
