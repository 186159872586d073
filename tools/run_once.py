#!/usr/bin/env python3
"""Run one coding configuration a few times (for rocprofv3 counter passes).

    python tools/run_once.py --field 16 --k 20 --p 8 --shard-mib 4 --stripes 32 --variant 3
"""
import argparse
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))

import torch  # noqa: E402

import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--field", type=int, default=8)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--shard-mib", type=int, default=16)
    ap.add_argument("--stripes", type=int, default=32)
    ap.add_argument("--variant", type=int, default=-1)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--op", default="encode", choices=["encode", "reconstruct"])
    a = ap.parse_args()
    lib = R._lib.load()
    lib.rse_set_option(4, a.variant)
    L = a.shard_mib << 20
    buf = torch.empty(a.stripes * (a.k + a.p) * L, dtype=torch.uint8, device="cuda")
    v = buf.view(a.stripes, a.k + a.p, L)
    for s in range(a.stripes):
        for i in range(a.k):
            fill_splitmix(v[s, i], 1, (s << 8) | i)
    r = R.core.ReedSolomon(a.k, a.p, a.field)
    n = L // (a.field // 8)
    present = [i not in (0, 1) for i in range(a.k + a.p)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(a.reps):
        ev[0].record()
        if a.op == "encode":
            r.encode_flat(buf, n, a.stripes)
        else:
            r.reconstruct_data_flat(buf, n, a.stripes, present)
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1])
        nb = a.stripes * ((a.k + a.p) if a.op == "encode" else (a.k + 2)) * L
        print(f"{a.op} gf{a.field} {a.k}+{a.p} variant {a.variant}: {ms:.3f} ms "
              f"{nb / ms / 1e6:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
