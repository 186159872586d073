#!/usr/bin/env python3
"""Bytes of the 1 / 2 KiB-shard kernels built under RSE_OPT_SUB_DEPTH (argv[1])
against the oracle: encode of 8+8 and 4+4 x 1 KiB and 5+2 x 2 KiB flat
batches, and reconstruct of one lost shard of 16+16 x 1 KiB (its pattern
kernel), every stripe checked.  Test infrastructure (imports the oracle)."""
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reed-solomon-erasure_amd")]
import reed_solomon_erasure as R  # noqa: E402
from oracle import oracle as O  # noqa: E402

lib = R._lib.load()
assert lib.rse_set_option(50, int(sys.argv[1])) == 0
assert lib.rse_set_option(9, 2) == 0  # wait for the modules (prebuilt in jitcache/)
rng = np.random.default_rng(50)
bad = 0
for k, p, L, S in ((8, 8, 1024, 1003), (4, 4, 1024, 2049), (5, 2, 2048, 777)):
    r = R.core.ReedSolomon(k, p, 8)
    host = rng.integers(0, 256, (S, k + p, L), dtype=np.uint8)
    buf = torch.from_numpy(host.copy()).cuda()
    r.encode_flat(buf.view(-1), L, S)
    got = buf.cpu().numpy()
    oc = O.Codec(8, k, p)
    for s in range(S):
        sh = [host[s, i].copy() for i in range(k)] + [np.zeros(L, np.uint8) for _ in range(p)]
        oc.encode(sh)
        for j in range(p):
            bad += int(not (got[s, k + j] == sh[k + j]).all())
    print(f"encode {k}+{p} x {L}: {S} stripes, kernel {R.core.last_kernel()}", flush=True)
k, p, L, S = 16, 16, 1024, 1001
r = R.core.ReedSolomon(k, p, 8)
host = rng.integers(0, 256, (S, k + p, L), dtype=np.uint8)
buf = torch.from_numpy(host.copy()).cuda()
r.encode_flat(buf.view(-1), L, S)
want = buf.cpu().numpy().copy()
present = [i != 0 for i in range(k + p)]
for rep in range(2):  # the second use runs the pattern kernel
    buf.view(S, k + p, L)[:, 0] = 0x33
    r.reconstruct_data_flat(buf.view(-1), L, S, present)
    got = buf.cpu().numpy()
    bad += int(not (got == want).all())
    print(f"reconstruct 16+16 x 1 KiB, shard 0 lost (use {rep + 1}): kernel {R.core.last_kernel()}",
          flush=True)
print("mismatches", bad)
sys.exit(1 if bad else 0)
