#!/usr/bin/env python3
"""Which outputs / planes of a bit-sliced syndrome reconstruct differ from the
oracle, per erasure pattern and RSE_OPT_RECON_MIX (debugging aid)."""
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
sys.path.insert(0, ROOT)
import reed_solomon_erasure as R  # noqa: E402
from oracle import oracle as O  # noqa: E402

lib = R._lib.load()
k, p, field = 20, 8, 16
nbytes = 16384 * 2
rng = np.random.default_rng(1)
full = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(k)] + \
       [np.zeros(nbytes, np.uint8) for _ in range(p)]
O.Codec(field, k, p).encode(full)
r = R.core.ReedSolomon(k, p, field)
pats = [list(range(8)), list(range(7)), [0, 1, 2, 3, 4, 5, 20, 21], [0, 1, 2, 3, 4, 5, 20, 27],
        [0, 1, 2, 3, 4, 5, 26, 27], [0, 1, 2, 3, 4, 5, 6, 27], [0, 1, 2, 3, 4, 5, 6, 20]]
for mix in (2, 1):
    lib.rse_set_option(17, mix)
    for erased in pats:
        present = [i not in erased for i in range(k + p)]
        tb = [torch.from_numpy(x.copy()).cuda().view(-1, 2) for x in full]
        for e in erased:
            tb[e].fill_(0x33)
        r.reconstruct_data(list(zip(tb, present)))
        torch.cuda.synchronize()
        bad = []
        for i in erased:
            if i >= k:
                continue
            got = tb[i].cpu().numpy().reshape(-1)
            d = got ^ full[i]
            if d.any():
                u16 = d.view(np.uint16)
                bits = [b for b in range(16) if ((u16 >> b) & 1).any()]
                bad.append((i, int((u16 != 0).mean() * 1000), bits))
        print(f"mix={mix} erased={erased} kernel={R.core.last_kernel()} bad={bad}", flush=True)
