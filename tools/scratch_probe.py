"""Device memory after waves of short-lived threads (per-thread
resources).  Prints free HBM and RSE_OPT_SCRATCH_LIVE after every wave for
several per-thread workloads, to tell library-held memory from the runtime's."""
import os
import sys
import threading

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "reed-solomon-erasure_amd"))
import reed_solomon_erasure as R  # noqa: E402

lib = R._lib.load()
r = R.galois_8.ReedSolomon(10, 4)
n = 3 << 20
rng = np.random.default_rng(1)
data = [torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).pin_memory() for _ in range(10)]
par = [[torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(4)] for _ in range(4)]


def nothing(i):
    torch.cuda.synchronize()


def hip_only(i):
    lib.rse_fill_splitmix(None, 0, 0, 0, None)


def encode(i):
    r.encode_host(data + par[i])


def verify(i):
    r.encode_host(data + par[i])
    assert r.verify_host(data + par[i])


for name, fn in (("nothing", nothing), ("hip_only", hip_only), ("encode", encode), ("verify", verify)):
    fn(0)
    torch.cuda.synchronize()
    base = torch.cuda.mem_get_info()[0]
    row = []
    for w in range(12):
        ts = [threading.Thread(target=fn, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()
        row.append((base - torch.cuda.mem_get_info()[0]) >> 20)
    print(f"{name:9s} MiB held after each wave: {row} live={lib.rse_get_option(24)}", flush=True)
