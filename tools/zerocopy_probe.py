#!/usr/bin/env python3
"""Pinned host stripes coded in place (debugging aid, GPU box only): the
device kernels of rse_encode_flat / rse_verify_flat / rse_reconstruct_data_flat
run on the device mapping of pinned host memory, so PCIe carries exactly the
bytes each kernel reads and writes and no copy engine or stream pipeline is
involved.  Set beside the rse_*_host_flat pipeline and plain copies."""
import ctypes
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
k, p, L, ns = 10, 4, 16 * MiB, 8
lib = R._lib.load()
hip = ctypes.CDLL("libamdhip64.so")


def dev_ptr(t):
    """The device mapping of a pinned host tensor (None if it has none)."""
    d = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(t.data_ptr()), 0)
    return d.value if rc == 0 else None


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return nbytes * reps / (time.perf_counter() - t0) / 1e9


def main():
    v = torch.empty((ns, k + p, L), dtype=torch.uint8, device="cuda")
    for s in range(ns):
        for i in range(k):
            fill_splitmix(v[s, i], bench.SEED, bench.shard_id(s, i))
    r = R.galois_8.ReedSolomon(k, p)
    r.encode_flat(v.view(-1), L, ns)
    torch.cuda.synchronize()
    h = v.reshape(-1).cpu().pin_memory()
    d = dev_ptr(h)
    print(f"pinned host {h.data_ptr():#x} device mapping {d and hex(d)}", flush=True)
    if d is None:
        print("no device mapping: zero-copy not tried", flush=True)
        return
    st = torch.cuda.current_stream().cuda_stream
    hv = h.view(ns, k + p, L)
    hv[:, k:].zero_()
    alg = ns * (k + p) * L
    g = rate(lambda: lib.rse_encode_flat(r._h, ctypes.c_void_p(d), L, ns, ctypes.c_void_p(st)), alg)
    ok = torch.equal(hv[:, k:], v[:, k:].cpu())
    print(f"zero-copy encode_flat        {g:6.1f} GB/s data+parity  parity ok {ok}  "
          f"kernel {lib.rse_last_kernel().decode()}", flush=True)
    oks = (ctypes.c_uint8 * ns)()
    g = rate(lambda: lib.rse_verify_flat(r._h, ctypes.c_void_p(d), L, ns, oks, ctypes.c_void_p(st)), alg)
    print(f"zero-copy verify_flat        {g:6.1f} GB/s (k+p reads)  all ok {all(oks)}", flush=True)
    pres = (ctypes.c_uint8 * (k + p))(*[0, 0] + [1] * (k + p - 2))
    want = hv[:, :2].clone()

    def rec():
        lib.rse_reconstruct_data_flat(r._h, ctypes.c_void_p(d), L, ns, pres, ctypes.c_void_p(st))
    hv[:, :2].zero_()
    g = rate(rec, ns * (k + 2) * L)
    print(f"zero-copy reconstruct_data   {g:6.1f} GB/s (k reads + 2 writes)  rebuilt ok "
          f"{torch.equal(hv[:, :2], want)}", flush=True)
    # the pipeline on the same buffer
    hv[:, k:].zero_()
    g = rate(lambda: r.encode_host_flat(h, L, ns), alg, reps=3)
    print(f"pipeline encode_host_flat    {g:6.1f} GB/s data+parity  parity ok "
          f"{torch.equal(hv[:, k:], v[:, k:].cpu())}", flush=True)
    # copy engines: one 40 MiB copy per stream on 1, 2, 4 streams at once
    dst = torch.empty(4 * 10 * 4 * MiB, dtype=torch.uint8, device="cuda")
    src = h[:4 * 10 * 4 * MiB]
    for nst in (1, 2, 4):
        sts = [torch.cuda.Stream() for _ in range(nst)]
        part = 40 * MiB

        def go():
            for j, s_ in enumerate(sts):
                with torch.cuda.stream(s_):
                    for q in range(4 // nst):
                        o = (j * (4 // nst) + q) * part
                        dst[o:o + part].copy_(src[o:o + part], non_blocking=True)
        print(f"H2D 4 x 40 MiB over {nst} stream(s)  {rate(go, 4 * part):6.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
