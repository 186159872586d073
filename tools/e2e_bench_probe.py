#!/usr/bin/env python3
"""The bench's slow pinned-host flat encode leg, reproduced inside bench.py's
own sequence (headline buffer, host_leg, the buffer freed, the extra legs),
then the same rse_encode_host_flat call under variants at that point: a
repeat, new pipeline streams (RSE_OPT_HOST_QUEUES 0 / 1), per-shard copies
instead of 2D ones, H2D stream counts, chunk sizes, a fresh pinned buffer,
and plain duplex copies of the same bytes.  The other legs are skipped.
GPU box only; run under rocprofv3 --memory-copy-trace to see the copies."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)
import bench  # noqa: E402

MiB = 1 << 20
k, p, L, ns = 10, 4, 16 * MiB, 8
orig_extra = bench.extra_legs


def rate(r, h, reps=3):
    r.encode_host_flat(h, L, ns)
    t0 = time.perf_counter()
    for _ in range(reps):
        r.encode_host_flat(h, L, ns)
    dt = (time.perf_counter() - t0) / reps
    return f"{ns * (k + p) * L / dt / 1e9:6.1f} GB/s (H2D {ns * k * L / dt / 1e9:5.1f})"


def probed_extra_legs(r, v, k_, p_, L_, n_stripes, stream, stripe0=0):
    import torch
    out = orig_extra(r, v, k_, p_, L_, n_stripes, stream, stripe0)
    lib = bench.R_lib()
    f = out["end_to_end_pinned_host_flat"]
    print("bench flat leg:", f["MB_per_s"], "MB/s, first call", f["first_call_MB_per_s"],
          "outputs in place", f["outputs_in_place"], flush=True)
    h = v[:ns].reshape(-1).cpu().pin_memory()
    print(f"{'same call, new pinned buffer':44s}", rate(r, h), flush=True)
    print(f"{'again':44s}", rate(r, h), flush=True)
    for key, vals, dflt in ((53, (0, 1, 0, 1), 1), (52, (0, 1), 1), (21, (0,), 1),
                            (8, (1, 3, 4), 2), (7, (1024, 8192), 4096), (53, (0, 1), 1)):
        for val in vals:
            lib.rse_set_option(key, val)
            print(f"{f'  option {key} = {val}':44s}", rate(r, h), flush=True)
        lib.rse_set_option(key, dflt)
        print(f"{f'  option {key} back to {dflt}':44s}", rate(r, h), flush=True)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    print(f"{'after empty_cache':44s}", rate(r, h), flush=True)
    # plain duplex copies of the same bytes (two torch streams)
    d = torch.empty_like(h, device="cuda")
    hv, dv = h.view(ns, k + p, L), d.view(ns, k + p, L)
    hpar = torch.empty((ns, p, L), dtype=torch.uint8).pin_memory()
    up, down = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():
        with torch.cuda.stream(up):
            for s_ in range(ns):
                dv[s_, :k].copy_(hv[s_, :k], non_blocking=True)
        with torch.cuda.stream(down):
            for s_ in range(ns):
                hpar[s_].copy_(dv[s_, k:], non_blocking=True)
    duplex()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        duplex()
    torch.cuda.synchronize()
    print(f"{'plain duplex copies':44s} {ns * (k + p) * L / ((time.perf_counter() - t0) / 3) / 1e9:6.1f} GB/s",
          flush=True)
    return out


bench.extra_legs = probed_extra_legs
bench.other_configs = lambda stream: {}
bench.gf16_proper_leg = lambda stream: {}
bench.batch_leg = lambda stream: {}
bench.reference_bench_matrix = lambda stream: {}

if __name__ == "__main__":
    bench.main(["--no-cpu", "--steps", "5", "--warmup", "2",
                "--full-out", os.path.join(ROOT, "gpurun_out", "e2e_bench_probe.json")])
