#!/usr/bin/env python3
"""What the resident dispatcher's idle time costs callers that synchronise
the device or use other streams: 10+4 x 4 KiB rse_encode_now
calls, per RSE_OPT_DISPATCH_IDLE_US (and with the dispatcher off), in
microseconds per iteration of
  back_to_back:   encode_now
  then_devsync:   encode_now; torch.cuda.synchronize()
  other_stream:   a torch kernel on a second stream; encode_now; that stream
                  synchronised (does the resident kernel hold it up?)
  spaced_300us:   encode_now every 300 us (the dispatcher idles out between
                  calls when its idle time is shorter)
GPU box only."""
import os
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
import torch  # noqa: E402

import reed_solomon_erasure as R  # noqa: E402

DISPATCH, IDLE_US, LAUNCHES = 39, 40, 43
lib = R._lib.load()
k, p, n = 10, 4, 4096


def per_iter(fn, iters=200):
    fn()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    r = R.galois_8.ReedSolomon(k, p)
    t = [torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda") for _ in range(k + p)]
    x = torch.zeros(1 << 20, device="cuda")
    s2 = torch.cuda.Stream()
    torch.cuda.synchronize()

    def back():
        r.encode_now(t)

    def devsync():
        r.encode_now(t)
        torch.cuda.synchronize()

    def other():
        with torch.cuda.stream(s2):
            x.add_(1)
        r.encode_now(t)
        s2.synchronize()

    def spaced():
        t0 = time.perf_counter()
        r.encode_now(t)
        while time.perf_counter() - t0 < 300e-6:
            pass

    print(f"{'idle_us':>8} {'back_to_back':>13} {'then_devsync':>13} {'other_stream':>13} "
          f"{'spaced_300us':>13} {'launches':>9}", flush=True)
    for idle in (2000, 500, 200, 100, 50, 0):
        if idle:
            lib.rse_set_option(DISPATCH, 1)
            lib.rse_set_option(IDLE_US, idle)
        else:
            lib.rse_set_option(DISPATCH, 0)
        lib.rse_dispatcher_stop()
        l0 = lib.rse_get_option(LAUNCHES)
        row = [per_iter(back), per_iter(devsync, 50), per_iter(other), per_iter(spaced, 100)]
        name = str(idle) if idle else "off"
        print(f"{name:>8} " + " ".join(f"{v:13.1f}" for v in row)
              + f" {lib.rse_get_option(LAUNCHES) - l0:9d}", flush=True)
    lib.rse_set_option(DISPATCH, 1)


if __name__ == "__main__":
    main()
