#!/usr/bin/env python3
"""In-process A/B sweep of the fused encode kernel's launch shape on MI355X.

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24):
every configuration is timed once per round, the median over rounds reported.

    python tools/tune.py [--stripes 128] [--rounds 5] [--k 10 --p 4]

The timing-split kernels (RSE_OPT_RECON_PAIRS 4 / 5: phases skipped, wrong
bytes) exist only in the tune build: `make -C reed-solomon-erasure_amd tune`,
then run with RSE_LIB_PATH=reed-solomon-erasure_amd/build-tune/librse_hip.so.
"""
import argparse
import json
import os
import statistics
import sys
os.environ.setdefault("RSE_TUNE", "1")  # tuning switches (include/rse_hip_tune.h)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
# the tree's prebuilt run-time modules (tools/prebuild_all.sh), as bench.py
os.environ.setdefault("RSE_JIT_CACHE_DIR", os.path.join(ROOT, "jitcache"))

import torch  # noqa: E402

import reed_solomon_erasure as R  # noqa: E402
from reed_solomon_erasure.core import fill_splitmix  # noqa: E402

MiB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--p", type=int, default=4)
    ap.add_argument("--field", type=int, default=8)
    ap.add_argument("--shard-mib", type=int, default=16)
    ap.add_argument("--shard-kib", type=int, default=0, help="overrides --shard-mib")
    ap.add_argument("--op", default="encode", choices=["encode", "reconstruct", "batch"],
                    help="batch: rse_reconstruct_batch, every stripe its own random pattern "
                         "of len(--erase) erased shards")
    ap.add_argument("--variants", type=int, default=1)
    ap.add_argument("--variant-list", default="", help="comma list of variants (overrides --variants)")
    ap.add_argument("--bitslice", default="1", help="comma list of RSE_OPT_BITSLICE values")
    ap.add_argument("--shapes", default="", help="gx:gy,gx:gy,... (default: built-in list)")
    ap.add_argument("--erase", default="0,1", help="reconstruct: erased shard indices")
    ap.add_argument("--nt-only", action="store_true", help="only non-temporal configurations")
    ap.add_argument("--patterns", default="1",
                    help="reconstruct: comma list of RSE_OPT_JIT_PATTERNS values (decode-pattern "
                         "kernels; the run-time builds are waited for)")
    ap.add_argument("--jit-cse", type=int, default=-1,
                    help="RSE_OPT_JIT_CSE for run-time specialised GF(2^16) modules (-1: default)")
    ap.add_argument("--recon-mix", default="2",
                    help="comma list of RSE_OPT_RECON_MIX values (syndrome reconstruct mixing: "
                         "2 Horner, 1 doubling chains, 0 v_perm tables)")
    ap.add_argument("--wide-split", type=int, default=0,
                    help="RSE_OPT_WIDE_SPLIT: outputs per wave of one-module kernels (0: default)")
    ap.add_argument("--wide-lds", type=int, default=-1,
                    help="RSE_OPT_WIDE_LDS for wide-codec modules (-1: default)")
    ap.add_argument("--batch-parity", action="store_true",
                    help="batch: rebuild lost parity too (data_only=False)")
    ap.add_argument("--batch-cycle", type=int, default=0,
                    help="batch: stripes alternate between this many fixed patterns "
                         "(rotations of --erase) instead of random ones (0)")
    ap.add_argument("--hog-gib", type=int, default=0,
                    help="allocate this much device memory first (the bench holds 112 GiB)")
    ap.add_argument("--recon-depth", default="1",
                    help="comma list of RSE_OPT_RECON_DEPTH values (syndrome reconstruct: inputs "
                         "in flight per lane; compiled codecs)")
    ap.add_argument("--ab", default="", metavar="KEY=V1,V2",
                    help="one more interleaved dimension: RSE_OPT KEY set to each value")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="rse_set_option(KEY, VALUE) before the codec is created (repeatable)")
    args = ap.parse_args()
    hog = torch.empty(args.hog_gib << 30, dtype=torch.uint8, device="cuda") if args.hog_gib else None
    lib = R._lib.load()
    for kv in args.set:
        key, val = (int(x) for x in kv.split("="))
        if lib.rse_set_option(key, val) != 0:
            sys.exit(f"unknown option {key}")
    if args.wide_lds >= 0:
        lib.rse_set_option(14, args.wide_lds)
    if args.wide_split > 0:
        lib.rse_set_option(18, args.wide_split)
    lib.rse_set_option(9, 2)  # time run-time specialised kernels, not their build
    if args.jit_cse >= 0:
        lib.rse_set_option(13, args.jit_cse)
    k, p, S = args.k, args.p, args.stripes
    L = args.shard_kib * 1024 if args.shard_kib else args.shard_mib * MiB
    buf = torch.empty(S * (k + p) * L, dtype=torch.uint8, device="cuda")
    v = buf.view(S, k + p, L)
    if S * k <= 8192:
        for s in range(S):
            for i in range(k):
                fill_splitmix(v[s, i], 1, (s << 8) | i)
    else:  # many small stripes: one fill (timing does not depend on the bytes)
        fill_splitmix(buf, 1, 0)
    r = R.core.ReedSolomon(k, p, args.field)
    # codecs without compiled-in bit-sliced kernels: let the run-time
    # specialisation (rse_jit.cpp) finish before timing, printing while it
    # builds (a wide module is minutes of hiprtc on a slow host)
    import threading
    import time
    t0 = time.time()
    kind = []
    th = threading.Thread(target=lambda: kind.append(r.kernel_kind(wait=True)))
    th.start()  # the build (ctypes drops the GIL while it waits)
    while th.is_alive():
        th.join(10)
        if th.is_alive():
            print(f"  building ... {time.time() - t0:.0f} s", flush=True)
    print(f"kernels: {kind[0]} ({time.time() - t0:.1f} s)", flush=True)
    elems = L // (args.field // 8)
    erased = [int(x) for x in args.erase.split(",")]
    present = [i not in erased for i in range(k + p)]

    import numpy as np
    rng = np.random.default_rng(5)
    batch_present = np.ones((S, k + p), bool)
    for s_ in range(S):
        if args.batch_cycle:
            batch_present[s_, [(e + s_ % args.batch_cycle) % (k + p) for e in erased]] = False
        else:
            batch_present[s_, rng.choice(k + p, len(erased), replace=False)] = False

    def op():
        if args.op == "encode":
            r.encode_flat(buf, elems, S)
        elif args.op == "batch":
            r.reconstruct_batch(buf, elems, S, batch_present, data_only=not args.batch_parity)
        else:
            r.reconstruct_data_flat(buf, elems, S, present)

    if args.op == "batch":  # per stripe with missing data: k reads + the missing data written
        miss = (~batch_present[:, :k]).sum(axis=1)
        if args.batch_parity:  # k reads + every lost shard written
            lost = (~batch_present).sum(axis=1)
            nbytes = int((lost > 0).sum() * k + lost.sum()) * L
        else:
            nbytes = int((miss > 0).sum() * k + miss.sum()) * L
    else:
        nbytes = S * ((k + p) if args.op == "encode" else (k + len(erased))) * L
    shapes = [(512, 1), (1024, 1), (2048, 1), (4096, 1), (8, 0), (16, 0)]
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split(":")) for s in args.shapes.split(",")]
    bss = [int(x) for x in args.bitslice.split(",")]
    pats = [int(x) for x in args.patterns.split(",")] if args.op != "encode" else [1]
    nts = (0, 1) if not args.nt_only else (1,)
    mixes = [int(x) for x in args.recon_mix.split(",")]
    vlist = ([int(x) for x in args.variant_list.split(",")] if args.variant_list
             else list(range(args.variants)))
    depths = [int(x) for x in args.recon_depth.split(",")]
    ab_key, ab_vals = -1, [0]
    if args.ab:
        ab_key, vals = args.ab.split("=")
        ab_key, ab_vals = int(ab_key), [int(x) for x in vals.split(",")]
    configs = [(nt, gx, gy, var, bs, pat, mx, dp, ab) for ab in ab_vals for dp in depths
               for mx in mixes for pat in pats for bs in bss for var in vlist for nt in nts
               for gx, gy in shapes]
    res = {c: [] for c in configs}
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    op()
    torch.cuda.synchronize()
    for rnd in range(args.rounds):
        for c in configs:
            nt, gx, gy, var, bs, pat, mx, dp, ab = c
            if ab_key >= 0:
                lib.rse_set_option(ab_key, ab)
            lib.rse_set_option(27, dp)
            lib.rse_set_option(17, mx)
            lib.rse_set_option(11, pat)
            lib.rse_set_option(5, bs)
            lib.rse_set_option(1, nt)
            lib.rse_set_option(2, gx)
            lib.rse_set_option(3, gy)
            lib.rse_set_option(4, var)
            op()  # warm this shape
            a.record()
            op()
            b.record()
            torch.cuda.synchronize()
            res[c].append(nbytes / (a.elapsed_time(b) * 1e-3) / 1e9)
        print(f"round {rnd} done", flush=True)
    rows = sorted(((statistics.median(x), min(x), max(x), c) for c, x in res.items()), reverse=True)
    what = f" erased {erased}" if args.op == "reconstruct" else ""
    size = f"{args.shard_kib} KiB" if args.shard_kib else f"{args.shard_mib} MiB"
    print(f"{args.op} GF(2^{args.field}) {k}+{p} x {size}, {S} stripes{what}; GB/s (1e9)")
    for med, lo, hi, (nt, gx, gy, var, bs, pat, mx, dp, ab) in rows:
        abs_ = f"opt{ab_key}={ab} " if ab_key >= 0 else ""
        print(f"  {abs_}bitslice={bs} patterns={pat} mix={mx} depth={dp} variant={var} nt={nt} "
              f"grid_x={gx:<5} stripes_in_flight={gy:<3}  median {med:7.1f}  [{lo:7.1f}, {hi:7.1f}]")
    b = rows[0][3]
    from reed_solomon_erasure.core import last_kernel
    print(f"last kernel: {last_kernel()}")
    print(json.dumps({"best": {"bitslice": b[4], "variant": b[3], "nt": b[0], "grid_x": b[1],
                               "stripes_in_flight": b[2], "GBps": round(rows[0][0], 1)}}))


if __name__ == "__main__":
    main()
