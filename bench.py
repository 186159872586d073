#!/usr/bin/env python3
"""Headline benchmark: device-resident GF(2^8) encode of 10+4 x 16 MiB stripes.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): "device-resident encode MB/s (data+parity)" -- bytes of
data + parity shards per second, MB = 2^20 (the reference's unit,
CHANGELOG.md:59-63), over the whole job.  A *step* encodes one batch of
`--stripes` independent 10+4 x 16 MiB stripes per GPU (default 512, so N = 8
is BASELINE config 4's 4096 stripes) with ONE launch of the fused kernel
(rse_encode_flat).  Every stripe occupies its own HBM (no re-use of cached
bytes); stripes are split across ranks with no data-path collective
("scaling": "weak").  Inputs are resident in HBM before the timed region.

Also reported (not `value`): the kernel's HBM roofline fraction (HIP events on
the launch stream), the reference's own SIMD CPU path on this host (rank 0,
N = 1, bounded sample), reconstruct of 2 erased data shards, and the
pinned-host end-to-end rate (PCIe-inclusive).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-erasure_amd"))
sys.path.insert(0, ROOT)
# run-time specialised kernels (rse_jit.cpp): the code objects prebuilt on the
# host into the tree's cache (tools/prebuild_all.sh) load in milliseconds; a
# module whose source differs is rebuilt (the key hashes the whole source)
os.environ.setdefault("RSE_JIT_CACHE_DIR", os.path.join(ROOT, "jitcache"))

METRIC = "device-resident encode MB/s (data+parity), 10+4 × 16 MiB shards, 1/2/4/8 GPU"
MiB = 1 << 20
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
SEED = 0x5EED


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--data-shards", type=int, default=10)
    ap.add_argument("--parity-shards", type=int, default=4)
    ap.add_argument("--shard-mib", type=int, default=16)
    ap.add_argument("--stripes", type=int, default=512, help="stripes per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip reconstruct / e2e legs")
    ap.add_argument("--full-out", default=None,
                    help="where the full results (every leg) go; default "
                         "gpurun_out/bench_full_n<N>.json")
    return ap.parse_args(argv)


# ----------------------------------------------------------- distribution
def stripes_for_rank(total: int, rank: int, world: int) -> range:
    """Contiguous block of global stripe ids for `rank` (weak scaling: every
    rank gets the same count when world divides total)."""
    per, extra = divmod(total, world)
    start = rank * per + min(rank, extra)
    return range(start, start + per + (1 if rank < extra else 0))


def shard_id(global_stripe: int, i: int) -> int:
    """PRNG stream of shard i of a stripe; stripe 0 uses ids 0..k-1, which is
    what tests/golden's full-size digests were made from."""
    return (global_stripe << 8) | i


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def collective_timeout_s() -> float:
    return float(os.environ.get("RSE_BENCH_COLLECTIVE_TIMEOUT", "300"))


def init_collective(world: int, rank: int, local: int, rehearsal: bool) -> str:
    """Joins the process group and proves it with one all-reduce, or ends this
    rank with a non-zero status -- never a hang.  RCCL ("nccl") with one GPU
    per rank; gloo for the one-GPU rehearsal and on a host without a GPU.  The
    rendezvous and the first collective run under a deadline
    (RSE_BENCH_COLLECTIVE_TIMEOUT, default 300 s): a rank whose peers never
    arrive, or whose RCCL init or first all-reduce fails, exits with status 4
    (an error) or 5 (the deadline) after saying so, so the driver sees every
    rank fail instead of waiting forever."""
    import datetime
    import threading

    import torch
    import torch.distributed as dist
    backend = "gloo" if rehearsal or not torch.cuda.is_available() else "nccl"
    timeout = collective_timeout_s()

    def expire():
        print(f"rank {rank}/{world}: {backend} rendezvous or first all-reduce not done after "
              f"{timeout:.0f} s; exiting", file=sys.stderr, flush=True)
        os._exit(5)

    dog = threading.Timer(timeout, expire)
    dog.daemon = True
    dog.start()
    try:
        kw = {"timeout": datetime.timedelta(seconds=timeout)}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        t = torch.ones(1, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t)
        if int(t.item()) != world:
            raise RuntimeError(f"all-reduce of ones gave {t.item()}, not {world}")
    except Exception as e:  # noqa: BLE001 -- any failure ends the rank
        print(f"rank {rank}/{world}: {backend} init failed: {e!r}", file=sys.stderr, flush=True)
        os._exit(4)
    finally:
        dog.cancel()
    return backend


def device_identity(local: int) -> dict:
    """What this rank computes on: the GPU's PCI address and UUID (so a
    multi-GPU line shows N ranks on N distinct GPUs), or the host CPU."""
    import torch
    if not torch.cuda.is_available():
        return {"device": "cpu", "host": os.uname().nodename, "pid": os.getpid()}
    p = torch.cuda.get_device_properties(local)
    pci = None
    if hasattr(p, "pci_bus_id"):
        pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    uuid = getattr(p, "uuid", None)
    return {"device": f"cuda:{local}", "name": p.name, "pci": pci,
            "uuid": str(uuid) if uuid is not None else None}


def collective_info(world: int, local: int, rehearsal: bool) -> dict:
    """What the collective saw: backend, world size, and every rank's device
    (gathered), with whether they are all distinct GPUs."""
    ident = device_identity(local)
    if world == 1:
        return {"backend": None, "world_size": 1, "rank_devices": [ident],
                "distinct_gpus": ident["device"] != "cpu", "rehearsal": rehearsal}
    import torch.distributed as dist
    ids = [None] * world
    dist.all_gather_object(ids, ident)
    keys = {(i.get("pci"), i.get("uuid")) for i in ids if i["device"] != "cpu"}
    return {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
            "rank_devices": ids, "distinct_gpus": len(keys) == world, "rehearsal": rehearsal}


def reduce_timing(elapsed: float, world: int, device=None) -> float:
    """Job time = the slowest rank's timed region (all_reduce MAX).  The only
    collective in the benchmark; stripes never cross ranks."""
    if world == 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(steps: int, stripes_per_rank: int, world: int, stripe_bytes: int,
                   elapsed_max: float) -> float:
    """Whole-job MB/s (MB = 2^20): every rank's stripes over the slowest rank's time."""
    return steps * stripes_per_rank * world * stripe_bytes / elapsed_max / MiB


# ------------------------------------------------------------ CPU baseline
def host_cpu():
    """Host CPU description for the baseline legs (model, CPUs visible)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"model": model, "os_cpu_count": os.cpu_count(),
            "affinity_cpus": len(os.sched_getaffinity(0))}


def cpu_threads():
    """Threads for the all-cores legs: the CPUs this process may run on,
    capped at 16 -- the GPU box's CPU share for one GPU (the box reports the
    whole machine's CPUs through nproc / os.cpu_count)."""
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _cpu_workload(field, k, p, shard_bytes, rows_fn, seed):
    """One stripe's inputs, outputs and coding rows for a CPU leg."""
    import numpy as np
    from oracle import oracle as O
    data = [O.splitmix_bytes(seed, i, shard_bytes) for i in range(k)]
    out = [np.zeros(shard_bytes, np.uint8) for _ in range(p)]
    return data, out, np.ascontiguousarray(rows_fn(O))


def cpu_leg(name, field, k, n_out, shard_bytes, rows_fn, alg_bytes, seconds, threads):
    """The reference's CPU path on this host for one workload: GF(2^8) runs the
    reference's own simd_c kernel (compiled from the reference sources into
    oracle/_ref, driven in core.rs:481-509 loop order: "reference"); GF(2^16)
    runs the C restatement of the Field default loops the reference uses for it
    (lib.rs:99-118 over galois_16.rs:146-162: "port").  `threads` threads each
    code their own stripe (ctypes drops the GIL), for ~`seconds`; the rate
    counts `alg_bytes` per stripe (the metric's data+parity convention)."""
    import threading

    from oracle import oracle as O
    use_ref = field == 8 and O.ref_available()
    work = [_cpu_workload(field, k, n_out, shard_bytes, rows_fn, SEED + t) for t in range(threads)]
    if use_ref:
        ref = O.ref()

        def run(t):
            data, out, rows = work[t]
            ref.ref_gf8_code_some_slices(rows.ctypes.data_as(O._u8p), n_out, k, O._ptrs(data),
                                         O._ptrs(out), shard_bytes)
    else:
        def run(t):
            data, out, rows = work[t]
            O.code_some_slices(field, rows, data, out)
    run(0)  # warm
    counts = [0] * threads
    stop = threading.Event()

    def loop(t):
        while not stop.is_set():
            run(t)
            counts[t] += 1

    ths = [threading.Thread(target=loop, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(seconds)
    stop.set()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    n = sum(counts)
    kernel = ("reference simd_c kernel -O3 -march=haswell" if use_ref else
              "C restatement of the scalar Field loops")
    return {"value": round(n * alg_bytes / dt / MiB, 1), "unit": "MB/s", "cores": threads,
            "kind": "reference" if use_ref else "port",
            "sample": f"{name}: {n} stripes ({threads} thread(s), each its own stripe, "
                      f"{dt:.1f} s, {kernel})"}


def cpu_baselines(seconds, threads):
    """CPU legs beside the GPU numbers (rank 0, N = 1): the headline 10+4 x
    16 MiB encode at 1 thread (`cpu_baseline`) and on all cores, plus the other
    BASELINE configs: 10+2 x 1 MiB encode, 10+4 reconstruct of data shards 0,1
    (decode rows of the k valid shards, core.rs:850-861) and GF(2^16) 20+8 x
    4 MiB encode (BASELINE.md:37-45, benches/bandwidth.rs:58-86)."""
    from oracle import oracle as O

    def parity(field, k, p):
        return lambda O_: O_.Codec(field, k, p).matrix()[k:]

    def decode_0_1(O_):
        m = O_.Codec(8, 10, 4).matrix()
        valid = [i for i in range(14) if i not in (0, 1)][:10]
        return O_.matrix_invert(8, m[valid])[[0, 1]]

    L = 16 * MiB
    head = cpu_leg("10+4 x 16 MiB encode", 8, 10, 4, L, parity(8, 10, 4), 14 * L, seconds, 1)
    out = {"cpu_baseline": head}
    legs = {}
    specs = [("encode_10_4_16MiB", "10+4 x 16 MiB encode", 8, 10, 4, L, parity(8, 10, 4), 14 * L),
             ("encode_10_2_1MiB", "10+2 x 1 MiB encode", 8, 10, 2, MiB, parity(8, 10, 2), 12 * MiB),
             ("reconstruct_10_4_16MiB_0_1", "10+4 x 16 MiB reconstruct_data, shards 0,1 erased",
              8, 10, 2, L, decode_0_1, 12 * L),
             ("gf16_encode_20_8_4MiB", "GF(2^16) 20+8 x 4 MiB encode", 16, 20, 8, 4 * MiB,
              parity(16, 20, 8), 28 * 4 * MiB)]
    for key, name, field, k, n_out, sb, rows_fn, alg in specs:
        one = head if key == "encode_10_4_16MiB" else cpu_leg(name, field, k, n_out, sb, rows_fn,
                                                              alg, seconds / 2, 1)
        legs[key] = {"1_thread": one,
                     "all_cores": cpu_leg(name, field, k, n_out, sb, rows_fn, alg, seconds / 2,
                                          threads)}
    out["cpu_baseline_legs"] = legs
    out["cpu_host"] = dict(host_cpu(), threads_used_all_cores=threads,
                           cap="16 threads: the GPU box's CPU share for one GPU")
    return out


def load_traffic(workload, kernel_id):
    """Per-launch HBM bytes from the newest committed rocprofv3 PMC summary
    (profiles/*pmc_traffic*.json, written by tools/pmc_traffic.py: FETCH_SIZE
    x2 gfx950 correction + WRITE_SIZE) -- only if it was measured on this
    workload AND on the kernel that ran here (rse_last_kernel); else None."""
    best = None
    lib_sha = library_info().get("sha256")
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if d.get("workload") == workload and d.get("kernel_id") == kernel_id:
            # a measurement of this very library wins over any other
            if best is None or d.get("library_sha256") == lib_sha or \
                    best.get("library_sha256") != lib_sha:
                best = dict(d, file=os.path.relpath(path, ROOT))
    return best


def library_info():
    """What ran: librse_hip.so's SHA-256 and the source commit its Makefile
    stamped (BUILD_INFO.json next to it; the GPU box has no .git)."""
    d = os.path.join(ROOT, "reed-solomon-erasure_amd", "reed_solomon_erasure")
    out = {"sha256": hashlib.sha256(open(os.path.join(d, "librse_hip.so"), "rb").read()).hexdigest()}
    try:
        info = json.load(open(os.path.join(d, "BUILD_INFO.json")))
        out.update(source_commit=info.get("source_commit"),
                   uncommitted_source_files=info.get("uncommitted_source_files"),
                   build_info_matches=info.get("library_sha256") == out["sha256"])
    except (OSError, ValueError):
        out["source_commit"] = None
    return out


# ------------------------------------------------------ the printed line
# The driver reads the LAST stdout line and keeps only the tail of stdout
# (~8 KB), so that line is a compact summary (< LINE_LIMIT bytes): the
# contract keys, the roofline, the CPU baseline and one number per extra leg.
# Every leg in full goes to a JSON file named on the line (`full_results`).
LINE_LIMIT = 4000
# booleans in the full results that are descriptions, not correctness flags
NOT_FLAGS = {"higher_is_better", "distinct_gpus", "rehearsal", "build_info_matches",
             "pattern_kernel"}


def _get(d, *path):
    for key in path:
        if not isinstance(d, dict) or key not in d:
            return None
        d = d[key]
    return d


def correctness_flags(d, prefix=""):
    """(path, value) of every boolean correctness flag in the full results:
    rebuilt-shard checks, parity-vs-digest checks, verify verdicts."""
    out = []
    if isinstance(d, dict):
        for key, x in d.items():
            path = f"{prefix}.{key}" if prefix else key
            if isinstance(x, bool):
                if key not in NOT_FLAGS:
                    out.append((path, x))
            else:
                out += correctness_flags(x, path)
    elif isinstance(d, list):
        for i, x in enumerate(d):
            out += correctness_flags(x, f"{prefix}[{i}]")
    return out


def leg_summary(full):
    """One number per extra leg (algorithmic GB/s unless the key says
    otherwise), read from the full results; legs that did not run are left out."""
    oc = full.get("other_configs") or {}
    s = {
        "reconstruct_10_4_lost_0_1_GBps": _get(full, "reconstruct", "algorithmic_GB_per_s"),
        "reconstruct_10_4_cached_pattern_GBps": _get(full, "reconstruct_cached_pattern",
                                                     "algorithmic_GB_per_s"),
        "verify_10_4_c_abi_us_per_call": _get(full, "verify", "c_abi", "us_per_call"),
        "verify_flat_10_4_GBps": _get(full, "verify_flat", "algorithmic_GB_per_s"),
        "e2e_pinned_host_flat_MBps": _get(full, "end_to_end_pinned_host_flat", "MB_per_s"),
        "e2e_pinned_host_flat_vs_raw_duplex": _get(full, "end_to_end_pinned_host_flat",
                                                   "vs_raw_duplex"),
        "e2e_pinned_host_reconstruct_MBps": _get(full, "end_to_end_pinned_host_reconstruct",
                                                 "MB_per_s"),
        "e2e_host_all_ranks_MBps": _get(full, "end_to_end_host_all_ranks", "MB_per_s_all_ranks"),
        "gf8_10_2_1MiB_encode_GBps": _get(oc, "gf8_10_2", "encode_GB_per_s"),
        "gf16_20_8_4MiB_encode_GBps": _get(oc, "gf16_20_8", "encode_GB_per_s"),
        "gf16_20_8_4MiB_lost8_GBps": _get(oc, "gf16_20_8", "reconstruct_8_erased_syndrome_GB_per_s"),
        "gf8_50_20_1MiB_encode_GBps": _get(oc, "gf8_50_20", "encode_GB_per_s"),
        "gf16_40_12_1MiB_encode_GBps": _get(oc, "gf16_40_12", "encode_GB_per_s"),
        "gf16_100_30_1MiB_encode_GBps": _get(oc, "gf16_100_30", "encode_GB_per_s"),
        "gf16_proper_encode_GBps": _get(full, "gf16_proper", "encode_GB_per_s"),
        "gf16_proper_reconstruct_GBps": _get(full, "gf16_proper", "reconstruct_GB_per_s"),
        "batch_4k_gf16_20_8_lost4_GBps": _get(full, "reconstruct_batch_4k", "GB_per_s"),
        "batch_4k_data_only_GBps": _get(full, "reconstruct_batch_4k", "data_only_GB_per_s"),
        "cpu_all_cores_10_4_MBps": _get(full, "cpu_baseline_legs", "encode_10_4_16MiB",
                                        "all_cores", "value"),
        "crossover_10_4_device_call_beats_cpu_from_bytes": _get(
            full, "reference_bench_matrix", "crossover_10_4",
            "gpu_call_device_beats_cpu_from_shard_bytes"),
    }
    s = {key: x for key, x in s.items() if x is not None}
    ents = _get(full, "reference_bench_matrix", "entries") or []
    enc = {e["shape"].replace(" x ", "x").replace(" KiB", "K"): _get(e, "gpu_flat", "GB_per_s")
           for e in ents if e.get("op") == "encode"}
    if enc:
        s["ref_bench_encode_GBps"] = enc
    for key, col in (("call_10_4_1KiB_encode_device_us", "gpu_call_device_us"),
                     ("call_10_4_1KiB_encode_now_us", "gpu_call_now_us"),
                     ("cpu_10_4_1KiB_encode_call_us", "cpu_reference_call_us")):
        one = [e.get(col) for e in ents
               if e.get("shape") == "10+4 x 1 KiB" and e.get("op") == "encode"]
        if one and one[0] is not None:
            s[key] = one[0]
    now_win = _get(full, "reference_bench_matrix", "crossover_10_4",
                   "gpu_call_now_beats_cpu_from_shard_bytes")
    if now_win is not None:
        s["crossover_10_4_now_call_beats_cpu_from_bytes"] = now_win
    return s


def compact_line(line, full, full_path):
    """The printed line: `line`'s contract keys, roofline and cpu_baseline
    (trimmed), the leg summary, every correctness flag folded into one, and
    where the full results are; shortened until it fits LINE_LIMIT."""
    c = {key: line[key] for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                    "ms_per_step", "higher_is_better", "scaling",
                                    "vs_baseline", "dtype", "data")}
    c["config"] = dict(line["config"])  # incl. every rank's verdict (N ints)
    coll = line.get("collective") or {}
    c["collective"] = {key: coll.get(key) for key in ("backend", "world_size", "distinct_gpus",
                                                      "rehearsal")}
    roof = {key: x for key, x in line["roofline"].items() if key != "traffic_source"}
    src = line["roofline"].get("traffic_source")
    roof["traffic_file"] = src.get("file") if src else None
    c["roofline"] = roof
    c["cpu_baseline"] = line.get("cpu_baseline")
    lib = line.get("library") or {}
    c["library"] = {"sha256_16": (lib.get("sha256") or "")[:16],
                    "source_commit": lib.get("source_commit")}
    flags = correctness_flags(full)
    bad = [path for path, ok in flags if not ok]
    c["checks"] = {"flags": len(flags), "all_true": not bad, "false": bad[:4]}
    c["legs"] = leg_summary(full)
    c["full_results"] = full_path
    # shorten (least important first) until the line fits
    for cut in ("ref_bench_encode_GBps", "legs", "sample", "false"):
        if len(json.dumps(c)) < LINE_LIMIT:
            break
        if cut == "ref_bench_encode_GBps":
            c["legs"].pop(cut, None)
        elif cut == "legs":
            c.pop("legs")
        elif cut == "sample" and c.get("cpu_baseline"):
            c["cpu_baseline"] = dict(c["cpu_baseline"], sample=c["cpu_baseline"]["sample"][:80])
        elif cut == "false":
            c["checks"]["false"] = bad[:1]
    return c


def emit_results(line, cpu, extras, path):
    """Writes the full results (line + CPU legs + every extra leg) to `path`
    and prints the compact line as the last stdout line."""
    full = dict(line)
    for key in ("cpu_baseline_legs", "cpu_host"):
        if key in cpu:
            full[key] = cpu[key]
    full.update(extras)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(full, f, indent=1)
    shown = os.path.relpath(os.path.abspath(path), ROOT)
    print(f"full results (every leg): {shown}", file=sys.stderr, flush=True)
    out = compact_line(line, full, shown)
    print(json.dumps(out), flush=True)
    return out


# ----------------------------------------------------------------- main
def golden_stripes():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["generated"]
    return g["gf8_10_4_stripe_parity"]


def check_stripes(v, mine, resident, k, p):
    """This rank's verdict on its own output: the parity of its first and last
    resident stripe against the reference digests (tests/golden).  1 = every
    checked stripe matches, 0 = a mismatch, -1 = no digest for these stripes."""
    gold = golden_stripes()
    checked, ok = [], True
    for s in sorted({0, resident - 1}):
        g = mine.start + s
        if str(g) not in gold:
            continue
        got = [hashlib.sha256(v[s, k + i].cpu().numpy().tobytes()).hexdigest() for i in range(p)]
        checked.append(g)
        ok = ok and got == gold[str(g)]
    return (1 if ok else 0) if checked else -1, checked


def gather(values, world, rank, device):
    """Every rank's value (float64), in rank order, on every rank."""
    import torch
    import torch.distributed as dist
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[rank] = float(values)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def host_leg(r, v, k, p, L, stream, world, rank, coll_dev):
    """Host-memory encode on every rank at once (multi-GPU host bandwidth,
    SURVEY 8f): each rank streams 8 of its stripes from pinned host memory
    through its GPU; the job rate is all ranks' bytes over the slowest rank."""
    import torch
    import torch.distributed as dist
    ns = min(8, v.shape[0])
    hflat = v[:ns].reshape(-1).cpu().pin_memory()
    warm_calls(lambda: r.encode_host_flat(hflat, L, ns))  # first use of the buffer, the
    reps = 10                                               # pipeline's resources, steady state
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        r.encode_host_flat(hflat, L, ns)
    dt = (time.perf_counter() - t0) / reps
    ok = torch.equal(hflat.view(ns, k + p, L)[:, k:], v[:ns, k:].cpu())
    per = gather(dt, world, rank, coll_dev)
    oks = gather(1.0 if ok else 0.0, world, rank, coll_dev)
    return {"what": f"rse_encode_host_flat on every rank at once, {ns} stripes each from pinned "
                    "host memory (H2D data, kernel, D2H parity)",
            "ranks": world, "MB_per_s_all_ranks": round(world * ns * (k + p) * L / max(per) / MiB, 1),
            "GB_per_s_pcie_h2d_all_ranks": round(world * ns * k * L / max(per) / 1e9, 1),
            "parity_matches_device_all_ranks": all(x == 1.0 for x in oks)}


def main(argv=None):
    args = parse(argv)
    world, rank, local = init_dist(args)
    import torch
    import torch.distributed as dist

    # RSE_BENCH_REHEARSAL=1: every rank on cuda:0 over gloo, so the N > 1 path
    # can be exercised on a one-GPU box (tests/test_gpu_parity.py); the
    # driver's multi-GPU runs use one GPU per rank over RCCL ("nccl")
    rehearsal = os.environ.get("RSE_BENCH_REHEARSAL") == "1"
    if rehearsal:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        init_collective(world, rank, local, rehearsal)
    coll_dev = None if rehearsal else "cuda"
    coll = collective_info(world, local, rehearsal)
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix, last_kernel

    k, p = args.data_shards, args.parity_shards
    L = args.shard_mib * MiB
    stripe_bytes = (k + p) * L
    total_stripes = args.stripes * world
    mine = stripes_for_rank(total_stripes, rank, world)
    n_local = len(mine)
    free, _ = torch.cuda.mem_get_info()
    # one HBM region per stripe when it fits (it does on 288 GB); otherwise a
    # pool far larger than the 256 MiB Infinity Cache, cycled.
    share = world if rehearsal else 1  # rehearsal ranks share one GPU
    pool = min(n_local, max(8, int(0.8 * free / share) // stripe_bytes))
    buf = torch.empty(pool * stripe_bytes, dtype=torch.uint8, device="cuda")
    v = buf.view(pool, k + p, L)
    for s in range(pool):
        for i in range(k):
            fill_splitmix(v[s, i], SEED, shard_id(mine.start + s, i))
    torch.cuda.synchronize()
    r = R.galois_8.ReedSolomon(k, p)
    stream = torch.cuda.current_stream()

    def step():
        done = 0
        while done < n_local:
            cnt = min(pool, n_local - done)
            r.encode_flat(buf, L, cnt)
            done += cnt

    lib = R._lib.load()
    n_bs = lib.rse_get_option(6)  # RSE_OPT_BITSLICE_LAUNCHES
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    kernel = "bitslice" if lib.rse_get_option(6) > n_bs else "table"
    kernel_id = last_kernel()
    # correctness gate, every rank on its own stripes, verdicts combined
    verdict, checked = (check_stripes(v, mine, pool, k, p) if (k, p, L) == (10, 4, 16 * MiB)
                        else (-1, []))
    verdicts = gather(verdict, world, rank, coll_dev)
    if any(x == 0 for x in verdicts):
        if rank == 0:
            print(f"PARITY MISMATCH vs reference digests, per-rank verdicts {verdicts}",
                  file=sys.stderr)
        if world > 1:
            dist.destroy_process_group()
        sys.exit(3)  # every rank together: nobody is left waiting in a collective
    check = all(x == 1 for x in verdicts) if any(x == 1 for x in verdicts) else None

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    kern_ms = sorted(a.elapsed_time(b) for a, b in ev)
    elapsed = reduce_timing(elapsed, world, device=coll_dev)
    value = job_throughput(args.steps, n_local, world, stripe_bytes, elapsed)
    launches = -(-n_local // pool)
    mean_ms = sum(kern_ms) / len(kern_ms) / launches
    rank_ms = gather(mean_ms, world, rank, coll_dev)

    extras = {}
    if not args.no_extras:
        extras["end_to_end_host_all_ranks"] = host_leg(r, v, k, p, L, stream, world, rank,
                                                       coll_dev)
    if rank == 0 and not args.no_extras and world == 1:  # single-GPU legs
        if (k, p, L) == (10, 4, 16 * MiB):
            # every other leg gets HBM of its own, allocated after the
            # headline's 112 GiB is freed (not the memory left around it)
            del v, buf, step
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            extras.update(fresh_extra_legs(r, k, p, L, min(pool, 256), stream))
            extras["other_configs"] = other_configs(stream)
            extras["gf16_proper"] = gf16_proper_leg(stream)
            extras["reconstruct_batch_4k"] = batch_leg(stream)
            extras["reference_bench_matrix"] = reference_bench_matrix(stream)
        else:
            extras.update(extra_legs(r, v, k, p, L, min(pool, 256), stream))
        host_agreement(extras)

    if rank == 0:
        per_launch_bytes = n_local * stripe_bytes / launches
        achieved = per_launch_bytes / (mean_ms * 1e-3) / 1e9
        workload = f"gf8 {k}+{p} x {args.shard_mib} MiB encode, {pool} stripes/launch"
        tr = load_traffic(workload, kernel_id)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": (tr["hbm_bytes_per_launch"] if tr else None),
                "traffic_source": ({"file": tr["file"], "kernel_id": tr["kernel_id"],
                                    "commit": tr.get("commit")} if tr else None),
                "kernel": kernel, "kernel_id": kernel_id,
                "kernel_ms_per_launch": round(mean_ms, 4),
                "kernel_ms_per_launch_per_rank": [round(x, 4) for x in rank_ms],
                "kernel_ms_per_launch_min_max": [round(min(rank_ms), 4), round(max(rank_ms), 4)],
                "algorithmic_bytes_per_launch": int(per_launch_bytes)}
        cpu = {}
        if world == 1 and not args.no_cpu:
            cpu = cpu_baselines(args.cpu_seconds, cpu_threads())
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "MB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (splitmix64 shards generated in HBM)",
            "config": {"workload": workload, "field": "GF(2^8)", "data_shards": k,
                       "parity_shards": p, "shard_bytes": L,
                       "stripes_per_gpu_per_step": n_local, "global_stripes_per_step":
                       total_stripes, "parallelism": f"stripes split over {world} GPU(s), no collective",
                       "parity_check_vs_reference": check,
                       "parity_check_per_rank": [int(x) for x in verdicts],
                       "parity_checked_stripes_rank0": checked},
            "collective": coll,
            "roofline": roof, "cpu_baseline": cpu.get("cpu_baseline"),
        }
        line["library"] = library_info()
        emit_results(line, cpu, extras, args.full_out or os.path.join(
            ROOT, "gpurun_out", f"bench_full_n{world}.json"))
    if world > 1:
        dist.destroy_process_group()


def warm_calls(fn, seconds=0.5):
    """Untimed calls for `seconds` before a host-memory leg's timed ones: the
    pinned-host pipeline's copies run at about half rate for up to a second
    after the bench's large device allocations and frees, then settle
    (profiles/r06/s9/probe.log); the legs report the steady state (and the
    flat leg its first call on its own)."""
    t0 = time.perf_counter()
    fn()
    while time.perf_counter() - t0 < seconds:
        fn()


def host_agreement(extras):
    """The two pinned-host rse_encode_host_flat legs (host_leg, made first,
    and extra_legs', made after every other leg) time the same call on the
    same 8 stripes: flag whether they agree within 10 % (they
    read 76.1 and 41.6 GB/s in one process), and report the flat leg against
    plain duplex copies of the same bytes."""
    a = _get(extras, "end_to_end_host_all_ranks", "MB_per_s_all_ranks")
    flat = extras.get("end_to_end_pinned_host_flat")
    if a is None or not flat or _get(extras, "end_to_end_host_all_ranks", "ranks") != 1:
        return
    b = flat["MB_per_s"]
    flat["vs_host_leg"] = round(b / a, 3)
    flat["host_flat_legs_agree_within_10pct"] = abs(b - a) <= 0.1 * max(a, b)
    raw = flat.get("raw_pinned_duplex_MB_per_s")
    if raw:  # a performance ratio, not a correctness flag
        flat["vs_raw_duplex"] = round(b / raw, 3)


def _sync():
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def timed_ms(fn, reps, stream=None):
    """Mean milliseconds per call of `reps` back-to-back fn() calls, by HIP
    events on the launch stream (None: the current stream)."""
    import torch
    _sync()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def timed_gbps(fn, nbytes, stream, reps=5, prepare=None, warm_s=0.0):
    """Algorithmic GB/s (1e9) of fn() over `reps` back-to-back calls (HIP
    events on the launch stream) after one untimed call (or untimed calls for
    `warm_s` seconds: the VALU-bound wide kernels run at a power-managed clock
    that settles over tens of milliseconds).  `prepare` runs between the
    untimed calls and the timed ones (outside the timed region): the
    reconstruct legs poison the shards the timed calls must rebuild."""
    fn()
    if warm_s > 0:
        _sync()
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < warm_s:
            fn()
            _sync()
    if prepare is not None:
        prepare()
    return round(nbytes / (timed_ms(fn, reps, stream) * 1e-3) / 1e9, 1)


# --------------------------------------------- correctness of the extra legs
# The driver-run bench line is the hardware record, so every reconstruct and
# verify leg on it proves its own output: erased shards are overwritten with a
# poison byte before the timed calls, and every rebuilt shard is compared with
# its synthetic bytes afterwards; the verify legs see corrupted stripes that
# must come back false.  A kernel that writes nothing fails these checks.
POISON = 0xA5


def poison(v, n_stripes, shards):
    """Overwrite shards `shards` of the first `n_stripes` stripes of the
    stripe view v[stripe, shard, byte] with POISON."""
    for i in shards:
        v[:n_stripes, i].fill_(POISON)


def rebuilt_ok(v, n_stripes, shards, stripe_ids, fill):
    """True iff shard i of stripe s holds the synthetic bytes of (SEED,
    shard_id(stripe_ids[s], i)) for every s < n_stripes and i in `shards`.
    `fill(t, seed, shard)` regenerates them (the device fill kernel, a
    separate kernel from the one under test) into a scratch shard; with
    `fill` a tensor instead, the shards are compared with that saved copy
    (v[:n_stripes, shards] taken before they were poisoned)."""
    import torch
    if isinstance(fill, torch.Tensor):
        return bool(torch.equal(v[:n_stripes, list(shards)], fill))
    tmp = torch.empty(v.shape[-1], dtype=torch.uint8, device=v.device)
    for s in range(n_stripes):
        for i in shards:
            fill(tmp, SEED, shard_id(stripe_ids[s], i))
            if not torch.equal(tmp, v[s, i]):
                return False
    return True


def digests_ok(v, shards, want):
    """Stripe 0's shards `shards` against SHA-256 digests `want` (tests/golden)."""
    got = [hashlib.sha256(v[0, i].cpu().numpy().tobytes()).hexdigest() for i in shards]
    return got == list(want)


def reconstruct_leg(r, v, k, erased, elems, n_stripes, stream, fill, stripe_ids,
                    want_digests=None, reps=5, warm_s=0.0):
    """reconstruct_data_flat of `n_stripes` stripes of the view v with data
    shards `erased` lost (one shared pattern, core.rs:680-695), timed; the
    erased shards are poisoned before the timed calls and checked after them:
    every rebuilt shard of every stripe against its synthetic bytes, and
    stripe 0's against the fixture digests when given."""
    T = v.shape[1]
    flat = v[:n_stripes].reshape(-1)
    present = [i not in erased for i in range(T)]
    if fill is None:  # no generator for these bytes: keep a copy to compare with
        fill = v[:n_stripes, list(erased)].clone()
    gbps = timed_gbps(lambda: r.reconstruct_data_flat(flat, elems, n_stripes, present),
                      n_stripes * (k + len(erased)) * v.shape[-1], stream, reps=reps,
                      prepare=lambda: poison(v, n_stripes, erased), warm_s=warm_s)
    out = {"GB_per_s": gbps,
           "rebuilt_ok_all_stripes": rebuilt_ok(v, n_stripes, erased, stripe_ids, fill)}
    if want_digests is not None:
        out["rebuilt_stripe0_vs_digests"] = digests_ok(v, erased, want_digests)
    return out


def verify_leg(r, v, k, p, L, n_stripes, reps=5):
    """verify (one synchronous call per stripe, core.rs:637-651) and
    verify_flat (one pass) over `n_stripes` stripes, two of them corrupted --
    one byte of a parity shard in one, of a data shard in another -- which
    must come back false while every other stripe comes back true."""
    bad = {n_stripes // 3: k + p - 1, (2 * n_stripes) // 3: k // 2}  # stripe -> shard
    offs = {s: (L // 2 + 4097 * s) % L for s in bad}
    for s, i in bad.items():
        v[s, i, offs[s]] ^= 0x5A
    want = [s not in bad for s in range(n_stripes)]
    flat = v[:n_stripes].reshape(-1)
    shards = [[v[s_, i] for i in range(k + p)] for s_ in range(n_stripes)]
    try:
        _sync()
        t0 = time.perf_counter()
        got = [r.verify(sh) for sh in shards]
        dt = time.perf_counter() - t0
        capi = verify_capi(r, shards, L, want)
        flat_first = [bool(x) for x in r.verify_flat(flat, L, n_stripes)]
        res = {}

        def run():
            res["oks"] = r.verify_flat(flat, L, n_stripes)
        ms = timed_ms(run, reps)
        flat_got = [bool(x) for x in res["oks"]]
    finally:
        for s, i in bad.items():
            v[s, i, offs[s]] ^= 0x5A
    nbytes = n_stripes * (k + p) * L
    corrupted = sorted(bad)
    per_call = {"what": f"verify, {n_stripes} stripes, one call each (synchronous, through the "
                        f"Python mirror); stripes {corrupted} corrupted",
                "corrupted_stripes": corrupted, "verdicts_ok": got == want,
                "algorithmic_GB_per_s": round(nbytes / dt / 1e9, 1)}
    if capi is not None:
        per_call["c_abi"] = {
            "what": "the same calls through the C ABI with prebuilt pointer arrays (what the "
                    "reference's Rust caller binding rse_verify pays; ctypes adds ~1 us)",
            "verdicts_ok": capi[1], "us_per_call": round(capi[0] * 1e6, 2),
            "algorithmic_GB_per_s": round(nbytes / n_stripes / capi[0] / 1e9, 1)}
    return (per_call,
            {"what": f"verify_flat, {n_stripes} stripes in one pass (reads k+p shards); stripes "
                     f"{corrupted} corrupted", "corrupted_stripes": corrupted,
             "verdicts_ok": flat_got == want and flat_first == want,
             "algorithmic_GB_per_s": round(nbytes / (ms * 1e-3) / 1e9, 1)})


def verify_capi(r, shards, L, want, reps=3):
    """Seconds per synchronous rse_verify call over the stripes `shards`
    (best of `reps` passes) and whether every verdict equals `want`; None
    without a device codec (the CPU tests' stand-ins)."""
    import ctypes
    import torch
    if not hasattr(r, "_h") or not torch.cuda.is_available():
        return None
    lib = R_lib()
    sh = torch.cuda.current_stream().cuda_stream
    T = len(shards[0])
    lens = (ctypes.c_size_t * T)(*([L] * T))
    arrs = [(ctypes.c_void_p * T)(*[t.data_ptr() for t in s]) for s in shards]
    ok = ctypes.c_int(0)
    best, good = None, True
    for _ in range(reps):
        got = []
        t0 = time.perf_counter()
        for a in arrs:
            _ck(lib.rse_verify(r._h, a, lens, T, ctypes.byref(ok), sh))
            got.append(bool(ok.value))
        dt = (time.perf_counter() - t0) / len(arrs)
        good = good and got == want
        best = dt if best is None else min(best, dt)
    return best, good


def other_configs(stream):
    """BASELINE.json configs[1] (galois_8 10+2 x 1 MiB) and configs[4]
    (galois_16 20+8 x 4 MiB encode/reconstruct) on this GPU, each with stripe
    0's parity checked against the digests of tests/golden (GF(2^8): the
    reference's own kernel; GF(2^16): the restatement), and every reconstruct
    leg's rebuilt shards checked after poisoning."""
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix
    lib = R_lib()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["generated"]
    out = {}
    for field, k, p, nbytes, stripes in ((8, 10, 2, MiB, 2048), (16, 20, 8, 4 * MiB, 256)):
        T = k + p
        buf = torch.empty(stripes * T * nbytes, dtype=torch.uint8, device="cuda")
        v = buf.view(stripes, T, nbytes)
        for s_ in range(stripes):
            for i in range(k):
                fill_splitmix(v[s_, i], SEED, shard_id(s_, i))
        r = R.core.ReedSolomon(k, p, field)
        elems = nbytes // (field // 8)
        enc = timed_gbps(lambda: r.encode_flat(buf, elems, stripes), stripes * T * nbytes, stream,
                         reps=10, warm_s=0.1)
        fs = g["full_size"][f"gf{field}_{k}_{p}_{nbytes}"]
        d = {"workload": f"gf{field} {k}+{p} x {nbytes // MiB} MiB, {stripes} stripes/launch",
             "encode_GB_per_s": enc, "encode_MB_per_s": round(enc * 1e9 / MiB, 1),
             "encode_roofline_frac": round(enc / HBM_PEAK_GBPS, 4)}
        d["parity_check_vs_reference" if field == 8 else "parity_check_vs_restatement"] = \
            digests_ok(v, range(k, T), fs["parity_sha256"])
        if field == 16:
            # first uses of an erasure pattern (syndrome kernels, no decode-
            # pattern kernel): 8 data shards lost (bit-sliced mixing) and 4;
            # timed as the wide legs: 0.25 s of untimed calls, then 10
            d["reconstruct_timing"] = "0.25 s of untimed calls, then 10 back to back (HIP events)"
            ids = list(range(stripes))
            for lost in (8, 4):
                erased = list(range(lost))
                lib.rse_set_option(11, 0)
                try:
                    leg = reconstruct_leg(r, v, k, erased, elems, stripes, stream, fill_splitmix,
                                          ids, fs["data_sha256"][:lost], reps=10, warm_s=0.25)
                finally:
                    lib.rse_set_option(11, 1)
                d[f"reconstruct_{lost}_erased_syndrome_GB_per_s"] = leg["GB_per_s"]
                d[f"reconstruct_{lost}_erased_syndrome_rebuilt_ok"] = (
                    leg["rebuilt_ok_all_stripes"] and leg["rebuilt_stripe0_vs_digests"])
            old = lib.rse_get_option(9)
            lib.rse_set_option(9, 2)
            try:
                leg = reconstruct_leg(r, v, k, [0, 1, 2, 3], elems, stripes, stream,
                                      fill_splitmix, ids, fs["data_sha256"][:4], reps=10,
                                      warm_s=0.25)
            finally:
                lib.rse_set_option(9, old)
            d["reconstruct_4_erased_cached_pattern_GB_per_s"] = leg["GB_per_s"]
            d["reconstruct_4_erased_cached_pattern_rebuilt_ok"] = (
                leg["rebuilt_ok_all_stripes"] and leg["rebuilt_stripe0_vs_digests"])
        out[f"gf{field}_{k}_{p}"] = d
        del buf, v
        torch.cuda.empty_cache()
    out["gf8_50_20"] = wide_config(stream, g, 8, 50, 20)
    out["gf16_40_12"] = wide_config(stream, g, 16, 40, 12)
    # round 3's GF(2^16) 100+30 target (>= 4.0 TB/s); a subfield codec, so the
    # GF(2^8) wide module (half chunks)
    out["gf16_100_30"] = wide_config(stream, g, 16, 100, 30)
    return out


# k, p, shard bytes, stripes per launch.  1000+24: galois_16.rs's reason to
# exist (far past 256 shards); it runs as a chain of 8 wide modules over
# blocks of 125 data shards (rse_jit.cpp "wide modules over input blocks"),
# prebuilt into jitcache/ by tools/prebuild_all.sh.  512 stripes (32 GiB) per
# launch: the chain ran 2.32 TB/s there against 2.15 at 128
# (profiles/r05/s19/).  (A one-module GF(2^16) 256+16 did not finish
# compiling in 25 minutes of hiprtc on the build host.)
GF16_PROPER = (1000, 24, 64 << 10, 512)
# how long a leg waits for its run-time modules before it reports itself
# skipped (RSE_BENCH_JIT_BUDGET_S): with the tree's jitcache/ they load in
# milliseconds; a cold build of the largest would hold the bench for minutes
JIT_BUDGET_S = float(os.environ.get("RSE_BENCH_JIT_BUDGET_S", "180"))


def kernels_within(r, budget_s):
    """r.kernel_kind(wait=True) if it returns within budget_s, else None (the
    build goes on in the background; its helpers stop at exit)."""
    import threading
    out = []
    th = threading.Thread(target=lambda: out.append(r.kernel_kind(wait=True)), daemon=True)
    th.start()
    th.join(budget_s)
    return out[0] if out else None


def gf16_proper_leg(stream, k=GF16_PROPER[0], p=GF16_PROPER[1], nbytes=GF16_PROPER[2],
                    stripes=GF16_PROPER[3], check=4096, lost=4):
    """GF(2^16) proper: a codec past GF(2^8)'s 256 shards (galois_16.rs:20-21,
    ORDER = 65536), whose Vandermonde points leave the subfield, so it codes
    on the GF(2^16) kernels (16 x 16 bit matrices), not the GF(2^8) ones.
    Encode of `stripes` stripes per launch (the run-time specialised block
    modules, waited for), stripe 0's parity checked against the oracle
    on its first and last `check` bytes (column j of the parity depends only
    on column j of the data); then reconstruct_data_flat with data shards
    0..lost-1 erased (first use: no decode-pattern kernel), every rebuilt
    shard of every stripe checked against a copy taken before they were
    poisoned."""
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix, last_kernel
    T = k + p
    assert T > 256, "GF(2^16) proper: past the subfield's 256 shards"
    buf = torch.empty(stripes * T * nbytes, dtype=torch.uint8, device="cuda")
    v = buf.view(stripes, T, nbytes)
    fill_splitmix(buf, SEED, 0x16 << 40)  # one stream over everything; encode overwrites parity
    r = R.core.ReedSolomon(k, p, 16)
    t0 = time.perf_counter()
    kind = kernels_within(r, JIT_BUDGET_S)
    build_s = time.perf_counter() - t0
    if kind is None:  # cold JIT cache: do not hold the bench for the build
        del buf, v
        torch.cuda.empty_cache()
        return {"skipped": f"the {k}+{p} chain modules were not built within {JIT_BUDGET_S:.0f} s "
                           "(a cold JIT cache: ~20-45 min of hiprtc; tools/prebuild_all.sh "
                           "builds them into jitcache/)"}
    elems = nbytes // 2
    enc = timed_gbps(lambda: r.encode_flat(buf, elems, stripes), stripes * T * nbytes, stream,
                     reps=10, warm_s=0.25)
    d = {"workload": f"gf16 {k}+{p} x {nbytes >> 10} KiB, {stripes} stripes/launch "
                     f"({T} shards: past GF(2^8)'s 256, no subfield)",
         "kernels": kind, "kernel": last_kernel(), "build_seconds": round(build_s, 1),
         "timing": "0.25 s of untimed launches, then 10 back to back (HIP events)",
         "encode_GB_per_s": enc, "encode_MB_per_s": round(enc * 1e9 / MiB, 1),
         "encode_roofline_frac": round(enc / HBM_PEAK_GBPS, 4)}
    d["parity_check_vs_oracle_stripe0_head_tail"] = head_tail_ok(v, 16, k, p, check)
    lib = R_lib()
    lib.rse_set_option(11, 0)  # a first use of the pattern
    try:
        leg = reconstruct_leg(r, v, k, list(range(lost)), elems, stripes, stream, None, None,
                              reps=10, warm_s=0.25)
    finally:
        lib.rse_set_option(11, 1)
    d[f"reconstruct_{lost}_lost_kernel"] = last_kernel()
    d["reconstruct_GB_per_s"] = leg["GB_per_s"]
    d["reconstruct_rebuilt_ok_all_stripes"] = leg["rebuilt_ok_all_stripes"]
    del buf, v
    torch.cuda.empty_cache()
    return d


def batch_leg(stream, stripes=65536, erasures=4, reps=10):
    """rse_reconstruct_batch (core.rs:680-923 per stripe, every stripe its own
    erasure pattern, planned on the device) of GF(2^16) 20+8 x 4 KiB stripes,
    `erasures` random shards lost per stripe, flags in HBM (read in place).
    The lost shards are poisoned before the timed calls; afterwards every
    stripe must equal its encoded bytes again.  GB/s counts the k shards read
    and the lost ones written per stripe."""
    import numpy as np
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix, last_kernel
    k, p, L, field = 20, 8, 4096, 16
    T = k + p
    buf = torch.empty(stripes * T * L, dtype=torch.uint8, device="cuda")
    fill_splitmix(buf, SEED, 0xB4)
    r = R.core.ReedSolomon(k, p, field)
    elems = L // 2
    r.encode_flat(buf, elems, stripes)
    want = buf.clone()
    rng = np.random.default_rng(0xB4)
    lost = np.argsort(rng.random((stripes, T)), axis=1)[:, :erasures]
    pres = np.ones((stripes, T), bool)
    np.put_along_axis(pres, lost, False, axis=1)
    dpres = torch.from_numpy(pres).cuda()
    v = buf.view(stripes, T, L)

    def poison_lost():
        v[~dpres] = POISON

    gbps = timed_gbps(lambda: r.reconstruct_batch(buf, elems, stripes, dpres), stripes *
                      (k + erasures) * L, stream, reps=reps, prepare=poison_lost)
    out = {"workload": f"gf16 {k}+{p} x 4 KiB, {stripes} stripes, {erasures} random shards lost "
                       "per stripe, flags in HBM", "GB_per_s": gbps, "kernel": last_kernel(),
           "rebuilt_ok_all_stripes": bool(torch.equal(buf, want))}
    # reconstruct_data (core.rs:690): the lost data shards only; stripes that
    # lost none are left alone, and lost parity keeps its poison
    miss = (~pres[:, :k]).sum(axis=1)
    nbytes = int(((miss > 0) * k + miss).sum()) * L
    out["data_only_GB_per_s"] = timed_gbps(
        lambda: r.reconstruct_batch(buf, elems, stripes, dpres, data_only=True), nbytes, stream,
        reps=reps, prepare=poison_lost)
    dmask = torch.from_numpy(pres).cuda()
    dmask[:, k:] = True  # parity shards: not compared
    out["data_only_rebuilt_ok_all_stripes"] = bool(torch.equal(v[~dmask], want.view(
        stripes, T, L)[~dmask])) and bool(torch.equal(v[:, :k], want.view(stripes, T, L)[:, :k]))
    del buf, want, v
    torch.cuda.empty_cache()
    return out


def head_tail_ok(v, field, k, p, check):
    """Stripe 0's parity in the stripe view v[stripe, shard, byte] against the
    oracle's encode of its first and last `check` bytes (byte column j of the
    parity depends only on byte column j of the data)."""
    import numpy as np
    from oracle import oracle as O
    oc = O.Codec(field, k, p)
    n = v.shape[-1]
    ok = True
    for sl in (slice(0, check), slice(n - check, n)):
        sh = [v[0, i, sl].cpu().numpy().copy() for i in range(k)] + \
             [np.zeros(check, np.uint8) for _ in range(p)]
        oc.encode(sh)
        ok = ok and all(np.array_equal(sh[k + j], v[0, k + j, sl].cpu().numpy())
                        for j in range(p))
    return ok


def wide_config(stream, g, field, k, p):
    """A wide codec x 1 MiB shards on its one-module kernel (rse_jit.cpp
    kJitWide, built by hiprtc in helper processes before timing), stripe 0's
    parity against the digests of tests/golden: GF(2^8) 50+20, the widest
    codec of the reference's own bench (benches/bandwidth.rs:128; digest from
    the reference's compiled kernel), and GF(2^16) 40+12 (digest from the
    restatement of lib.rs:99-118)."""
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix, last_kernel
    nbytes, stripes = MiB, 128
    T = k + p
    buf = torch.empty(stripes * T * nbytes, dtype=torch.uint8, device="cuda")
    v = buf.view(stripes, T, nbytes)
    for s_ in range(stripes):
        for i in range(k):
            fill_splitmix(v[s_, i], SEED, shard_id(s_, i))
    r = R.core.ReedSolomon(k, p, field)
    t0 = time.perf_counter()
    kind = kernels_within(r, JIT_BUDGET_S)
    build_s = time.perf_counter() - t0
    if kind is None:
        del buf, v
        torch.cuda.empty_cache()
        return {"skipped": f"modules not built within {JIT_BUDGET_S:.0f} s (cold JIT cache)"}
    elems = nbytes // (field // 8)
    enc = timed_gbps(lambda: r.encode_flat(buf, elems, stripes), stripes * T * nbytes, stream,
                     reps=20, warm_s=0.25)
    d = {"workload": f"gf{field} {k}+{p} x 1 MiB, {stripes} stripes/launch", "kernels": kind,
         "timing": "0.25 s of untimed launches, then 20 back to back (HIP events)",
         "kernel": last_kernel(), "build_seconds": round(build_s, 1),
         "encode_GB_per_s": enc, "encode_MB_per_s": round(enc * 1e9 / MiB, 1),
         "encode_roofline_frac": round(enc / HBM_PEAK_GBPS, 4)}
    fs = g["full_size"].get(f"gf{field}_{k}_{p}_{nbytes}")
    if fs is not None:
        d["parity_check_vs_reference" if field == 8 else "parity_check_vs_restatement"] = \
            digests_ok(v, range(k, T), fs["parity_sha256"])
    else:  # no fixture: stripe 0's first and last 4 KiB against the oracle
        d["parity_check_vs_oracle_stripe0_head_tail"] = head_tail_ok(v, field, k, p, 4096)
    del buf, v
    torch.cuda.empty_cache()
    return d


# ------------------------------------------------- the reference's own bench
# benches/bandwidth.rs:88-190: GF(2^8) 1 KiB blocks x {4+4, 8+8, 16+16, 32+32,
# 64+64, 5+2, 10+4, 50+20}, and 4+4 at 2, 4, 8 and 16 KiB; encode, and
# reconstruct after data shards 0..delete-1 are set to None (one: delete 1,
# all: delete p, none: delete 0).  Criterion counts data bytes (k x block) per
# iteration (bandwidth.rs:41-43, 65-67).
REF_BENCH_SHAPES = ([(1024, k, p) for k, p in ((4, 4), (8, 8), (16, 16), (32, 32), (64, 64),
                                               (5, 2), (10, 4), (50, 20))]
                    + [(b, 4, 4) for b in (2048, 4096, 8192, 16384)])
REF_BENCH_OPS = (("encode", None), ("reconstruct_one", 1), ("reconstruct_all", -1),
                 ("reconstruct_none", 0))


def per_call_us(fn, budget_s=0.02, min_calls=16):
    """Mean microseconds per fn() call over >= min_calls calls and >= budget_s."""
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if n >= min_calls and dt >= budget_s:
            return dt / n * 1e6


def _ref_rows(k, p, erased):
    """The rows the reference codes with: the parity rows (encode, core.rs:
    420-428), or the decode rows of the missing data shards over the first k
    present shards (core.rs:697-731, 801-861; the LRU-cached steady state)."""
    import numpy as np
    from oracle import oracle as O
    m = np.asarray(O.Codec(8, k, p).matrix(), np.uint8)
    if erased is None:
        return np.ascontiguousarray(m[k:]), list(range(k))
    valid = [i for i in range(k + p) if i not in erased][:k]
    return np.ascontiguousarray(O.matrix_invert(8, m[valid])[list(erased)]), valid


def cpu_reference_call_us(k, p, block, erased, budget_s=0.02):
    """The reference's simd_c kernel in code_some_slices order (oracle/_ref,
    1 thread) per encode / reconstruct call at this shape, the repetitions
    inside C (no per-call FFI cost); None when oracle/_ref is absent."""
    import numpy as np
    from oracle import oracle as O
    if not O.ref_available():
        return None
    rows, ins = _ref_rows(k, p, erased)
    data = [O.splitmix_bytes(SEED, i, block) for i in range(k + p)]
    outs = [np.zeros(block, np.uint8) for _ in range(rows.shape[0])]
    ref = O.ref()
    args = (rows.ctypes.data_as(O._u8p), rows.shape[0], k, O._ptrs([data[i] for i in ins]),
            O._ptrs(outs), block)
    reps = 1
    while True:
        t0 = time.perf_counter()
        ref.ref_gf8_code_repeat(*args, reps)
        dt = time.perf_counter() - t0
        if dt >= budget_s or reps >= 1 << 22:
            return dt / reps * 1e6
        reps *= 4


def reference_bench_matrix(stream, shapes=None, crossover_sizes=None):
    """The reference's criterion matrix on this GPU, three ways per shape:
    batched (many stripes per launch, the flat ABI: GB/s), one synchronous
    call per stripe on device shards (what a drop-in caller of
    ReedSolomon::encode with HBM-resident shards waits), and one call on
    pageable host shards (the reference's own memory: H2D, kernel, D2H);
    beside the reference's CPU kernel per call on this host.  Then a 10+4
    shard-size sweep for the per-call crossover."""
    import ctypes
    import numpy as np
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix
    from oracle import oracle as O
    lib = R_lib()
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    out = {"what": "benches/bandwidth.rs:88-190 shapes; data_MB_per_s counts k x block per "
                   "call as criterion does; *_call_us are per synchronous call (python ctypes "
                   "loop, ~1 us of call overhead included): gpu_call_device = the stream entry + "
                   "stream synchronisation, gpu_call_now = the synchronous entry (rse_*_now: "
                   "small stripes on the resident dispatcher), gpu_call_host = the *_host entry "
                   "on pageable host shards; cpu_reference = simd_c -O3 "
                   "-march=haswell in core.rs loop order, 1 thread, decode rows cached; "
                   "run-time kernel builds waited for (RSE_OPT_JIT 2): steady state, as the "
                   "reference's repeated calls with their decode rows cached",
           "entries": []}
    jit_old = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)
    try:
        _matrix_rows(lib, stream, st, sh, out, one_stripe_fn(), shapes)
    finally:
        lib.rse_set_option(9, jit_old)
    out["crossover_10_4"] = (per_call_crossover(stream, crossover_sizes) if crossover_sizes
                             else per_call_crossover(stream))
    return out


def one_stripe_fn():
    import ctypes
    import numpy as np

    def one_stripe(k, p, block, src):
        T = k + p
        ptrs = (ctypes.c_void_p * T)(*[src[i].data_ptr() for i in range(T)])
        lens = (ctypes.c_size_t * T)(*([block] * T))
        host = [np.ascontiguousarray(src[i].cpu().numpy()) for i in range(T)]
        hptrs = (ctypes.c_void_p * T)(*[h.ctypes.data for h in host])
        return ptrs, lens, hptrs, host  # `host` owns the memory hptrs points to
    return one_stripe


def _matrix_rows(lib, stream, st, sh, out, one_stripe, shapes):
    """reference_bench_matrix's rows, one per (shape, op)."""
    import ctypes
    import numpy as np
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix, last_kernel
    from oracle import oracle as O
    for block, k, p in (shapes or REF_BENCH_SHAPES):
        T = k + p
        r = R.core.ReedSolomon(k, p, 8)
        # time the codec's bit-sliced kernels, not the table kernels while they
        # build (1 and 2 KiB shards: RSE_OPT_SUB_CHUNKS)
        if kernels_within(r, JIT_BUDGET_S) is None:
            out["entries"].append({"shape": f"{k}+{p} x {block // 1024} KiB",
                                   "skipped": "modules not built in time (cold JIT cache)"})
            continue
        n = max(1, min(32768, (256 << 20) // (T * block)))
        buf = torch.empty(n * T * block, dtype=torch.uint8, device="cuda")
        fill_splitmix(buf, SEED, 0x7E57)
        v = buf.view(n, T, block)
        r.encode_flat(buf, block, n)
        torch.cuda.synchronize()
        ptrs, lens, hptrs, host_shards = one_stripe(k, p, block, v[0])
        data_bytes = k * block
        for op, delete in REF_BENCH_OPS:
            e = {"shape": f"{k}+{p} x {block // 1024} KiB", "op": op}
            if op == "encode":
                e["gpu_flat"] = {"stripes": n, "GB_per_s": timed_gbps(
                    lambda: r.encode_flat(buf, block, n), n * T * block, stream),
                    "kernel": last_kernel()}
                rows, _ = _ref_rows(k, p, None)
                want = [np.zeros(block, np.uint8) for _ in range(p)]
                O.code_some_slices(8, rows, [v[0, i].cpu().numpy() for i in range(k)], want)
                e["parity_stripe0_vs_oracle"] = all(
                    np.array_equal(v[0, k + i].cpu().numpy(), want[i]) for i in range(p))

                def dev():
                    _ck(lib.rse_encode(r._h, ptrs, lens, T, sh))
                    st.synchronize()

                def dev_async():
                    _ck(lib.rse_encode(r._h, ptrs, lens, T, sh))

                def host():
                    _ck(lib.rse_encode_host(r._h, hptrs, lens, T, sh))

                def now():
                    _ck(lib.rse_encode_now(r._h, ptrs, lens, T))
                erased = None
            else:
                d = p if delete == -1 else delete
                erased = list(range(d))
                pres = (ctypes.c_uint8 * T)(*[0 if i in erased else 1 for i in range(T)])
                if d:
                    leg = reconstruct_leg(r, v, k, erased, block, n, stream, None, None)
                    e["gpu_flat"] = {"stripes": n, "GB_per_s": leg["GB_per_s"],
                                     "kernel": last_kernel()}
                    e["rebuilt_ok_all_stripes"] = leg["rebuilt_ok_all_stripes"]

                def dev():
                    _ck(lib.rse_reconstruct(r._h, ptrs, lens, pres, T, sh))
                    st.synchronize()

                def dev_async():
                    _ck(lib.rse_reconstruct(r._h, ptrs, lens, pres, T, sh))

                def host():
                    _ck(lib.rse_reconstruct_host(r._h, hptrs, lens, pres, T, sh))

                def now():
                    _ck(lib.rse_reconstruct_now(r._h, ptrs, lens, pres, T))
            if "gpu_flat" in e:
                f = e["gpu_flat"]
                alg = T if op == "encode" else k + len(erased)
                f["data_MB_per_s"] = round(f["GB_per_s"] * 1e9 * k / alg / MiB, 1)
            e["gpu_call_device_us"] = round(per_call_us(dev), 2)
            t_async = per_call_us(dev_async)
            st.synchronize()
            e["gpu_call_device_async_us"] = round(t_async, 2)
            e["gpu_call_host_us"] = round(per_call_us(host), 2)
            st.synchronize()
            e["gpu_call_now_us"] = round(per_call_us(now), 2)
            if erased is None or erased:
                c = cpu_reference_call_us(k, p, block, erased)
                e["cpu_reference_call_us"] = round(c, 3) if c is not None else None
            for key in ("gpu_call_device_us", "gpu_call_host_us", "gpu_call_now_us",
                        "cpu_reference_call_us"):
                if e.get(key):
                    e[key.replace("_us", "_data_MB_per_s")] = round(data_bytes / e[key] / MiB * 1e6, 1)
            out["entries"].append(e)
        del buf, v, host_shards
        torch.cuda.empty_cache()


def _ck(rc):
    if rc != 0:
        raise RuntimeError(f"rse call failed with status {rc}")


def per_call_crossover(stream, sizes=(1 << 10, 4 << 10, 8 << 10, 16 << 10, 32 << 10,
                                      64 << 10, 256 << 10, 1 << 20, 4 << 20)):
    """One 10+4 stripe per synchronous encode call at growing shard sizes:
    device shards, pageable host shards and the reference CPU kernel, and the
    smallest size at which each GPU form beats the CPU."""
    import ctypes
    import numpy as np
    import torch
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix
    lib = R_lib()
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    k, p = 10, 4
    T = k + p
    r = R.core.ReedSolomon(k, p, 8)
    rows = []
    for L in sizes:
        dv = torch.empty((T, L), dtype=torch.uint8, device="cuda")
        fill_splitmix(dv, SEED, 0xC0)
        ptrs = (ctypes.c_void_p * T)(*[dv[i].data_ptr() for i in range(T)])
        lens = (ctypes.c_size_t * T)(*([L] * T))
        host = [np.ascontiguousarray(dv[i].cpu().numpy()) for i in range(T)]
        hptrs = (ctypes.c_void_p * T)(*[h.ctypes.data for h in host])

        def dev():
            _ck(lib.rse_encode(r._h, ptrs, lens, T, sh))
            st.synchronize()

        def host_call():
            _ck(lib.rse_encode_host(r._h, hptrs, lens, T, sh))

        def now():
            _ck(lib.rse_encode_now(r._h, ptrs, lens, T))
        row = {"shard_bytes": L, "gpu_call_device_us": round(per_call_us(dev), 2),
               "gpu_call_host_us": round(per_call_us(host_call), 2)}
        st.synchronize()
        row["gpu_call_now_us"] = round(per_call_us(now), 2)
        c = cpu_reference_call_us(k, p, L, None)
        row["cpu_reference_call_us"] = round(c, 2) if c is not None else None
        rows.append(row)
        del dv
    out = {"what": "10+4 encode, one stripe per synchronous call (device shards: rse_encode + "
                   "stream synchronisation, and rse_encode_now; pageable host shards; reference "
                   "CPU kernel, 1 thread)", "rows": rows}
    for key in ("gpu_call_device_us", "gpu_call_now_us", "gpu_call_host_us"):
        win = [x["shard_bytes"] for x in rows
               if x["cpu_reference_call_us"] is not None and x[key] < x["cpu_reference_call_us"]]
        out[f"{key.replace('_us', '')}_beats_cpu_from_shard_bytes"] = min(win) if win else None
    return out


def R_lib():
    import reed_solomon_erasure as R
    return R._lib.load()


def fresh_extra_legs(r, k, p, L, n_stripes, stream):
    """extra_legs on `n_stripes` stripes in an allocation of their own, made
    after the headline's buffer is freed: the reconstruct and verify legs do
    not depend on where the headline's 112 GiB left free memory."""
    import torch
    from reed_solomon_erasure.core import fill_splitmix
    buf = torch.empty(n_stripes * (k + p) * L, dtype=torch.uint8, device="cuda")
    v = buf.view(n_stripes, k + p, L)
    for s in range(n_stripes):
        for i in range(k):
            fill_splitmix(v[s, i], SEED, shard_id(s, i))
    r.encode_flat(buf, L, n_stripes)
    try:
        return extra_legs(r, v, k, p, L, n_stripes, stream)
    finally:
        del v, buf
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def extra_legs(r, v, k, p, L, n_stripes, stream, stripe0=0):
    """Reconstruct (data shards 0 and 1 erased, BASELINE config 3), verify
    with corrupted stripes, and the pinned-host end-to-end legs
    (PCIe-inclusive; never `value`).  Every reconstruct leg poisons the erased
    shards before its timed calls and checks every rebuilt shard after them."""
    import torch
    from reed_solomon_erasure.core import fill_splitmix
    out = {}
    lib = R_lib()
    ids = [stripe0 + s for s in range(n_stripes)]
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["generated"]
    fs = g["full_size"].get(f"gf8_{k}_{p}_{L}")
    want = fs["data_sha256"][:2] if (fs and stripe0 == 0) else None
    lib.rse_set_option(11, 0)  # decode-pattern kernels off: the syndrome kernel
    try:
        leg = reconstruct_leg(r, v, k, [0, 1], L, n_stripes, stream, fill_splitmix, ids, want)
    finally:
        lib.rse_set_option(11, 1)
    out["reconstruct"] = {"what": "reconstruct_data, data shards 0,1 erased, first uses of the "
                                  "pattern (bit-sliced syndrome kernel); erased shards poisoned "
                                  "before the timed calls", "stripes": n_stripes,
                          "MB_per_s": round(leg["GB_per_s"] * 1e9 / MiB, 1),
                          "algorithmic_GB_per_s": leg["GB_per_s"],
                          "rebuilt_ok_all_stripes": leg["rebuilt_ok_all_stripes"],
                          "rebuilt_stripe0_vs_reference": leg.get("rebuilt_stripe0_vs_digests")}
    # a repeated pattern: its decode rows get their own specialised kernel
    # (rse_jit.cpp), like the reference's decode-matrix cache (core.rs:697-731);
    # RSE_OPT_JIT 2 waits for that build before timing
    old = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)
    p0 = lib.rse_get_option(12)
    reps = 5
    try:
        leg = reconstruct_leg(r, v, k, [0, 1], L, n_stripes, stream, fill_splitmix, ids, want,
                              reps=reps)
    finally:
        lib.rse_set_option(9, old)
    out["reconstruct_cached_pattern"] = {
        "what": "reconstruct_data, data shards 0,1 erased, repeated pattern (decode-pattern "
                "kernel specialised at run time); erased shards poisoned before the timed calls",
        "stripes": n_stripes, "pattern_kernel": lib.rse_get_option(12) - p0 == reps + 1,
        "MB_per_s": round(leg["GB_per_s"] * 1e9 / MiB, 1),
        "algorithmic_GB_per_s": leg["GB_per_s"],
        "rebuilt_ok_all_stripes": leg["rebuilt_ok_all_stripes"],
        "rebuilt_stripe0_vs_reference": leg.get("rebuilt_stripe0_vs_digests")}
    # verify (check mode: k+p reads, no writes), stripe by stripe as the API
    # is, and the same check over every stripe in one pass (rse_verify_flat)
    n_stripes = min(n_stripes, 64)
    out["verify"], out["verify_flat"] = verify_leg(r, v, k, p, L, n_stripes, reps=reps)
    # end to end from pinned host memory: one stripe, H2D data, D2H parity
    hs = [v[0, i].cpu().pin_memory() for i in range(k)] + \
         [torch.empty(L, dtype=torch.uint8).pin_memory() for _ in range(p)]
    r.encode_host(hs)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        r.encode_host(hs)
    dt = (time.perf_counter() - t0) / reps
    ok = all(torch.equal(hs[k + i], v[0, k + i].cpu()) for i in range(p))
    out["end_to_end_pinned_host"] = {
        "what": "rse_encode_host, 1 stripe from pinned host memory (H2D data + kernel + D2H parity)",
        "MB_per_s": round((k + p) * L / dt / MiB, 1), "parity_matches_device": ok}
    # many stripes through one pipeline (rse_encode_host_flat): the first call
    # on its own, then 0.5 s of untimed calls and 3 timed ones (steady state)
    ns = min(8, n_stripes)
    hflat = v[:ns].reshape(-1).cpu().pin_memory()
    hflat.view(ns, k + p, L)[:, k:].zero_()
    t0 = time.perf_counter()
    r.encode_host_flat(hflat, L, ns)
    dt_first = time.perf_counter() - t0
    warm_calls(lambda: r.encode_host_flat(hflat, L, ns))
    t0 = time.perf_counter()
    reps = 10  # ~0.3 s: the same count as host_leg, whose figure this is compared with
    for _ in range(reps):
        r.encode_host_flat(hflat, L, ns)
    dt = (time.perf_counter() - t0) / reps
    ok = torch.equal(hflat.view(ns, k + p, L)[:, k:], v[:ns, k:].cpu())
    # the PCIe ceiling in this process: one plain pinned H2D copy of the same bytes
    dbuf = torch.empty_like(hflat, device="cuda")
    dbuf.copy_(hflat, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dbuf.copy_(hflat, non_blocking=True)
    torch.cuda.synchronize()
    raw_h2d = hflat.numel() / ((time.perf_counter() - t0) / reps) / 1e9
    # ... and the ceiling of the encode's own traffic: plain copies of the data
    # shards up and the parity shards down at the same time (two streams)
    hv = hflat.view(ns, k + p, L)
    dv = dbuf.view(ns, k + p, L)
    hpar = torch.empty((ns, p, L), dtype=torch.uint8).pin_memory()
    up, down = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():  # per stripe: each copy is one contiguous block
        with torch.cuda.stream(up):
            for s_ in range(ns):
                dv[s_, :k].copy_(hv[s_, :k], non_blocking=True)
        with torch.cuda.stream(down):
            for s_ in range(ns):
                hpar[s_].copy_(dv[s_, k:], non_blocking=True)
    duplex()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        duplex()
    torch.cuda.synchronize()
    dt_raw = (time.perf_counter() - t0) / reps
    del dbuf, hpar
    out["end_to_end_pinned_host_flat"] = {
        "what": f"rse_encode_host_flat, {ns} stripes from pinned host memory, one "
                "H2D/kernel/D2H pipeline",
        "MB_per_s": round(ns * (k + p) * L / dt / MiB, 1),
        "first_call_MB_per_s": round(ns * (k + p) * L / dt_first / MiB, 1),
        "timing": "first call alone; then 0.5 s of untimed calls, 10 timed",
        "outputs_in_place": bool(lib.rse_get_option(53)),
        "GB_per_s_pcie_h2d": round(ns * k * L / dt / 1e9, 1),
        "raw_pinned_h2d_copy_GB_per_s": round(raw_h2d, 1),
        "raw_pinned_duplex_MB_per_s": round(ns * (k + p) * L / dt_raw / MiB, 1),
        "raw_pinned_duplex_what": "plain copies of the same data shards H2D and parity "
                                  "shards D2H at once (the encode's traffic, no kernel)",
        "parity_matches_device": ok}
    # the decode direction from host memory: data shards 0 and 1 of every
    # stripe lost; only the k valid shards go up, only the 2 rebuilt come back
    want = hflat.view(ns, k + p, L)[:, :2].clone()
    pres = [[i not in (0, 1) for i in range(k + p)]] * ns
    hflat.view(ns, k + p, L)[:, :2].zero_()
    r.reconstruct_host_batch(hflat, L, ns, pres, data_only=True)
    warm_calls(lambda: r.reconstruct_host_batch(hflat, L, ns, pres, data_only=True))
    t0 = time.perf_counter()
    for _ in range(reps):
        hflat.view(ns, k + p, L)[:, :2].zero_()
        r.reconstruct_host_batch(hflat, L, ns, pres, data_only=True)
    dt = (time.perf_counter() - t0) / reps
    ok = torch.equal(hflat.view(ns, k + p, L)[:, :2], want)
    out["end_to_end_pinned_host_reconstruct"] = {
        "what": f"rse_reconstruct_host_batch (data_only), {ns} stripes in pinned host memory, "
                "data shards 0,1 erased: H2D of the 10 valid shards, kernel, D2H of 2",
        "MB_per_s": round(ns * (k + 2) * L / dt / MiB, 1),
        "GB_per_s_pcie_h2d": round(ns * k * L / dt / 1e9, 1),
        "raw_pinned_h2d_copy_GB_per_s": round(raw_h2d, 1), "rebuilt_matches": ok}
    # verify from host memory (reads all k + p shards over PCIe)
    t0 = time.perf_counter()
    for _ in range(reps):
        oks = r.verify_host_flat(hflat, L, ns)
    dt = (time.perf_counter() - t0) / reps
    out["end_to_end_pinned_host_verify"] = {
        "what": f"rse_verify_host_flat, {ns} stripes in pinned host memory (H2D of k + p shards)",
        "MB_per_s": round(ns * (k + p) * L / dt / MiB, 1),
        "GB_per_s_pcie_h2d": round(ns * (k + p) * L / dt / 1e9, 1), "all_ok": bool(oks.all())}
    return out


if __name__ == "__main__":
    main()
