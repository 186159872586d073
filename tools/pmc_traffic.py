#!/usr/bin/env python3
"""Per-launch HBM traffic of the headline kernel from rocprofv3 PMC counters.

Runs bench.py twice under rocprofv3 (one counter per pass: FETCH_SIZE, then
WRITE_SIZE -- they cannot share a pass), keeps the dispatches of the fused
encode kernel with the bench's grid, and applies the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide
coalesced stream, so hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Writes profiles/<tag>_pmc_traffic.json, which bench.py reports as
roofline.traffic when the kernel that ran (rse_last_kernel, "kernel_id") is the
one profiled here.  The library's BUILD_INFO.json (its source commit, stamped
by the Makefile when it was built) and its SHA-256 record what was measured.

    python tools/pmc_traffic.py --tag r01 [bench args...]
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(counter, outdir, bench_args):
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-include-regex", "gf8_code|gf8_pipe|bitslice_kernel|bitslice_deep_kernel",
           "--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-extras"] + bench_args
    out = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
    if out.returncode != 0:
        sys.stderr.write(out.stdout[-3000:] + out.stderr[-3000:])
        raise SystemExit(out.returncode)
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    rows = []
    for path in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(path)))
    return json.loads(line), rows


def build_info(lib_path):
    """BUILD_INFO.json next to the library (written by its Makefile where the
    tree has .git): the commit of the library's sources, stamped at build time."""
    try:
        return json.load(open(os.path.join(os.path.dirname(lib_path), "BUILD_INFO.json")))
    except (OSError, ValueError):
        return {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    args, bench_args = ap.parse_known_args()
    base = os.path.join(ROOT, "gpurun_out", "pmc")
    bench, fetch = run("FETCH_SIZE", base + "_fetch", bench_args)
    _, write = run("WRITE_SIZE", base + "_write", bench_args)
    grid = max(int(r["Grid_Size"]) for r in fetch)  # the bench's launches
    f = [float(r["Counter_Value"]) for r in fetch if int(r["Grid_Size"]) == grid]
    w = [float(r["Counter_Value"]) for r in write if int(r["Grid_Size"]) == grid]
    fetch_b = 2 * sum(f) / len(f) * 1024
    write_b = sum(w) / len(w) * 1024
    alg = bench["roofline"]["algorithmic_bytes_per_launch"]
    lib_path = os.path.join(ROOT, "reed-solomon-erasure_amd", "reed_solomon_erasure", "librse_hip.so")
    res = {
        "workload": bench["config"]["workload"],
        "kernel_family": bench["roofline"].get("kernel", "table"),
        "kernel_id": bench["roofline"].get("kernel_id"),
        "commit": build_info(lib_path).get("source_commit"),
        "uncommitted_source_files": build_info(lib_path).get("uncommitted_source_files"),
        "library_sha256": hashlib.sha256(open(lib_path, "rb").read()).hexdigest(),
        "build_info_matches_library": build_info(lib_path).get("library_sha256") ==
        hashlib.sha256(open(lib_path, "rb").read()).hexdigest(),
        "kernel": [r["Kernel_Name"] for r in fetch][0],
        "dispatches": len(f),
        "fetch_size_kb_raw_mean": sum(f) / len(f),
        "write_size_kb_raw_mean": sum(w) / len(w),
        "hbm_read_bytes_per_launch": int(fetch_b),
        "hbm_write_bytes_per_launch": int(write_b),
        "hbm_bytes_per_launch": int(fetch_b + write_b),
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": round((fetch_b + write_b) / alg, 4),
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md §HBM); WRITE_SIZE as is; KB = 1024 B",
    }
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for d in ("profiles", "gpurun_out"):  # gpurun only ships gpurun_out/ back
        os.makedirs(os.path.join(ROOT, d), exist_ok=True)
        json.dump(res, open(os.path.join(ROOT, d, f"{args.tag}_pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
