#!/usr/bin/env python3
"""The headline roofline recomputed from a rocprofv3 kernel trace of the bench
(VERDICT r05 §5): keeps the per-dispatch rows of the headline kernel at the
bench's grid (the 512-stripe launches, not the same kernel's other launches),
and recomputes achieved GB/s and the fraction of 8 TB/s from their mean
duration and the line's algorithmic bytes per launch, beside the bench line's
own HIP-event figure and the PMC traffic file it cites.

    python tools/headline_roofline.py <kernel_trace.csv> <bench stdout log> <out dir>
writes <out dir>/headline_dispatches.csv and <out dir>/headline_roofline.json."""
import csv
import json
import os
import sys

PEAK = 8000.0


def main(trace, log, out):
    line = [l for l in open(log) if l.startswith("{")][-1]
    b = json.loads(line)
    roof = b["roofline"]
    alg = roof["algorithmic_bytes_per_launch"]
    rows = [r for r in csv.DictReader(open(trace)) if "bitslice_deep_kernel" in r["Kernel_Name"]
            and "Bs8_10_4" in r["Kernel_Name"]]
    grid = max(int(r["Grid_Size_X"]) for r in rows)  # the 512-stripe launches
    head = [r for r in rows if int(r["Grid_Size_X"]) == grid]
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in head]
    os.makedirs(out, exist_ok=True)
    keep = ["Dispatch_Id", "Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "Start_Timestamp",
            "End_Timestamp"]
    with open(os.path.join(out, "headline_dispatches.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(keep + ["duration_ms"])
        for r, d in zip(head, durs):
            w.writerow([r[k] for k in keep] + [f"{d:.6f}"])
    mean = sum(durs) / len(durs)
    timed = durs[-b["steps"]:] if len(durs) >= b["steps"] else durs
    tmean = sum(timed) / len(timed)
    res = {
        "trace": trace, "bench_log": log, "kernel": head[0]["Kernel_Name"], "grid_size_x": grid,
        "dispatches": len(durs), "mean_ms_all": round(mean, 4),
        "mean_ms_last_steps": round(tmean, 4), "min_ms": round(min(durs), 4),
        "max_ms": round(max(durs), 4), "algorithmic_bytes_per_launch": alg,
        "achieved_GBps_from_trace": round(alg / (tmean * 1e-3) / 1e9, 1),
        "frac_from_trace": round(alg / (tmean * 1e-3) / 1e9 / PEAK, 4),
        "bench_line": {"frac": roof["frac"], "kernel_ms_per_launch": roof["kernel_ms_per_launch"],
                       "traffic": roof.get("traffic"), "traffic_file": roof.get("traffic_file"),
                       "library": b.get("library")},
    }
    res["frac_agreement"] = round(res["frac_from_trace"] / roof["frac"], 4)
    json.dump(res, open(os.path.join(out, "headline_roofline.json"), "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
