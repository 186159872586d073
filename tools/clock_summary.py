#!/usr/bin/env python3
"""Per-kernel table of rocprofv3 --pmc passes, one directory per workload
(tools/clock_session.sh): mean dispatch duration (its own Start/End
timestamps), the per-dispatch mean of every counter, and -- when the pass
holds GRBM_GUI_ACTIVE (GPU-busy cycles) -- the average clock, cycles / ns.

    python tools/clock_summary.py gpurun_out/clock
"""
import collections
import csv
import glob
import os
import sys

SKIP = ("fill_splitmix", "elementwise", "rocclr", "bs_recon_plan", "recon_plan")


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, "*", ""))):
        tag = os.path.basename(os.path.dirname(d))
        sums = collections.defaultdict(collections.Counter)   # kernel -> counter -> sum
        ns = collections.defaultdict(dict)                     # kernel -> dispatch -> ns
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                name = r["Kernel_Name"]
                if any(s in name for s in SKIP):
                    continue
                k = name[:100]
                sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
                ns[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k in sorted(sums, key=lambda x: -sum(ns[x].values())):
            n = len(ns[k])
            mean_ns = sum(ns[k].values()) / n
            parts = [f"{tag:14s} {n:3d} disp {mean_ns / 1e3:9.1f} us"]
            c = sums[k]
            if "GRBM_GUI_ACTIVE" in c:
                parts.append(f"clock {c['GRBM_GUI_ACTIVE'] / n / mean_ns:5.2f} GHz")
            for cn in sorted(c):
                parts.append(f"{cn}={c[cn] / n:.4g}")
            print("  ".join(parts) + f"  [{k}]")


if __name__ == "__main__":
    main()
