#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel and grid size, call
count and mean/min/max duration (so the bench's launches are not averaged with
the smoke/extras launches of the same kernel).

    python tools/trace_summary.py gpurun_out/prof_trace/bench_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path):
    g = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        grid = (r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        g[(r["Kernel_Name"], grid)].append(dur)
    print("kernel | grid | calls | mean_ms | min_ms | max_ms")
    for (name, grid), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:90]} | {'x'.join(grid)} | {len(d)} | {sum(d)/len(d):.4f} | "
              f"{min(d):.4f} | {max(d):.4f}")


if __name__ == "__main__":
    main(sys.argv[1])
