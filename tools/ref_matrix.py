#!/usr/bin/env python3
"""bench.py's reference bench matrix (benches/bandwidth.rs:88-190 shapes) on
its own: one JSON object on stdout.

    python3 tools/ref_matrix.py [--shapes 1024:4:4,1024:64:64] [--no-crossover]
"""
import argparse
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (sets the JIT cache default, the package path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="", help="block:k:p,... (default: all)")
    ap.add_argument("--no-crossover", action="store_true")
    a = ap.parse_args()
    import torch
    shapes = [tuple(int(x) for x in s.split(":")) for s in a.shapes.split(",") if s] or None
    out = bench.reference_bench_matrix(torch.cuda.current_stream(), shapes,
                                       (1024, 65536) if a.no_crossover else None)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
