#!/usr/bin/env python3
"""Per-kernel SQ counter summary of rocprofv3 --pmc runs (one directory per
pass): every counter summed over the kernel's dispatches, then the ratios that
say where a wave's cycles go.

    python tools/pmc_summary.py gpurun_out/pmc_recon8 [regex]

Ratios (SQ_* counters are per wave, summed over waves; SQ_BUSY_CYCLES counts
SQ-busy cycles of the whole chip, per SE):
  valu_per_wave_cycle   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES
  any_per_wave_cycle    SQ_ACTIVE_INST_ANY  / SQ_WAVE_CYCLES   (issuing anything)
  wait_any              SQ_WAIT_ANY / SQ_WAVE_CYCLES            (waiting on a dependency)
  wait_inst_any         SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES       (waiting to issue, incl. ifetch)
  valu_insts_per_wave   SQ_INSTS_VALU / SQ_WAVES
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(root, regex):
    tot = collections.Counter()
    disp = collections.Counter()
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if regex and not re.search(regex, r["Kernel_Name"]):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]] += 1
    return tot, disp


def main():
    root = sys.argv[1]
    regex = sys.argv[2] if len(sys.argv) > 2 else ""
    raw, disp = load(root, regex)
    # every pass repeats SQ_WAVE_CYCLES / SQ_WAVES: ratios are taken between
    # per-dispatch means, so a counter of one pass and one of all passes agree
    tot = {k: raw[k] / disp[k] for k in raw}
    out = {"counters": {k: raw[k] for k in sorted(raw)}, "dispatches": dict(disp),
           "per_dispatch_mean": {k: round(tot[k], 1) for k in sorted(tot)}}
    wc = tot.get("SQ_WAVE_CYCLES")
    if wc:
        for name, key in (("valu_per_wave_cycle", "SQ_ACTIVE_INST_VALU"),
                          ("any_per_wave_cycle", "SQ_ACTIVE_INST_ANY"),
                          ("wait_any", "SQ_WAIT_ANY"), ("wait_inst_any", "SQ_WAIT_INST_ANY"),
                          ("sca_per_wave_cycle", "SQ_ACTIVE_INST_SCA"),
                          ("vmem_per_wave_cycle", "SQ_ACTIVE_INST_VMEM"),
                          ("lds_per_wave_cycle", "SQ_ACTIVE_INST_LDS"),
                          ("misc_per_wave_cycle", "SQ_ACTIVE_INST_MISC"),
                          ("salu_cycles_per_wave_cycle", "SQ_INST_CYCLES_SALU")):
            if key in tot:
                out[name] = round(tot[key] / wc, 4)
    if tot.get("SQ_WAVES"):
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM",
                    "SQ_IFETCH", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS",
                    "SQ_WAVE_CYCLES"):
            if key in tot:
                out[key.lower() + "_per_wave"] = round(tot[key] / tot["SQ_WAVES"], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
