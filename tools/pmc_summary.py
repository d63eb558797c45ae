#!/usr/bin/env python3
"""Per-launch averages of rocprofv3 --pmc counters for the GEMM kernel of pmc_gemm.sh passes.

    python tools/pmc_summary.py gpurun_out/pmc [OPS]
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md); the shares below
are of SQ_WAVE_CYCLES.  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 · 256 CUs · 4 SIMDs).
"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
ops = sys.argv[2].split(",") if len(sys.argv) > 2 else ["0", "1", "2"]
for op in ops:
    tot = collections.defaultdict(float)
    n = collections.defaultdict(int)
    for f in glob.glob(os.path.join(root, f"op{op}_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "gemm" not in r["Kernel_Name"]:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
    if not tot:
        continue
    avg = {k: tot[k] / n[k] for k in tot}
    wave = avg.get("SQ_WAVE_CYCLES", 0)
    print(f"== op{op} (per launch averages over {max(n.values())} launches)")
    for k in sorted(avg):
        share = f"  {100 * avg[k] / wave:5.1f}% of wave-cycles" if wave and k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
        print(f"  {k:28s} {avg[k]:16.0f}{share}")
    if "GRBM_GUI_ACTIVE" in avg and "SQ_VALU_MFMA_BUSY_CYCLES" in avg:
        cyc = avg["GRBM_GUI_ACTIVE"] / 8
        print(f"  MFMA busy {100 * avg['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 256 * 4):.1f}% of {cyc:.0f} GPU cycles")
