#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 --pmc counters for kernels whose name contains SUBSTR.

    python tools/pmc_kernel.py gpurun_out/TAG SUBSTR [SUBSTR ...]
FETCH_SIZE / WRITE_SIZE are in KiB units on gfx950 (MI355X_MICROARCH.md: HBM bytes ≈
(2·FETCH_SIZE + WRITE_SIZE)·1 KiB is the guide's correction for this part)."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
for sub in sys.argv[2:]:
    vals = collections.defaultdict(list)
    for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {sub}")
    for k, v in sorted(vals.items()):
        print(f"  {k:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
