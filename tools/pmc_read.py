#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per dispatch of the GEMM kernel found under a directory."""
import collections
import csv
import glob
import sys

vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm" not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
