#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch for kernels matching a substring."""
import collections
import csv
import glob
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else "attn_fwd"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:28s} n={len(v):3d} avg={sum(v) / len(v):.4g}")
