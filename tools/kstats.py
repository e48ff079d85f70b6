#!/usr/bin/env python3
"""Print a rocprofv3 *kernel_stats.csv compactly: calls, average us, total share (names cut)."""
import csv
import glob
import sys

for path in sys.argv[1:]:
    for f in sorted(glob.glob(path + "/**/*kernel_stats.csv", recursive=True)) or [path]:
        print(f"== {f}")
        for r in csv.DictReader(open(f)):
            name = r["Name"].split("(")[0].replace("void ", "")[:70]
            print(f"  {name:70s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1000:9.2f} us {float(r['Percentage']):6.2f}%")
