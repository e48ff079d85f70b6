#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel_trace.csv: per-call timeline of the attention path (kernel
start/end relative to the call's first kernel), overlap between streams, and idle gaps."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60], r.get("Stream_Id", r.get("Queue_Id", "?"))))
ks.sort()
# find attention kernels to delimit calls
att = [i for i, k in enumerate(ks) if "attn_fwd_kernel" in k[2]]
print(f"{len(ks)} kernels, {len(att)} attention launches")
# look at calls in the middle of the run
for ci in att[len(att) // 2: len(att) // 2 + 3]:
    lo = max(0, ci - 12)
    t0 = ks[lo][0]
    print("---- call ending at kernel", ci)
    for k in ks[lo:ci + 1]:
        print(f"  {(k[0]-t0)/1000:9.1f} -> {(k[1]-t0)/1000:9.1f} us  dur {(k[1]-k[0])/1000:8.1f}  q={k[3]:>3} {k[2]}")
# overall busy fraction between first and last attention kernel of the steady region
a0, a1 = ks[att[len(att) // 4]][0], ks[att[3 * len(att) // 4]][1]
ev = []
for s, e, n, q in ks:
    if e < a0 or s > a1:
        continue
    ev.append((max(s, a0), 1))
    ev.append((min(e, a1), -1))
ev.sort()
busy = 0
cur = 0
last = a0
for t, d in ev:
    if cur > 0:
        busy += t - last
    cur += d
    last = t
print(f"steady region {(a1-a0)/1e6:.3f} ms, GPU busy {busy/(a1-a0)*100:.1f} %")
n = att[3 * len(att) // 4] - att[len(att) // 4]
print(f"per call: {(a1-a0)/1000/max(1,(3*len(att)//4 - len(att)//4)):.1f} us")
