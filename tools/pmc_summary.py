#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch for kernels matching a substring, one block per
distinct kernel (template arguments kept, so the dK/dV, dQ and prep kernels of a backward or the
D=64/D=128 instantiations stay apart), with derived per-wave figures where the counters allow."""
import collections
import csv
import glob
import sys

pat = sys.argv[2] if len(sys.argv) > 2 else "attn_fwd"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in agg.items():
    print(f"-- {name}")
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    for k, v in cs.items():
        print(f"  {k:28s} n={len(v):3d} avg={avg[k]:.4g}")
    if "SQ_INSTS_VALU" in avg and "SQ_INSTS_MFMA" in avg and avg["SQ_INSTS_MFMA"] > 0:
        print(f"  VALU per MFMA (other VALU)   {(avg['SQ_INSTS_VALU'] - avg['SQ_INSTS_MFMA']) / avg['SQ_INSTS_MFMA']:.2f}")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "GRBM_GUI_ACTIVE" in avg and "SQ_BUSY_CYCLES" in avg:
        # MFMA busy cycles summed over SIMDs vs the launch's SIMD-cycles (GRBM_GUI_ACTIVE sums the
        # 8 XCDs: 32 CUs x 4 SIMDs each per XCD)
        simd_cycles = avg["GRBM_GUI_ACTIVE"] / 8 * 256 * 4
        print(f"  MFMA busy fraction            {avg['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f}")
