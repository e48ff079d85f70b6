#!/usr/bin/env python3
"""attn_fwd_kernel HBM-side traffic per launch (bench.pmc_traffic: FETCH_SIZE / WRITE_SIZE passes)
for the Wan2.1 and CogVideoX points, on the predicted masks of the synthetic inputs and on a band
mask with the same kept count per row (tools/attn_only.py "band"): whether the excess over the
algorithmic bytes follows the kernel's traversal or the masks' locality.
usage: python tools/diag/traffic_probe.py [--out FILE]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    res = []
    for variant, density in (("wan", None), ("cog", None), ("cog", 0.05)):
        for band in (False, True):
            t = bench.pmc_traffic(variant, density=density, band=band)
            r = {"variant": variant, "mask": ("energy rule" if density is None else f"density {density}")
                 + (" -> band" if band else " (predicted)"), "traffic": t}
            res.append(r)
            print(json.dumps(r), flush=True)
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
