#!/usr/bin/env python3
"""rocprofv3 target: the predictor alone (score only) and whole calls, on one library variant.
usage: python tools/diag/pred_prof.py TAG [variant]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import ab  # noqa: E402
import vblade  # noqa: E402
from vblade import _lib  # noqa: E402
from bench import realistic_qkv  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] != "tree":
    _lib._lib = ab.load(sys.argv[1])
variant = sys.argv[2] if len(sys.argv) > 2 else "cog"
mode = sys.argv[3] if len(sys.argv) > 3 else "both"
dev = torch.device("cuda")
H, D = (48, 64) if variant == "cog" else (12, 128)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(H, L, D, 0, dev)
qo = vblade.draw_sample_offsets(1, H, dev)
ko = vblade.draw_sample_offsets(1, H, dev)
with torch.no_grad():
    if mode in ("both", "pred"):
        for _ in range(20):
            m.predict_mask(q, k, qo, ko)
    if mode in ("both", "call"):
        for _ in range(20):
            m(q, k, v)
torch.cuda.synchronize()
print("done")
