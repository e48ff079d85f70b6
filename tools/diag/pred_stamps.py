#!/usr/bin/env python3
"""Per-phase s_memtime sums of the predictor's score kernel (diagnostic build: tools/build_variant.sh
pstamp with VB_EXTRA_FLAGS=-DVB_PRED_STAMPS=1): per active wave, the cycles spent waiting for its
K tile's DMA, at the barrier, issuing the next DMAs, in the whole loop body, and in the epilogue
up to the Po row. usage: python tools/diag/pred_stamps.py [cog|wan] [pred|call]"""
import ctypes
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

variant = sys.argv[1] if len(sys.argv) > 1 else "cog"
what = sys.argv[2] if len(sys.argv) > 2 else "pred"
lib = ab.load("pstamp")
lib.vb_debug_pred_stamps.restype = ctypes.c_int
lib.vb_debug_pred_stamps.argtypes = [ctypes.c_void_p]
_lib._lib = lib
dev = torch.device("cuda")
H, D = (48, 64) if variant == "cog" else (12, 128)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(H, L, D, 0, dev)
qo = vblade.draw_sample_offsets(1, H, dev)
ko = vblade.draw_sample_offsets(1, H, dev)
buf = (ctypes.c_ulonglong * 8)()
with torch.no_grad():
    for rep in range(2):
        torch.cuda.synchronize()
        lib.vb_debug_pred_stamps(buf)   # clear
        for _ in range(10):
            if what == "pred":
                m.predict_mask(q, k, qo, ko)
            else:
                m(q, k, v)
        torch.cuda.synchronize()
        assert lib.vb_debug_pred_stamps(buf) == 0
n = max(buf[5], 1)
names = ["dma wait", "barrier", "issue", "loop total", "epilogue to Po"]
print(f"{variant} {what}: {n // 10} waves per launch; cycles per wave:")
for i, nm in enumerate(names):
    print(f"  {nm:16s} {buf[i] / n:10.0f}")
