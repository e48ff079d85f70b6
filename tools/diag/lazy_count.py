#!/usr/bin/env python3
"""Diagnostic: how often the forward's lazy-max slow path fires (needs variants/lib_<tag>.so built
with -DVB_LAZY_COUNT=1). usage: python tools/diag/lazy_count.py TAG"""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vblade  # noqa: E402
from vblade import ops, _lib  # noqa: E402
from bench import realistic_qkv  # noqa: E402
from ab import load  # noqa: E402

lib = load(sys.argv[1])
lib.vb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib._lib = lib
for variant in ("cog", "wan"):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    dev = torch.device("cuda")
    for kind in ("realistic", "randn"):
        with torch.no_grad():
            if kind == "realistic":
                q, k, v = realistic_qkv(H, L, D, 0, dev)
            else:
                q, k, v = (torch.randn(1, H, L, D, device=dev).bfloat16() for _ in range(3))
            rows = m._rows(dev)
            _, mask = m.predict_mask(q, k)
            kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
            buf = (ctypes.c_ulonglong * 16)()
            lib.vb_diag_stamps(buf, 1)
            ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                              kp_log_bias=math.log(m.sample_gap), heavy_rows=m.force_tail)
            lib.vb_diag_stamps(buf, 1)
        print(f"{variant} {kind}: slow paths {buf[10]} of {buf[11]} half-tiles per wave "
              f"({100 * buf[10] / max(1, buf[11]):.2f} %)", flush=True)
