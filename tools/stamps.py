#!/usr/bin/env python3
"""Diagnostic: per-segment cycle shares of the attention loop (needs libvblade_hip_diag.so)."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["VBLADE_LIB"] = os.path.join(ROOT, "video-blade_amd/vblade/libvblade_hip_diag.so")
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from vblade import ops, _lib  # noqa: E402
from bench import realistic_qkv  # noqa: E402

lib = _lib.load()
lib.vb_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
for variant in ("cog", "wan"):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    dev = torch.device("cuda")
    with torch.no_grad():
        q, k, v = realistic_qkv(H, L, D, 0, dev)
        rows = m._rows(dev)
        _, mask = m.predict_mask(q, k)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
        buf = (ctypes.c_ulonglong * 16)()
        ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                          kp_log_bias=math.log(m.sample_gap), heavy_rows=m.force_tail)
        lib.vb_diag_stamps(buf, 1)
        for _ in range(3):
            ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                              kp_log_bias=math.log(m.sample_gap), heavy_rows=m.force_tail)
        lib.vb_diag_stamps(buf, 1)
    names = ["wait+barrier", "dma issue", "tile total", "softmax", "PV"]
    tiles = buf[8]
    tot = sum(buf[i] for i in range(3))
    print(variant, "tiles", tiles, {n: f"{buf[i] / max(1, tiles) :.0f} cyc/tile ({100 * buf[i] / tot:.1f}%)" for i, n in enumerate(names)})
