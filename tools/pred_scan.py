#!/usr/bin/env python3
"""Diagnostic: predictor time vs number of heads (wave quantization of its grid)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from vblade import ops  # noqa: E402
from bench import realistic_qkv  # noqa: E402

dev = torch.device("cuda")
m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0)
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(48, L, 64, 0, dev)
rows = m._rows(dev)
for H in [8, 16, 21, 22, 24, 32, 40, 43, 44, 48]:
    qh, kh = q[:, :H], k[:, :H]
    qo = vblade.draw_sample_offsets(1, H, dev)
    ko = vblade.draw_sample_offsets(1, H, dev)
    f = lambda: ops.mask_predict(qh, kh, qo, ko, rows=rows, energy_threshold=0.95, min_keep=6,  # noqa
                                 max_keep=13, force_tail=2)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20
    print(f"H={H:2d} WGs={35 * H:5d} {t:.4f} ms  {t / H * 1000:.2f} us/head", flush=True)
