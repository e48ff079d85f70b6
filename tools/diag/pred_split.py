#!/usr/bin/env python3
"""Diagnostic: predictor time split (VB_DIAG build: VB_DEBUG_PRED=1 skips the epilogue, 2 the K loop)."""
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

_lib._lib = ab.load(sys.argv[1] if len(sys.argv) > 1 else "pdiag")
dev = torch.device("cuda")
for variant in ("cog", "wan"):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    qo = vblade.draw_sample_offsets(1, H, dev)
    ko = vblade.draw_sample_offsets(1, H, dev)
    for dbg in (sys.argv[2].split(",") if len(sys.argv) > 2 else ("0", "1", "2", "3", "5")):
        os.environ["VB_DEBUG_PRED"] = dbg
        for _ in range(3):
            m.predict_mask(q, k, qo, ko)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            m.predict_mask(q, k, qo, ko)
        e1.record()
        torch.cuda.synchronize()
        print(f"{variant} dbg={dbg} {e0.elapsed_time(e1) / 20:.4f} ms", flush=True)
