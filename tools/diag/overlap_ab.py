#!/usr/bin/env python3
"""A/B of a boolean module option in one process (default: overlap; --opt gather_kv)."""
import os
import statistics
import sys

import torch

OPT = sys.argv[sys.argv.index('--opt') + 1] if '--opt' in sys.argv else 'overlap'

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from bench import realistic_qkv  # noqa: E402

dev = torch.device("cuda")
for variant in ("cog", "wan"):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    mods = {ov: vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **{OPT: ov}) for ov in (True, False)}
    L = mods[True].gilbert_rearranger.seq_len
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    times = {True: [], False: []}
    with torch.no_grad():
        for ov, m in mods.items():
            for _ in range(3):
                m(q, k, v)
        torch.cuda.synchronize()
        for _ in range(15):
            for ov, m in mods.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    m(q, k, v)
                e1.record()
                torch.cuda.synchronize()
                times[ov].append(e0.elapsed_time(e1) / 10)
    for ov in (True, False):
        print(f"{variant} {OPT}={ov}: median {statistics.median(times[ov]):.4f} ms/call", flush=True)
