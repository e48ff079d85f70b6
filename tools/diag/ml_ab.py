#!/usr/bin/env python3
"""A/B of the multi-level module's pyramid placement in one process: overlap=True (the pyramid
pass as extra workgroups of the predictor's launch) vs overlap=False (its own launch after it)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
from vblade import multilevel  # noqa: E402
from bench import realistic_qkv  # noqa: E402

dev = torch.device("cuda")
mods = {ov: multilevel.AdaptiveBlockSparseAttnTrain(log_every=0, overlap=ov) for ov in (True, False)}
q, k, v = realistic_qkv(48, 17776, 64, 0, dev)
times = {True: [], False: []}
with torch.no_grad():
    for m in mods.values():
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
    print(f"cog-ml pyramid in predictor launch={ov}: median {statistics.median(times[ov]):.4f} ms/call",
          flush=True)
