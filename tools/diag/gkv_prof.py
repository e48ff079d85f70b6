#!/usr/bin/env python3
"""rocprofv3 target: 20 CogVideoX module calls with gather_kv=False (Gilbert copies), then 20 with
gather_kv=True (K/V rows gathered by the attention kernel; no copies in the pooled pass)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from bench import realistic_qkv  # noqa: E402

dev = torch.device("cuda")
q, k, v = realistic_qkv(48, 17776, 64, 0, dev)
with torch.no_grad():
    for gk in (False, True):
        m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0, gather_kv=gk)
        for _ in range(20):
            m(q, k, v)
        torch.cuda.synchronize()
print("done")
