#!/usr/bin/env python3
"""Where the gathered-K/V attention kernel's extra time goes (CogVideoX/Wan, the module's mask):
the same attention launch on (a) Gilbert-ordered copies (contiguous tiles), (b) the copies through
an identity row table (the gather code path, contiguous memory), (c) the caller's k/v through the
Gilbert row table (the gather code path, scattered rows). (b) - (a) is the code path's cost,
(c) - (b) the memory pattern's. usage: python tools/diag/gather_cost.py [cog|wan]"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from vblade import ops  # noqa: E402
from bench import realistic_qkv  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "cog"
dev = torch.device("cuda")
H, D = (48, 64) if variant == "cog" else (12, 128)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, gather_kv=False)
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(H, L, D, 0, dev)
with torch.no_grad():
    m(q, k, v)
    mask = m.last_mask
    rows = m._rows(dev)
    kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
    ident = torch.arange(L, device=dev, dtype=torch.int32)
    bias = m._log_gap(q.dtype)
    modes = {
        "copies": (k_r, v_r, None),
        "copies+identity rows": (k_r, v_r, ident),
        "caller k/v+Gilbert rows": (k, v, rows),
    }
    outs = {}
    times = {n: [] for n in modes}
    for n, (ks, vs, kr) in modes.items():
        outs[n] = ops.attention_fwd(q, ks, vs, block_mask=mask, q_rows=rows, kv_rows=kr, kp=kp, vp=vp,
                                    kp_log_bias=bias, heavy_rows=m.force_tail)
    same = all(torch.equal(outs["copies"], o) for o in outs.values())
    torch.cuda.synchronize()
    for _ in range(15):
        for n, (ks, vs, kr) in modes.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                ops.attention_fwd(q, ks, vs, block_mask=mask, q_rows=rows, kv_rows=kr, kp=kp, vp=vp,
                                  kp_log_bias=bias, heavy_rows=m.force_tail)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 10)
print(f"{variant}: outputs identical across modes: {same}")
base = statistics.median(times["copies"])
for n in modes:
    t = statistics.median(times[n])
    print(f"{variant} attn {n:26s} median {t:.4f} ms  x{base / t:.3f} vs copies", flush=True)
