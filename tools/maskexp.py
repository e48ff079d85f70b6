#!/usr/bin/env python3
"""Attention-kernel time vs mask structure at equal density (diagnostic)."""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vblade  # noqa: E402
from vblade import ops  # noqa: E402
from bench import attn_flops, realistic_qkv  # noqa: E402
from kbench import timeit  # noqa: E402

H, D = 48, 64
m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0)
L = m.gilbert_rearranger.seq_len
dev = torch.device("cuda")
with torch.no_grad():
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    rows = m._rows(dev)
    _, real = m.predict_mask(q, k)
    kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
    nb = real.shape[-1]
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = (torch.rand(1, H, nb, nb, generator=g, device=dev) < 0.105)
    idx = torch.arange(nb, device=dev)
    band = ((idx[:, None] - idx[None, :]).abs() <= 6)[None, None].expand(1, H, nb, nb)
    def forced(mk):
        mk = mk.clone()
        mk[..., -2:] = True
        mk[..., -2:, :] = True
        return mk.to(torch.uint8)
    cases = {"real": real, "random+tail": forced(rnd), "band+tail": forced(band),
             "random": rnd.to(torch.uint8), "band": band.to(torch.uint8).contiguous()}
    for name, mk in cases.items():
        for pooled in (True, False):
            f = lambda: ops.attention_fwd(q, k, v, block_mask=mk, q_rows=rows, kv_rows=rows,  # noqa
                                          kp=kp if pooled else None, vp=vp if pooled else None,
                                          kp_log_bias=math.log(15))
            t = timeit(f)
            fl = attn_flops(mk, L, D, kp.shape[2] if pooled else 0)
            print(f"{name:12s} pooled={pooled} density={mk.float().mean().item():.3f} {t:.3f} ms "
                  f"{fl / t / 1e9:.0f} TF/s", flush=True)
    # no row gather (identity), same real mask
    f = lambda: ops.attention_fwd(q, k, v, block_mask=real, kp=kp, vp=vp, kp_log_bias=math.log(15))  # noqa
    t = timeit(f)
    print(f"real, no Gilbert gather: {t:.3f} ms {attn_flops(real, L, D, kp.shape[2]) / t / 1e9:.0f} TF/s")
