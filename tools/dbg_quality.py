#!/usr/bin/env python3
"""Output quality of library variants on the bench's realistic inputs (full sequence length, a
subset of heads): PSNR and max|err| of the fused inference module vs the oracle's reference
combine, on one shared mask. usage: python tools/dbg_quality.py TAG [TAG ...]"""
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("video-blade_amd", "oracle", "tools", ""):
    sys.path.insert(0, os.path.join(ROOT, p))
import bsa_oracle as O  # noqa: E402
import vblade  # noqa: E402
from vblade import _lib  # noqa: E402
from ab import load  # noqa: E402
from bench import realistic_qkv  # noqa: E402


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    return 99.0 if mse == 0 else 10 * math.log10(ref.double().abs().max().item() ** 2 / mse)


for variant, H, D in (("cog", 2, 64), ("wan", 1, 128)):
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    q, k, v = realistic_qkv(H, L, D, 0, torch.device("cuda"))
    with torch.no_grad():
        m(q, k, v)
    mask = m.last_mask
    cfg = O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan()
    ref = O.adaptive_attention(q.cpu(), k.cpu(), v.cpu(), cfg, None, None, mask=mask.bool().cpu(),
                               store_dtype=torch.bfloat16)["out"]
    for tag in sys.argv[1:]:
        _lib._lib = load(tag)
        with torch.no_grad():
            out = m(q, k, v, block_mask=mask).float().cpu()
        print(f"{variant} {tag}: PSNR {psnr(out, ref):.2f} dB, max|err| {(out - ref).abs().max():.4f}, "
              f"mean|err| {(out - ref).abs().mean():.2e}", flush=True)
