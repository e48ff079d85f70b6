#!/usr/bin/env python3
"""Diagnostic: the huge-late-score forward case on several library variants; per-row errors vs the
fp64 oracle, with the unscaled and the pre-scaled (bf16(q*scale*log2e)) query."""
import ctypes
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bsa_oracle as O  # noqa: E402
from vblade import _lib, ops  # noqa: E402
from ab import load  # noqa: E402

for D in (64, 128):
    L = 700
    g = torch.Generator().manual_seed(0)
    q, k, v = ((torch.randn(1, 1, L, D, generator=torch.Generator().manual_seed(40 + s))).bfloat16() for s in range(3))
    for qi, ki, mult in ((5, 650, 12.0), (6, 300, 12.0), (7, 690, 14.0), (40, 70, 12.0),
                         (41, 200, 6.0), (130, 10, 20.0)):
        k[0, 0, ki] = q[0, 0, qi] * mult
    ref, _ = O.block_sparse_attention(q, k, v, None)
    c = 1 / math.sqrt(D) * 1.4426950408889634
    qs = (q.float() * c).bfloat16()
    ref2, _ = O.block_sparse_attention(qs, k, v, None, sm_scale=math.log(2))
    print(f"D={D}: |ref - ref_prescaled| max {(ref - ref2).abs().max():.4f}")
    for tag in sys.argv[1:]:
        _lib._lib = load(tag)
        out = ops.attention_fwd(q.cuda(), k.cuda(), v.cuda()).float().cpu()
        e1 = (out - ref).abs().amax(-1)[0, 0]
        e2 = (out - ref2).abs().amax(-1)[0, 0]
        top = torch.topk(e1, 5)
        print(f"  {tag}: max err {e1.max():.4f} (vs prescaled ref {e2.max():.4f}); worst rows "
              f"{top.indices.tolist()} {[round(x, 3) for x in top.values.tolist()]}")
