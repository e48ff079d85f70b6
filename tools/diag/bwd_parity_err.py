#!/usr/bin/env python3
"""Relative Frobenius errors of the default backward kernels (vb_attn_bwd: the pipeline dK/dV and
the 2-slot dQ) against the oracle's fp64 backward, per gradient, at several shapes and through the
two-branch module: the numbers behind tests/test_gpu_backward.py's tight bound."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bsa_oracle as O  # noqa: E402
import test_gpu_backward as T  # noqa: E402
from vblade import ops  # noqa: E402

DEV = "cuda"
for L, D, dtype, dens in [(1000, 64, torch.bfloat16, 0.25), (1000, 128, torch.bfloat16, 0.25),
                          (517, 64, torch.float16, 0.3), (700, 128, torch.float16, 0.4),
                          (300, 64, torch.bfloat16, 0.5), (260, 128, torch.bfloat16, 0.6)]:
    q, k, v, do = (T._rand(1, 2, L, D, dtype=dtype, seed=s) for s in range(4))
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(1, 2, nb, nb, dens, seed=7)
    out, lse = ops.attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV), need_lse=True)
    dq, dk, dv = ops.attention_bwd(do.to(DEV), q.to(DEV), k.to(DEV), v.to(DEV), out, lse, block_mask=mask.to(DEV))
    rq, rk, rv = O.block_sparse_attention_bwd(q, k, v, out.cpu(), lse.cpu(), do, mask)
    print(f"op L={L} D={D} {str(dtype)[6:]} density={dens}: dq {T.rel(dq, rq):.2e} dk {T.rel(dk, rk):.2e} dv {T.rel(dv, rv):.2e}", flush=True)
for variant, D in (("cog", 64), ("wan", 128)):
    m, cfg = T._small_module(variant)
    L = m.gilbert_rearranger.seq_len
    q, k, v, do = T._realistic(1, 2, L, D, seed=3)
    qd, kd, vd = (t.to(DEV).requires_grad_(True) for t in (q, k, v))
    o = m(qd, kd, vd)
    o.backward(do.to(DEV))
    fwd = O.adaptive_attention(q, k, v, cfg, None, None, mask=m.last_mask.bool().cpu())
    rq, rk, rv = O.adaptive_attention_bwd(q, k, v, do, cfg, fwd)
    print(f"module {variant} L={L} D={D}: out {T.rel(o.detach().float(), fwd['out']):.2e} dq {T.rel(qd.grad, rq):.2e} "
          f"dk {T.rel(kd.grad, rk):.2e} dv {T.rel(vd.grad, rv):.2e}", flush=True)
