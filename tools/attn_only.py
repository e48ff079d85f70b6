#!/usr/bin/env python3
"""Run only the fused attention kernel (and optionally the predictor) N times on CogVideoX / Wan
shapes — a target for rocprofv3 counter collection.
usage: attn_only.py [cog|wan|cog-ml] [N] [attn|pred|all] [density (fixed kept fraction; default:
the energy rule)] [band]
"band": the predicted mask replaced by a diagonal band with the same kept count per row (plus the
forced tail rows/columns) — a mask whose neighbouring q-blocks share key blocks, as the synthetic
random-centre inputs' masks do not (the L2-locality control for the traffic counters).
"local": the locality-faithful inputs (bench.local_qkv: centres a smooth function of the latent
x, y, t) and the energy rule's mask on them."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from vblade import ops  # noqa: E402
from bench import local_qkv, realistic_qkv  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "cog"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
what = sys.argv[3] if len(sys.argv) > 3 else "attn"
H, D = (12, 128) if variant == "wan" else (48, 64)
if variant == "cog-ml":   # the multi-level sampler path
    from vblade import multilevel
    m = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0)
    L = m.gilbert_rearranger.seq_len
    dev = torch.device("cuda")
    with torch.no_grad():
        q, k, v = realistic_qkv(H, L, D, 0, dev)
        rows = m._rows(dev)
        _, mask = multilevel.predict_level_mask(q, k, rows=rows)
        kp, vp = ops.kv_pyramid(k, v, rows)
        for _ in range(n):
            ops.ml_attention_fwd(q, kp, vp, mask, q_rows=rows, heavy_rows=2)
        torch.cuda.synchronize()
    print("done")
    sys.exit(0)
density = float(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] != "none" else None
over = {} if density is None else dict(min_retain_ratio=density, max_retain_ratio=density)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **over)
L = m.gilbert_rearranger.seq_len
dev = torch.device("cuda")
local = len(sys.argv) > 5 and sys.argv[5] == "local"
with torch.no_grad():
    q, k, v = local_qkv(variant, H, D, 0, dev) if local else realistic_qkv(H, L, D, 0, dev)
    rows = m._rows(dev)
    qo = vblade.draw_sample_offsets(1, H, dev)
    ko = vblade.draw_sample_offsets(1, H, dev)
    _, mask = m.predict_mask(q, k, qo, ko)
    if len(sys.argv) > 5 and sys.argv[5] == "band":
        nb, ft = mask.shape[-1], m.force_tail
        kk = int(round(mask[..., : nb - ft, :].float().sum(-1).mean().item()))
        i = torch.arange(nb, device=dev).view(nb, 1)
        j = torch.arange(nb, device=dev).view(1, nb)
        lo = (i - kk // 2).clamp(0, nb - kk)
        band = ((j >= lo) & (j < lo + kk)) | (j >= nb - ft) | (i >= nb - ft)
        mask = band.to(mask.dtype).expand_as(mask).contiguous()
        print(f"band mask: {kk} of {nb} blocks per row")
    kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
    # the module's K/V source (gather_kv="auto": gathered rows at D=128, Gilbert copies at D=64),
    # dispatch order and persistent launch, so the counters describe the kernel bench.py times
    gather = m._gather(D)
    k_src, v_src, kv_rows = (k, v, rows) if gather else (k_r, v_r, None)
    for _ in range(n):
        if what in ("attn", "all"):
            ops.attention_fwd(q, k_src, v_src, block_mask=mask, q_rows=rows, kv_rows=kv_rows, kp=kp,
                              vp=vp, kp_log_bias=m._log_gap(q.dtype), heavy_rows=m.force_tail,
                              order=m.order, order_window=m.order_window, persistent=m.persistent)
        if what in ("pred", "all"):
            m.predict_mask(q, k, qo, ko)
    torch.cuda.synchronize()
print("done")
