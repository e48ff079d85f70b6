#!/usr/bin/env python3
"""Per-kernel timing of the hot path (HIP events, one process, interleaved reps) for quick A/B
iteration on the GPU box. Not the contract bench (bench.py)."""
import argparse
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
import vblade  # noqa: E402
from vblade import ops  # noqa: E402

sys.path.insert(0, ROOT)
from bench import attn_flops, realistic_qkv  # noqa: E402


def timeit(fn, reps=20):
    s = torch.cuda.current_stream()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def run(variant, density=None):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    over = {} if density is None else dict(min_retain_ratio=density, max_retain_ratio=density)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **over)
    L = m.gilbert_rearranger.seq_len
    dev = torch.device("cuda")
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    rows = m._rows(dev)
    qo = vblade.draw_sample_offsets(1, H, dev)
    ko = vblade.draw_sample_offsets(1, H, dev)
    _, mask = m.predict_mask(q, k, qo, ko)
    kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
    t_pred = timeit(lambda: m.predict_mask(q, k, qo, ko))
    t_pool = timeit(lambda: ops.pool_kv(k, v, m.sample_gap, rows, reordered=True))
    fa = lambda: ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp,  # noqa
                                   vp=vp, kp_log_bias=math.log(m.sample_gap), heavy_rows=m.force_tail)
    t_attn = timeit(fa)
    t_call = timeit(lambda: m(q, k, v), reps=10)
    t_dense = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v), reps=5)
    fl = attn_flops(mask, L, D, kp.shape[2])
    dens = mask.float().mean().item()
    print(f"{variant} density={dens:.3f} pred={t_pred:.3f}ms pool={t_pool:.3f}ms attn={t_attn:.3f}ms "
          f"({fl / t_attn / 1e9:.0f} TF/s) call={t_call:.3f}ms dense_sdpa={t_dense:.3f}ms "
          f"speedup={t_dense / t_call:.2f}x", flush=True)


def run_bwd(variant):
    """Training-path backward: the two-branch forward's saved tensors -> vb_attn_bwd."""
    H, D = (48, 64) if variant == "cog" else (12, 128)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    dev = torch.device("cuda")
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    do = torch.randn_like(q)
    rows = m._rows(dev)
    _, mask = m.predict_mask(q, k)
    gap = m.sample_gap
    kp, vp, k_r, v_r = ops.pool_kv(k, v, gap, rows, reordered=True)
    out1, lse1 = ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True,
                                   heavy_rows=m.force_tail)
    out2, lse2 = ops.attention_fwd(q, None, None, use_main=False, q_rows=rows, kp=kp, vp=vp,
                                   need_lse=True)
    out, alpha = ops.lse_combine(out1, lse1, out2, lse2, gap)
    fb = lambda: ops.attention_bwd(do, q, k_r, v_r, out1, lse1, block_mask=mask, q_rows=rows,  # noqa
                                   kv_rows=rows, kp=kp, vp=vp, out2=out2, lse2=lse2, alpha=alpha,
                                   gap=gap, heavy_rows=m.force_tail)
    t_bwd = timeit(fb, reps=5)
    fl = 2.5 * attn_flops(mask, L, D, kp.shape[2])
    print(f"{variant} bwd density={mask.float().mean().item():.3f} bwd={t_bwd:.3f}ms "
          f"({fl / t_bwd / 1e9:.0f} TF/s at 2.5x fwd FLOPs)", flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="both")
    ap.add_argument("--densities", default="")
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--only-bwd", action="store_true", help="skip the forward timings (PMC passes)")
    a = ap.parse_args()
    with torch.no_grad():
        for var in (["cog", "wan"] if a.variant == "both" else [a.variant]):
            if not a.only_bwd:
                run(var)
            for d in [float(x) for x in a.densities.split(",") if x]:
                run(var, d)
            if a.bwd or a.only_bwd:
                run_bwd(var)
