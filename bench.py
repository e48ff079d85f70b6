#!/usr/bin/env python3
"""Benchmark of the Video-BLADE hot path on MI355X: adaptive block-sparse attention.

Metric (BASELINE.json): frames/sec/GPU for CogVideoX-5B 8-step 49x720x480 bf16 (+ attention
TFLOPS vs dense). One bench STEP = the attention work of one 8-step video = 8 denoising steps x
42 transformer blocks = 336 calls of ``inner_attention(q, k, v)`` on q,k,v [1,48,17776,64] bf16
(Wan2.1-1.3B with --variant wan: 8 x 30 calls on [1,12,32760,128], 81 frames). Each call runs the
whole hot path: Gilbert-order mask prediction, pooled K/V, fused block-sparse + pooled attention,
scatter back to token order. Inputs are synthetic (no weights/datasets offline): N_SETS distinct
random q/k/v sets with the block-structured "realistic" distribution, resident in
HBM before the timed region, cycled across calls.

Attention-only frames/s = frames / (time of 8 x layers calls). The transformer's GEMMs, VAE and
scheduler are not in the hot path and are not timed.

N GPUs: one process per GPU (torchrun), each rank renders its own videos (prompt-batch replicas,
no data-path collective) — barrier + synchronize around the timed region, time = max
over ranks, value = all ranks' frames / time ("scaling": "weak").
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))

VARIANTS = {
    "cog": dict(H=48, D=64, layers=42, frames=49, name="CogVideoX-5B 8-step 49x720x480 bf16",
                video="13x30x45 latent tokens + 226 text"),
    "wan": dict(H=12, D=128, layers=30, frames=81, name="Wan2.1-1.3B 8-step 81x832x480 bf16",
                video="21x30x52 latent tokens"),
}
DENOISE_STEPS = 8
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--variant", choices=list(VARIANTS), default="cog")
    ap.add_argument("--density", type=float, default=None,
                    help="fixed block density (min=max retain) instead of the energy rule")
    ap.add_argument("--sets", type=int, default=3, help="distinct resident q/k/v sets")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    return ap.parse_args()


def realistic_qkv(H, L, D, seed, device):
    g = torch.Generator(device=device).manual_seed(seed)
    cent = torch.randn(1, H, L // 128 + 1, D, generator=g, device=device)
    cent = cent.repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(1, H, L, D, generator=g, device=device) + 2 * cent).bfloat16()
    k = (torch.randn(1, H, L, D, generator=g, device=device) + 2 * cent).bfloat16()
    v = torch.randn(1, H, L, D, generator=g, device=device).bfloat16()
    return q, k, v


def attn_flops(mask: torch.Tensor, L: int, D: int, Lkp: int) -> float:
    """Algorithmic FLOPs of one fused attention launch: sum over kept (i,j) blocks of
    4*m_i*n_j*D (true block sizes, tail included) + pooled branch 4*L*Lkp*D, per head."""
    nb = mask.shape[-1]
    sizes = torch.full((nb,), 128.0, device=mask.device)
    sizes[-1] = L - 128 * (nb - 1)
    m = mask.float()
    pairs = (sizes[:, None] * sizes[None, :] * m).sum().item()
    heads = mask.shape[0] * mask.shape[1]
    return 4.0 * D * pairs + 4.0 * heads * L * Lkp * D


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    import vblade
    from vblade import ops

    V = VARIANTS[args.variant]
    H, D, layers, frames = V["H"], V["D"], V["layers"], V["frames"]
    over = {}
    if args.density is not None:
        over = dict(min_retain_ratio=args.density, max_retain_ratio=args.density)
    mod = vblade.AdaptiveBlockSparseAttn(args.variant, log_every=0, **over)
    L = mod.gilbert_rearranger.seq_len
    calls = DENOISE_STEPS * layers
    sets = [realistic_qkv(H, L, D, 1000 * rank + s, dev) for s in range(args.sets)]
    torch.manual_seed(1234 + rank)

    def one_video():
        for c in range(calls):
            q, k, v = sets[c % len(sets)]
            mod(q, k, v)

    with torch.no_grad():
        for _ in range(args.warmup):
            one_video()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_video()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = 1000.0 * elapsed / args.steps
    ms_per_call = ms_per_step / calls
    value = world * frames * args.steps / elapsed
    sparsity = mod.sparsity

    result = {
        "metric": "frames/sec/GPU, " + V["name"] + " (attention path); attn TFLOPS vs dense",
        "value": round(value, 4),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic block-structured q/k/v (SURVEY §8d realistic option), "
                f"{args.sets} resident sets",
        "config": {
            "workload": f"{V['name']}: {calls} inner_attention calls per video "
                        f"(8 steps x {layers} blocks), q/k/v [1,{H},{L},{D}] ({V['video']})",
            "global_batch": world,
            "seq_len": L,
            "heads": H,
            "head_dim": D,
            "calls_per_step": calls,
            "mask": "energy rule (reference defaults)" if args.density is None
                    else f"fixed density {args.density}",
            "parallelism": f"replicas x{world} (prompt-batch DP, no collective)",
        },
        "ms_per_call": round(ms_per_call, 4),
        "mean_sparsity": round(sparsity, 4),
    }

    if rank == 0:
        with torch.no_grad():
            extra = measure_kernels(mod, sets, L, H, D, dev, ops, args)
        result.update(extra["top"])
        dense_ms = extra.get("dense_ms")
        if dense_ms:
            result["dense_sdpa_ms_per_call"] = round(dense_ms, 4)
            result["speedup_vs_dense_sdpa"] = round(dense_ms / ms_per_call, 3)
            dense_flops = 4.0 * H * L * L * D
            result["attn_tflops_dense_equiv"] = round(dense_flops / (ms_per_call * 1e-3) / 1e12, 2)
        if not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(args.variant, calls, frames)
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def measure_kernels(mod, sets, L, H, D, dev, ops, args):
    """Average duration of the dominant kernel (attn_fwd_kernel) with HIP events on the stream
    it runs on, its algorithmic FLOPs, and dense SDPA on the same shapes for the ratio."""
    stream = torch.cuda.current_stream(dev)
    rows = mod._rows(dev)
    recs = []
    for s, (q, k, v) in enumerate(sets):
        _, mask = mod.predict_mask(q, k)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, mod.sample_gap, rows, reordered=True)
        recs.append((q, k_r, v_r, mask, kp, vp))
    n_rep = 10
    flops = 0.0
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(n_rep * len(recs))]
    i = 0
    for _ in range(2):   # warm
        for q, k, v, mask, kp, vp in recs:
            ops.attention_fwd(q, k, v, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                              kp_log_bias=math.log(mod.sample_gap), heavy_rows=mod.force_tail)
    for _ in range(n_rep):
        for q, k, v, mask, kp, vp in recs:
            a, b = ev[i]
            a.record(stream)
            ops.attention_fwd(q, k, v, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                              kp_log_bias=math.log(mod.sample_gap), heavy_rows=mod.force_tail)
            b.record(stream)
            flops += attn_flops(mask, L, D, kp.shape[2])
            i += 1
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    flops /= len(ev)
    achieved = flops / (ms * 1e-3) / 1e12
    # compulsory HBM bytes of one launch: Q, O once; K/V of kept blocks (upper bound: all of K,V
    # once), pooled K/V, mask (for the roofline's traffic cross-check)
    top = {
        "roofline": {
            "bound": "mfma",
            "kernel": "attn_fwd_kernel",
            "achieved": round(achieved, 2),
            "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
            "traffic": None,
            "avg_launch_ms": round(ms, 4),
            "flops_per_launch": flops,
        }
    }
    out = {"top": top}
    if not args.no_dense:
        q, k, v = sets[0]
        for _ in range(2):
            torch.nn.functional.scaled_dot_product_attention(q, k, v)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(5):
            torch.nn.functional.scaled_dot_product_attention(q, k, v)
        b.record(stream)
        torch.cuda.synchronize()
        out["dense_ms"] = a.elapsed_time(b) / 5
    return out


def cpu_baseline(variant, calls, frames):
    """The oracle (CPU restatement of the whole adaptive path, oracle/bsa_oracle.py) timed on
    this host's cores on a bounded sample: 2 heads of one attention call at the full sequence
    length, scaled to a whole video's calls. Baseline only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bsa_oracle as O
    cfg = O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan()
    V = VARIANTS[variant]
    heads = 2
    L = cfg.width * cfg.height * cfg.depth + cfg.text_length
    g = torch.Generator().manual_seed(0)
    cent = torch.randn(1, heads, L // 128 + 1, V["D"], generator=g).repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    k = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    v = torch.randn(1, heads, L, V["D"], generator=g).bfloat16()
    qo = O.draw_sample_offsets(1, heads, generator=g)
    ko = O.draw_sample_offsets(1, heads, generator=g)
    threads = torch.get_num_threads()
    orig = O.block_sparse_attention

    def fp32_attn(*a, **kw):
        kw.setdefault("acc_dtype", torch.float32)
        return orig(*a, **kw)

    O.block_sparse_attention = fp32_attn
    try:
        t0 = time.perf_counter()
        O.adaptive_attention(q, k, v, cfg, qo, ko, store_dtype=torch.bfloat16)
        dt = time.perf_counter() - t0
    finally:
        O.block_sparse_attention = orig
    t_call = dt * V["H"] / heads
    return {"value": round(frames / (calls * t_call), 6), "unit": "frames/s",
            "cores": threads, "kind": "port",
            "sample": f"oracle adaptive path (fp32 torch CPU), {heads} of {V['H']} heads of one "
                      f"[1,{V['H']},{L},{V['D']}] call: {dt:.2f} s; scaled x{V['H'] // heads} heads "
                      f"x {calls} calls per video"}


if __name__ == "__main__":
    main()
