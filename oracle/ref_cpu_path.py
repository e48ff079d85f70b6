"""TEST INFRASTRUCTURE / CPU BASELINE ONLY — the reference's CPU attention path for BASELINE.json
config 1, and that config's inputs.

Only ``tests/`` and ``bench.py``'s ``cpu_baseline`` leg import this module. The product path is
``libvblade_hip.so``; it never calls into this file.

The reference's only CPU-capable attention is ``F.scaled_dot_product_attention``
(cogvideox/train/special_attentions_local/TrainRelated/blocksparseattn.py:93-94,
cogvideox/sample_evaluate/test_block_sparse_attention.py:98-102). A 128x128 block mask reaches it
as a token-level boolean ``attn_mask`` (True = attend). BASELINE.md §3 fixes the inputs:

* q, k, v ``[1, H, L, D]`` bf16, each N(0, 1) from ``torch.Generator().manual_seed`` 0, 1, 2;
* block mask ``[1, H, nb, nb]`` = ``(torch.rand(seed 3) < 0.5) | eye(nb)``, expanded x128 and
  trimmed to L.

CogVideoX: H=48, L=17776, D=64. Wan2.1: H=12, L=32760, D=128.
"""
from __future__ import annotations

import os
import statistics
import time

import torch

CONFIGS = {
    "cog": dict(H=48, L=17776, D=64, layers=42, frames=49),
    "wan": dict(H=12, L=32760, D=128, layers=30, frames=81),
}
DENOISE_STEPS = 8
BLOCK = 128


def config1_inputs(variant: str = "cog", heads: int | None = None, density: float = 0.5):
    """BASELINE.md §3 step 1. Returns q, k, v (bf16, CPU) and the bool block mask, sliced to the
    first ``heads`` heads (the draws are made at the full head count, so a slice is the same data
    as the first heads of the full call)."""
    c = CONFIGS[variant]
    H, L, D = c["H"], c["L"], c["D"]
    nb = (L + BLOCK - 1) // BLOCK
    q, k, v = (torch.randn(1, H, L, D, generator=torch.Generator().manual_seed(s)).bfloat16()
               for s in range(3))
    r = torch.rand(1, H, nb, nb, generator=torch.Generator().manual_seed(3))
    mask = (r < density) | torch.eye(nb, dtype=torch.bool)
    h = H if heads is None else heads
    return q[:, :h], k[:, :h], v[:, :h], mask[:, :h]


def token_mask(block_mask: torch.Tensor, Lq: int, Lk: int) -> torch.Tensor:
    """[B,H,nbq,nbk] bool -> [B,H,Lq,Lk] bool, each block entry repeated over its 128x128 tile."""
    m = block_mask.repeat_interleave(BLOCK, 2).repeat_interleave(BLOCK, 3)
    return m[:, :, :Lq, :Lk]


def masked_sdpa(q, k, v, block_mask, heads_per_call: int = 2):
    """The reference CPU path: F.scaled_dot_product_attention(q, k, v, attn_mask=token_mask),
    run ``heads_per_call`` heads at a time so the token mask stays a few GB."""
    outs = []
    for h0 in range(0, q.shape[1], heads_per_call):
        sl = slice(h0, h0 + heads_per_call)
        tm = token_mask(block_mask[:, sl], q.shape[2], k.shape[2])
        outs.append(torch.nn.functional.scaled_dot_product_attention(q[:, sl], k[:, sl], v[:, sl],
                                                                     attn_mask=tm))
    return torch.cat(outs, 1)


def host_threads() -> int:
    """Host cores this process may use: os.cpu_count(), capped by a cgroup CPU quota (the GPU box
    shows every CPU of the machine but grants a share of them)."""
    n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def time_cpu_sdpa(variant: str = "cog", heads: int = 4, threads: int | None = None,
                  reps: int = 3) -> dict:
    """BASELINE.md §3 step 2-4 on a head slice: 1 warm-up + median of ``reps`` of the masked and
    the dense SDPA call, scaled to all heads, and the attention-only frames/s of a whole video
    (frames / (t_call * layers * 8 steps))."""
    c = CONFIGS[variant]
    threads = threads or host_threads()
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        q, k, v, bm = config1_inputs(variant, heads)
        tm = token_mask(bm, q.shape[2], k.shape[2])   # built once, outside the timed calls

        def med(fn):
            fn()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            return statistics.median(ts)

        sdpa = torch.nn.functional.scaled_dot_product_attention
        t_mask = med(lambda: sdpa(q, k, v, attn_mask=tm))
        t_dense = med(lambda: sdpa(q, k, v))
    finally:
        torch.set_num_threads(old)
    scale = c["H"] / heads
    calls = DENOISE_STEPS * c["layers"]
    tm_call, td_call = t_mask * scale, t_dense * scale
    return {
        "masked_s_per_call": tm_call, "dense_s_per_call": td_call,
        "masked_frames_per_s": c["frames"] / (tm_call * calls),
        "dense_frames_per_s": c["frames"] / (td_call * calls),
        "threads": threads, "heads_timed": heads, "heads": c["H"], "reps": reps,
        "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
    }
