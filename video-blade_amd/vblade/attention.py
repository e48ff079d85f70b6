"""Adaptive block-sparse attention module — the ``attn.inner_attention(q, k, v)`` surface.

Mirrors ``AdaptiveBlockSparseAttnTrain`` (cogvideox/train/special_attentions_local/TrainRelated/
cogvideo_blocksparseattn.py:398-427; wanx_blocksparseattn.py:375-409) and its helpers
(``adaptive_block_sparse_attn`` :327-394, ``GilbertRearranger`` :110-161,
``transfer_attn_to_mask`` :177-249, ``simple_pooling`` :83-88), with the module-level globals
(:9-16) as constructor arguments. Every tensor op of the hot path runs in libvblade_hip.so:

  forward (inference, the 8-step samplers):
    1. vb_mask_predict  — sampled pooled scores + energy top-k -> block mask (Gilbert order); the
                          pooled K/V pass (mean over `sample_gap` reordered tokens) runs in the
                          same launch as extra workgroups (one stream, no events)
    2. vb_attn_fwd      — ONE softmax over kept full-res keys ∪ pooled keys (+ln gap bias):
                          the reference's two attention calls + LSE combine, fused; q/k/v rows
                          gathered and out rows scattered through the Gilbert index (no copies)
  training (grad required) keeps the reference's two-branch structure so the backward has the
  reference's semantics (LSE/alpha detached): see ``autograd.adaptive_split_attention``.

Only the tiny RNG draw of the sampling offsets (torch.rand + topk over [B,H,1,128], exactly as
cogvideo_blocksparseattn.py:45-46 so the RNG stream matches the reference) stays in PyTorch.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import ops

VARIANT_DEFAULTS = {
    # cogvideo_blocksparseattn.py:9-16
    "cog": dict(use_rearrange=True, max_retain_ratio=0.1, min_retain_ratio=0.05, width=45,
                height=30, depth=13, sample_gap=15, text_length=226, force_tail=2, log_every=800),
    # wanx_blocksparseattn.py:9-16 (+ no forced rows/cols, print every 200 calls :400)
    "wan": dict(use_rearrange=True, max_retain_ratio=0.17, min_retain_ratio=0.05, width=52,
                height=30, depth=21, sample_gap=30, text_length=0, force_tail=0, log_every=200),
}


# longest-first dispatch of the attention launch (one small ordering launch before it), per
# variant. Measured (tools/ab.py, round 5, profiles/archive/r05_attn_order_ab.log): Wan 1.047-1.054x per
# attention launch; CogVideoX 0.98x over the whole range and 0.976-0.989x with only the last
# 64-256 q-blocks of each XCD range re-ordered (its q-blocks differ little in length, and the
# Gilbert-neighbour order's L2 reuse and the extra launch cost more than the tail)
ORDER_DEFAULT = {"cog": False, "wan": True}

# persistent attention launch (resident-sized grid, per-XCD work queues; ops.attention_fwd
# persistent=True), per variant. Measured (tools/ab.py, profiles/r06_persist_*_ab.log): the
# CogVideoX attention launch alone 1.005-1.009x, but the whole call 0.99-1.00x (r06_persist_call_ab.log);
# Wan's inference launch (gathered K/V) 0.98x per call. Off for both; the training path's D=128 LSE
# launch runs persistent (autograd.py, 1.024-1.030x).
PERSISTENT_DEFAULT = {"cog": False, "wan": False}


def retain_counts(nb: int, min_ratio: float, max_ratio: float, variant: str):
    """Kept-block clamp bounds. cog: (seq * fp32 ratio tensor).to(int) clamped >= 1
    (cogvideo_blocksparseattn.py:230-231, 347-348); wan: max(1, int(seq * ratio)) (wanx :215-216)."""
    if variant == "cog":
        lo = int(np.float32(nb) * np.float32(min_ratio))
        hi = int(np.float32(nb) * np.float32(max_ratio))
    else:
        lo, hi = int(nb * min_ratio), int(nb * max_ratio)
    return max(1, lo), max(1, hi)


def draw_sample_offsets(B: int, H: int, device, block: int = 128, num_keep: int = 32,
                        generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """rand(B,H,1,block) -> topk(num_keep) offsets, shared by all blocks of a (b,h)
    (random_sample_tokens, cogvideo_blocksparseattn.py:45-46). int32 [B,H,num_keep]."""
    r = torch.rand(B, H, 1, block, device=device, generator=generator)
    return torch.topk(r, num_keep, dim=3).indices[:, :, 0, :].to(torch.int32)


def draw_sample_offsets_qk(B: int, H: int, device, block: int = 128, num_keep: int = 32,
                           generator: Optional[torch.Generator] = None):
    """The q and k draws of efficient_attn_with_pooling (:77-78): two torch.rand calls in the
    reference's order (the same RNG stream), the two topk selections in one HIP launch
    (vb_sample_offsets; same indices as torch.topk for distinct values)."""
    rq = torch.rand(B, H, 1, block, device=device, generator=generator)
    rk = torch.rand(B, H, 1, block, device=device, generator=generator)
    q_off, k_off = ops.sample_offsets(rq, rk, num_keep)
    return q_off[:, :, 0, :], k_off[:, :, 0, :]


class GilbertRearranger(nn.Module):
    """Index maps of the Gilbert reorder (cogvideo_blocksparseattn.py:110-161; wanx :102-159).

    ``rows[g]`` = caller row holding reordered position g. The attention kernels consume
    ``rows`` directly; ``rearrange``/``reversed_rearrange`` are provided for API parity and
    debugging (they materialise copies the fused path never makes)."""

    def __init__(self, width: int, height: int, depth: int, text_length: int = 0):
        super().__init__()
        self.width, self.height, self.depth, self.text_length = width, height, depth, text_length
        perm = ops.gilbert_perm(width, height, depth).astype(np.int64)
        inv = np.empty_like(perm)
        inv[perm] = np.arange(perm.size)
        self.register_buffer("original_order2gilbert_order", torch.from_numpy(perm), persistent=False)
        self.register_buffer("gilbert_order2original_order", torch.from_numpy(inv), persistent=False)
        rows = np.concatenate([perm + text_length, np.arange(text_length)]).astype(np.int32)
        self.register_buffer("rows", torch.from_numpy(rows), persistent=False)

    @property
    def seq_len(self) -> int:
        return self.width * self.height * self.depth + self.text_length

    def rearrange(self, q, k, v):
        r = self.rows.to(q.device).long()
        return q[..., r, :], k[..., r, :], v[..., r, :]

    def reversed_rearrange(self, out):
        r = self.rows.to(out.device).long()
        res = torch.empty_like(out)
        res[..., r, :] = out
        return res


class AdaptiveBlockSparseAttn(nn.Module):
    """``inner_attention(q, k, v) -> out`` with q,k,v,out [B,H,L,D] bf16/fp16 on a HIP device.

    variant: "cog" (CogVideoX-5B: text tail, forced last 2 block rows/cols) or "wan"
    (Wan2.1-1.3B). Keyword arguments override the reference's module globals.
    combine: "fused" (one softmax, inference default) or "reference" (two attention calls + the
    reference's bf16 LSE combine, bit-for-bit structure of :366-393; always used under autograd).
    mask_head_mode: how the reference's head_mask_type = ones(H) (:313) reads the predicted
    [B,H,nb,nb] mask, which SURVEY Appendix B leaves open offline: "per_head" (default: each head
    its own predicted mask, Block-Sparse-Attention's renumbering of the ones) or "shared_head0"
    (every head attends with head 0's mask). The sparsity statistic counts the predicted mask in
    both modes, as the reference's (:394) does.
    """

    def __init__(self, variant: str = "cog", *, combine: str = "fused", **overrides):
        super().__init__()
        if variant not in VARIANT_DEFAULTS:
            raise ValueError(f"variant must be one of {list(VARIANT_DEFAULTS)}")
        cfg = dict(VARIANT_DEFAULTS[variant])
        unknown = set(overrides) - set(cfg) - {"energy_threshold", "block", "num_keep", "overlap", "gather_kv",
                                               "mask_head_mode", "order", "order_window", "persistent"}
        if unknown:
            raise TypeError(f"unknown options {sorted(unknown)}")
        cfg.update(overrides)
        self.variant = variant
        self.combine = combine
        self.use_rearrange = cfg["use_rearrange"]
        self.max_retain_ratio = cfg["max_retain_ratio"]
        self.min_retain_ratio = cfg["min_retain_ratio"]
        self.sample_gap = int(cfg["sample_gap"])
        self.text_length = int(cfg["text_length"])
        self.force_tail = int(cfg["force_tail"])
        self.energy_threshold = float(cfg.get("energy_threshold", 0.95))
        self.block = int(cfg.get("block", 128))
        self.num_keep = int(cfg.get("num_keep", 32))
        if self.block != 128 or self.num_keep != 32:
            raise ValueError("block=128 and num_keep=32 are the reference's (only) values")
        self.log_every = int(cfg["log_every"])
        self.mask_head_mode = cfg.get("mask_head_mode", "per_head")
        ops.mask_head_mode_code(self.mask_head_mode)   # validates
        self.gilbert_rearranger = GilbertRearranger(cfg["width"], cfg["height"], cfg["depth"],
                                                    self.text_length)
        # running sparsity statistic kept on the device (the reference's .item() per call, :415,
        # is replaced by a device counter; read it through .sparsity)
        self.sparsity_counter = 0
        self._kept_slots = None
        self._slot_totals = []
        self.last_mask: Optional[torch.Tensor] = None
        # optional list: when set, every `attn_event_every`-th fused attention launch is bracketed
        # by a pair of HIP events on the launch stream (bench.py's live kernel timing; each pair is
        # two marker packets that cost the stream a few us, so the bench samples); None = no events
        self.attn_events: Optional[list] = None
        self.attn_event_every = 1
        self._attn_launches = 0
        # run the pooled K/V pass inside the predictor's launch (extra workgroups beside the score
        # workgroups, one stream) instead of as its own launch after it (inference only)
        self.overlap = bool(cfg.get("overlap", True))
        # The attention kernel gathers K/V rows through the Gilbert index (True) or streams the
        # Gilbert-ordered contiguous copies the pooled pass writes (False: 2·L·D·2 bytes more per
        # head, written beside the predictor). "auto" (default): what measured faster per head dim
        # (tools/diag/overlap_ab.py --opt gather_kv): gather at D=128 (Wan, +2.4 % per call), copies at
        # D=64 (CogVideoX, +0.9 %).
        self.gather_kv = cfg.get("gather_kv", "auto")
        # Dispatch each XCD's q-blocks of the attention launch longest first (the predictor writes
        # every mask row's kept-block count; a small launch sorts the XCD ranges before the kernel):
        # the kernel's tail is its last workgroups. Scheduling only: outputs are bit-identical.
        # order_window > 0 re-orders only each XCD range's last q-blocks (the tail), keeping the
        # head-major Gilbert-neighbour order elsewhere for its L2 reuse.
        self.order = bool(cfg.get("order", ORDER_DEFAULT[variant]))
        self.order_window = int(cfg.get("order_window", 0))
        # The fused attention launch is resident-sized (as many workgroups as fit on the device at
        # once) and its workgroups pull q-blocks from per-XCD queues in the order above, then help
        # the other XCDs: no per-workgroup launch gaps, no XCD left idle at the end. Scheduling
        # only: outputs are bit-identical.
        self.persistent = bool(cfg.get("persistent", PERSISTENT_DEFAULT[variant]))

    # -------------------------------------------------------------------------------- helpers
    def _rows(self, device):
        if not self.use_rearrange:
            return None
        r = self.gilbert_rearranger.rows
        if r.device != device:
            r = r.to(device)
            self.gilbert_rearranger.rows = r
        return r

    def _gather(self, D: int) -> bool:
        if self.gather_kv != "auto":
            return bool(self.gather_kv)
        return D == 128

    def _count_slot(self, device):
        if self._kept_slots is None or self._kept_slots.device != device:
            self._kept_slots = torch.zeros(4096, dtype=torch.int64, device=device)
            self._slot_totals = []
        i = len(self._slot_totals) % self._kept_slots.numel()
        if i == 0 and self._slot_totals:
            self._fold_slots()
            i = 0
        return self._kept_slots[i:i + 1]

    def _fold_slots(self):
        kept = self._kept_slots[:len(self._slot_totals)].double().cpu().numpy()
        tot = np.asarray(self._slot_totals, dtype=np.float64)
        self._folded = getattr(self, "_folded", 0.0) + float(np.sum(1.0 - kept / tot - 1.0 / self.sample_gap))
        self._kept_slots.zero_()
        self._slot_totals = []

    @property
    def sparsity(self) -> float:
        """Average reported sparsity 1 - mean(mask) - 1/sample_gap over all calls (:394, :415).
        Reading it synchronises once; the forward never does."""
        if self.sparsity_counter == 0:
            return 0.0
        if self._slot_totals:
            self._fold_slots()
        return getattr(self, "_folded", 0.0) / self.sparsity_counter

    def _log_gap(self, dtype) -> float:
        """ln(gap) as the reference computes it: torch.log of a tensor in the LSE's storage
        dtype (lse is cast to q.dtype at :324, the log taken in it at :375-376), i.e. 2.703125
        for g=15 in bf16. The training path's combine rounds it the same way (vb_pool.hip)."""
        return float(torch.log(torch.tensor(float(self.sample_gap), dtype=dtype)).item())

    # -------------------------------------------------------------------------------- forward
    def predict_mask(self, q, k, q_off=None, k_off=None, count=None, staged_event=None, pool=None,
                     rows_kept=None):
        """Block mask [B,H,nb,nb] (uint8, Gilbert order) and normalised pooled scores. ``pool``
        (v, gap, outs) runs the pooled K/V pass inside the score kernel's launch."""
        B, H, L, D = q.shape
        rand = philox = None
        if q_off is None and k_off is None:
            # the reference's two draws (:77-78, q first), generated and ranked inside the sampling
            # launch at the device generator's Philox state (the values torch.rand would return)
            philox = ops.claim_rand_draws(q.device, B * H * self.block)
            if philox is None:
                rand = (torch.rand(B, H, 1, self.block, device=q.device),
                        torch.rand(B, H, 1, self.block, device=q.device))
        elif q_off is None:
            q_off = draw_sample_offsets(B, H, q.device)
        elif k_off is None:
            k_off = draw_sample_offsets(B, H, q.device)
        nb = (L + self.block - 1) // self.block
        lo, hi = retain_counts(nb, self.min_retain_ratio, self.max_retain_ratio, self.variant)
        po, mask = ops.mask_predict(q, k, q_off, k_off, rows=self._rows(q.device),
                                    energy_threshold=self.energy_threshold, min_keep=lo,
                                    max_keep=hi, force_tail=self.force_tail, mask_count=count,
                                    staged_event=staged_event, rand=rand, philox=philox,
                                    pool=pool, rows_kept=rows_kept)
        return po, mask

    def forward(self, q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, *,
                q_off: Optional[torch.Tensor] = None, k_off: Optional[torch.Tensor] = None,
                block_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        B, H, L, D = q.shape
        if k.shape != q.shape or v.shape != q.shape:
            # the reference's index_select over the Gilbert index fails on a shorter k/v (e.g. the
            # Wan I2V image keys); every launch below assumes q's [B,H,L,D] for k and v
            raise ValueError(f"k and v must have q's shape {tuple(q.shape)}, got "
                             f"{tuple(k.shape)} and {tuple(v.shape)}")
        if self.use_rearrange and L != self.gilbert_rearranger.seq_len:
            raise ValueError(f"sequence length {L} != {self.gilbert_rearranger.seq_len} expected "
                             f"by the Gilbert grid (width/height/depth/text_length)")
        rows = self._rows(q.device)
        nb = (L + self.block - 1) // self.block
        count = self._count_slot(q.device)
        grad = torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad)
        fused = not grad and self.combine != "reference"
        pooled = None
        rows_kept = None
        if block_mask is None:
            # inference: the pooled K/V pass (one pass over K/V: pooled K/V + the Gilbert-ordered
            # contiguous copies the attention kernel streams by LDS-DMA; HBM-bound) runs inside the
            # predictor's score-kernel launch, beside the MFMA-bound score workgroups (overlap=True),
            # or after it (overlap=False)
            ride = fused and self.overlap
            gather = self._gather(D)
            copies = not (gather and rows is not None)
            outs = ops.pool_kv_outputs(k, self.sample_gap, reordered=copies) if ride else None
            if fused and self.order and self.mask_head_mode == "per_head":
                rows_kept = torch.empty(B, H, nb, device=q.device, dtype=torch.int32)
            with torch.no_grad():
                _, mask = self.predict_mask(q.detach(), k.detach(), q_off, k_off, count,
                                            pool=(v, self.sample_gap, outs) if ride else None,
                                            rows_kept=rows_kept)
            if ride:
                pooled = outs
            elif fused:
                pooled = ops.pool_kv(k, v, self.sample_gap, rows, reordered=copies)
        else:
            mask = block_mask.to(torch.uint8)
            count.add_(mask.sum())
            if fused:
                gather = self._gather(D)
                pooled = ops.pool_kv(k, v, self.sample_gap, rows, reordered=not (gather and rows is not None))
        self._slot_totals.append(B * H * nb * nb)
        self.sparsity_counter += 1
        self.last_mask = mask
        if self.mask_head_mode == "shared_head0":
            # head_mask_type's ones read literally: every head uses base_blockmask head 0 (a
            # head-stride-0 view; the kernels index the mask through its strides)
            mask = mask[:, :1].expand(B, H, mask.shape[2], mask.shape[3])
        if not fused:
            from .autograd import adaptive_split_attention
            out = adaptive_split_attention(q, k, v, mask, rows, self.sample_gap,
                                           heavy_rows=self.force_tail)
        else:
            # q rows gathered and out rows scattered inside the attention kernel
            if len(pooled) == 4:   # Gilbert-ordered copies: streamed contiguously
                kp, vp, k_src, v_src = pooled
                kv_rows = None
            else:                  # the caller's k/v, rows gathered through the Gilbert index
                kp, vp = pooled
                k_src, v_src, kv_rows = k, v, rows
            ev = self.attn_events
            if ev is not None:
                self._attn_launches += 1
                if (self._attn_launches - 1) % self.attn_event_every:
                    ev = None
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            out = ops.attention_fwd(q, k_src, v_src, block_mask=mask, q_rows=rows, kv_rows=kv_rows,
                                    kp=kp, vp=vp, kp_log_bias=self._log_gap(q.dtype),
                                    heavy_rows=self.force_tail, order=self.order, q_lengths=rows_kept,
                                    order_window=self.order_window, persistent=self.persistent)
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                ev.append((e0, e1))
        if self.log_every and self.sparsity_counter % self.log_every == 0:
            print(f"sparsity: {self.sparsity}")
        return out


# reference-named alias (the patch functions install one shared instance on every block)
AdaptiveBlockSparseAttnTrain = AdaptiveBlockSparseAttn
