"""Multi-level block-sparse attention — the VBench sampler's ``inner_attention``.

Mirrors cogvideox/sample_evaluate/Triton/cogvideo_newattn.py (imported by
cogvideox/sample_evaluate/modify_cogvideo.py:9):

  * ``adaptive_block_sparse_attn(q, k, v)`` (:210-234): sampled pooled scores
    (``efficient_attn_with_pooling`` :64-89, the same sampler and pooled-score kernel as the main
    path) -> ``transfer_attn_to_mask`` (:154-207, rank bands ``mask_ratios`` :12-18) -> the
    multi-level kernel ``sparse_attention_factory(BLOCK_M=128, BLOCK_N=128)`` (:9) of
    kernels/block_sparse_attn_kernel_with_backward_9_10.py. Returns ``(out, sparsity)``.
  * ``AdaptiveBlockSparseAttnTrain`` (:237-267): Gilbert reorder (text moved to the tail), the call
    above, the running sparsity print every 600 calls, and the reverse reorder.
  * ``sparse_attention_factory`` (kernel file :1590-1612): the op itself, [B,H,L,D] in/out with a
    [B,H,nb,nb] int level mask (0 skip, 1/2/4/8 = K/V mean-pooled by that factor, +ln p logit bias).

Every tensor op runs in libvblade_hip.so:
  1. vb_mask_predict (the rand draws generated and ranked inside its sampling launch) — sampled
     pooled scores (Gilbert order through ``rows``) and, in the score kernel's epilogue, the rank
     bands -> uint8 level mask (vb_level_mask's rule, ``mask_level``); the KV pyramid pass (one
     pass over K/V: reordered level-1 rows + 2x/4x/8x pooled rows, HBM-bound) runs as extra
     workgroups of the same launch
  2. vb_ml_attn_fwd — one softmax over every kept block's keys at its level; q rows gathered and
                      out rows scattered through the Gilbert index inside the kernel
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from . import ops
from .attention import GilbertRearranger, draw_sample_offsets_qk

# Triton/cogvideo_newattn.py:12-24
MASK_RATIOS = dict(ops.ML_MASK_RATIOS)
DEFAULTS = dict(use_rearrange=True, width=45, height=30, depth=13, text_length=226)
BLOCK = 128
FUSED_LEVEL_MASK = True   # False: the level mask as its own vb_level_mask launch (A/B timing only)


def density(mask_ratios=None) -> float:
    """The reported density of adaptive_block_sparse_attn (:227-231): sum over levels of
    (end - start) / level. The reference reports 1 - density as the sparsity."""
    r = MASK_RATIOS if mask_ratios is None else mask_ratios
    return sum((e - s) / v for v, (s, e) in r.items() if v != 0)


def predict_level_mask(q, k, *, rows=None, mask_ratios=None, q_off=None, k_off=None, pyr=None):
    """efficient_attn_with_pooling + transfer_attn_to_mask on the (reordered through ``rows``)
    q, k: returns (po [B,H,nb,nb] q.dtype, level mask uint8 [B,H,nb,nb]). ``pyr=(v, outs)``: the
    KV pyramid pass in the score kernel's launch (ops.mask_predict)."""
    B, H, L, D = q.shape
    rand = philox = None
    if q_off is None and k_off is None:
        # the reference's two draws (:77-78, q first), generated and ranked inside the sampling
        # launch, as in AdaptiveBlockSparseAttn.predict_mask
        philox = ops.claim_rand_draws(q.device, B * H * BLOCK)
        if philox is None:
            rand = (torch.rand(B, H, 1, BLOCK, device=q.device), torch.rand(B, H, 1, BLOCK, device=q.device))
    elif q_off is None or k_off is None:
        q_off, k_off = draw_sample_offsets_qk(B, H, q.device, BLOCK, 32)
    # the rank-band level mask comes out of the score kernel's epilogue (vb_predict_args.mask_level;
    # ops.level_mask is the stand-alone form of the same rule)
    if not FUSED_LEVEL_MASK:
        po, _ = ops.mask_predict(q, k, q_off, k_off, rows=rows, want_mask=False, rand=rand, philox=philox,
                                 pyr=pyr)
        return po, ops.level_mask(po, mask_ratios)
    return ops.mask_predict(q, k, q_off, k_off, rows=rows, rand=rand, philox=philox, pyr=pyr,
                            level=MASK_RATIOS if mask_ratios is None else mask_ratios)


def adaptive_block_sparse_attn(q, k, v, *, rows=None, mask_ratios=None, ref_tail=True,
                               q_off=None, k_off=None, return_mask=False):
    """adaptive_block_sparse_attn (Triton/cogvideo_newattn.py:210-234), inference.

    ``rows`` (optional int32 [L]) applies the Gilbert reorder inside the kernels: reordered row g
    is caller row rows[g] for q, k, v, and the output is written back at rows[g] — equivalent to
    rearrange -> this function -> reversed_rearrange without the copies."""
    with torch.no_grad():
        po, mask = predict_level_mask(q, k, rows=rows, mask_ratios=mask_ratios, q_off=q_off,
                                      k_off=k_off)
        kpyr, vpyr = ops.kv_pyramid(k, v, rows)
        out = ops.ml_attention_fwd(q, kpyr, vpyr, mask, q_rows=rows, ref_tail=ref_tail)
    sp = 1.0 - density(mask_ratios)
    if return_mask:
        return out, sp, mask, po
    return out, sp


class _SparseAttention(torch.autograd.Function):
    """The multi-level op with the reference kernel's autograd contract (:1580-1588)."""

    @staticmethod
    def forward(ctx, q, k, v, level_mask, sm_scale, ref_tail, rows=None):
        mask_u8 = level_mask.to(torch.uint8).contiguous()
        kpyr, vpyr = ops.kv_pyramid(k, v, rows)
        out, lse = ops.ml_attention_fwd(q, kpyr, vpyr, mask_u8, q_rows=rows, scale=sm_scale,
                                        ref_tail=ref_tail, want_lse=True)
        ctx.save_for_backward(q, kpyr, vpyr, mask_u8, out, lse, rows)
        ctx.sm_scale = sm_scale
        ctx.ref_tail = ref_tail
        return out

    @staticmethod
    def backward(ctx, dout):
        q, kpyr, vpyr, mask_u8, out, lse, rows = ctx.saved_tensors
        dq, dk, dv = ops.ml_attention_bwd(dout.contiguous(), q, kpyr, vpyr, mask_u8, out, lse,
                                          rows=rows, scale=ctx.sm_scale, ref_tail=ctx.ref_tail)
        return dq, dk, dv, None, None, None, None


def sparse_attention_factory(BLOCK_M=128, BLOCK_N=128, POOLING_BLOCK_N=128, ref_tail=True, **kwargs):
    """kernels/block_sparse_attn_kernel_with_backward_9_10.py:1590-1612: returns
    ``fn(q, k, v, level_mask, sm_scale=None) -> out``. Block sizes other than 128 are not
    supported (the reference's sampler uses 128/128/128)."""
    if (BLOCK_M, BLOCK_N, POOLING_BLOCK_N) != (128, 128, 128):
        raise ValueError("vblade: the multi-level op is built for BLOCK_M = BLOCK_N = POOLING_BLOCK_N = 128")

    def fn(q, k, v, block_sparse_dense, sm_scale=None):
        scale = sm_scale if sm_scale is not None else q.shape[-1] ** -0.5
        return _SparseAttention.apply(q, k, v, block_sparse_dense, scale, ref_tail)

    return fn


class AdaptiveBlockSparseAttnTrain(nn.Module):
    """``inner_attention(q, k, v)`` of the VBench sampler (Triton/cogvideo_newattn.py:237-267).

    Keyword arguments override the module globals (width/height/depth/text_length/use_rearrange,
    mask_ratios). ``ref_tail`` keeps the reference kernel's level-1 tail behaviour (see
    include/vblade.h, vb_ml_attn_fwd)."""

    def __init__(self, *, mask_ratios=None, ref_tail: bool = True, log_every: int = 600,
                 overlap: bool = True, persistent: bool = False, **overrides):
        """overlap: run the KV pyramid pass inside the predictor's launch (True) or as its own
        launch after it. persistent: the attention launch is resident-sized and pulls q-blocks
        from per-XCD work queues (scheduling only; see attention.PERSISTENT_DEFAULT)."""
        super().__init__()
        cfg = dict(DEFAULTS)
        unknown = set(overrides) - set(cfg)
        if unknown:
            raise TypeError(f"unknown options {sorted(unknown)}")
        cfg.update(overrides)
        self.use_rearrange = bool(cfg["use_rearrange"])
        self.text_length = int(cfg["text_length"])
        self.gilbert_rearranger = GilbertRearranger(cfg["width"], cfg["height"], cfg["depth"],
                                                    self.text_length)
        self.mask_ratios = dict(MASK_RATIOS if mask_ratios is None else mask_ratios)
        self.ref_tail = ref_tail
        self.log_every = int(log_every)
        self.sparsity_acc = 0.0
        self.sparsity_counter = 0
        self.last_mask: Optional[torch.Tensor] = None
        self.attn_events: Optional[list] = None   # bench.py's live kernel timing (see attention.py)
        self.attn_event_every = 1
        self._attn_launches = 0
        self.overlap = bool(overlap)
        self.persistent = bool(persistent)

    def _rows(self, device):
        if not self.use_rearrange:
            return None
        r = self.gilbert_rearranger.rows
        if r.device != device:
            r = r.to(device)
            self.gilbert_rearranger.rows = r
        return r

    def forward(self, q, k, v, *, q_off=None, k_off=None, level_mask=None):
        B, H, L, D = q.shape
        if self.use_rearrange and L != self.gilbert_rearranger.seq_len:
            raise ValueError(f"sequence length {L} != {self.gilbert_rearranger.seq_len} expected "
                             f"by the Gilbert grid (width/height/depth/text_length)")
        rows = self._rows(q.device)
        grad = torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad)
        if grad:   # training: the autograd op (deterministic HIP backward), reorder inside it
            with torch.no_grad():
                if level_mask is None:
                    _, mask = predict_level_mask(q.detach(), k.detach(), rows=rows,
                                                 mask_ratios=self.mask_ratios, q_off=q_off, k_off=k_off)
                else:
                    mask = level_mask.to(torch.uint8).contiguous()
            out = _SparseAttention.apply(q, k, v, mask, q.shape[-1] ** -0.5, self.ref_tail, rows)
            self.last_mask = mask
            self.sparsity_acc += 1.0 - density(self.mask_ratios)
            self.sparsity_counter += 1
            return out
        with torch.no_grad():
            # the pyramid pass (HBM-bound) rides in the predictor's launch beside the MFMA-bound
            # score workgroups (one stream, no events), or runs after it
            outs = ops.kv_pyramid_outputs(k)   # before the predictor's temporaries
            if level_mask is None:
                _, mask = predict_level_mask(q, k, rows=rows, mask_ratios=self.mask_ratios,
                                             q_off=q_off, k_off=k_off,
                                             pyr=(v, outs) if self.overlap else None)
            else:
                mask = level_mask.to(torch.uint8).contiguous()
            if level_mask is None and self.overlap:
                kpyr, vpyr = outs
            else:
                kpyr, vpyr = ops.kv_pyramid(k, v, rows, out=outs)
            ev = self.attn_events
            if ev is not None:
                self._attn_launches += 1
                if (self._attn_launches - 1) % self.attn_event_every:
                    ev = None
            if ev is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            out = ops.ml_attention_fwd(q, kpyr, vpyr, mask, q_rows=rows, ref_tail=self.ref_tail,
                                       heavy_rows=2, persistent=self.persistent)
            if ev is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                ev.append((e0, e1))
        self.last_mask = mask
        self.sparsity_acc += 1.0 - density(self.mask_ratios)
        self.sparsity_counter += 1
        if self.log_every and self.sparsity_counter % self.log_every == 0:
            print(f"sparsity: {self.sparsity_acc / self.sparsity_counter}")
        return out
