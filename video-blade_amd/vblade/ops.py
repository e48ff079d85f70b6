"""Torch-facing wrappers over the C ABI (include/vblade.h).

PyTorch supplies device memory and the current HIP stream only; every byte of the hot path is
computed by libvblade_hip.so. Calls on CPU tensors raise (there is no CPU fallback).
"""
from __future__ import annotations

import ctypes
import math
import os
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import AttnArgs, BwdArgs, MlAttnArgs, MlBwdArgs, PredictArgs, check

BLOCK = 128


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return _lib.VB_DTYPE_BF16
    if t.dtype == torch.float16:
        return _lib.VB_DTYPE_F16
    raise TypeError(f"vblade: unsupported dtype {t.dtype} (bf16/fp16 only)")


def _require_gpu(*ts: Optional[torch.Tensor]):
    dev = None
    for t in ts:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("vblade: tensors must live on a HIP (cuda) device; there is no CPU path")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError("vblade: tensors on different devices")
    return dev


def _stream(dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _s3(t: torch.Tensor):
    """(batch, head, row) element strides of a [B,H,L,D] tensor with unit d-stride."""
    if t.stride(-1) != 1:
        raise ValueError("vblade: last dimension must be contiguous")
    return (ctypes.c_int64 * 3)(t.stride(0), t.stride(1), t.stride(2))


def _aligned_bhld(t: torch.Tensor) -> torch.Tensor:
    """Return t if its strides/pointer satisfy the kernels' 16-byte rules, else a contiguous copy."""
    if (t.stride(-1) == 1 and all(s % 8 == 0 for s in t.stride()[:3]) and t.data_ptr() % 16 == 0):
        return t
    return t.contiguous()


_WORK_QUEUES = {}


def work_queue(dev) -> torch.Tensor:
    """The persistent forward's work queue (include/vblade.h VB_WORK_QUEUE_INTS) for ``dev``'s current
    stream: int32, zero when allocated, and left zero by every launch that uses it. One per (device,
    stream), since two launches that may overlap must not share one."""
    dev = torch.device(dev)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, _stream(dev))
    wq = _WORK_QUEUES.get(key)
    if wq is None:
        wq = _WORK_QUEUES[key] = torch.zeros(_lib.VB_WORK_QUEUE_INTS, device=dev, dtype=torch.int32)
    return wq


def _check_dev(name: str, t: torch.Tensor, dev):
    """A pointer handed to a kernel must live on the launch's device (a CPU or other-GPU tensor
    would be a device fault or a write to the wrong memory, not a Python error)."""
    if t.device != dev:
        raise ValueError(f"{name} must be on {dev}, got {t.device}")


# ----------------------------------------------------------------------------------------------
# Gilbert permutation
# ----------------------------------------------------------------------------------------------
def gilbert_perm(width: int, height: int, depth: int) -> np.ndarray:
    """perm[g] = x + W*(y + H*z) of the g-th Gilbert point (vb_gilbert3d_perm, host C++)."""
    n = width * height * depth
    out = np.empty(n, dtype=np.int32)
    check(_lib.load().vb_gilbert3d_perm(width, height, depth, out.ctypes.data), "vb_gilbert3d_perm")
    return out


def sequence_rows(width: int, height: int, depth: int, text_length: int) -> np.ndarray:
    """Reordered position -> caller row: [video[perm] (+text offset), text] (CogVideoX puts the
    text tail last, cogvideo_blocksparseattn.py:141-154; Wan has text_length 0)."""
    perm = gilbert_perm(width, height, depth).astype(np.int64) + text_length
    return np.concatenate([perm, np.arange(text_length)]).astype(np.int32)


# ----------------------------------------------------------------------------------------------
# attention forward
# ----------------------------------------------------------------------------------------------
def attention_fwd(q: torch.Tensor, k: Optional[torch.Tensor], v: Optional[torch.Tensor], *,
                  block_mask: Optional[torch.Tensor] = None, q_rows: Optional[torch.Tensor] = None,
                  kv_rows: Optional[torch.Tensor] = None, kp: Optional[torch.Tensor] = None,
                  vp: Optional[torch.Tensor] = None, kp_log_bias: float = 0.0, use_main: bool = True,
                  scale: Optional[float] = None, need_lse: bool = False,
                  out: Optional[torch.Tensor] = None, heavy_rows: int = 0, order: bool = False,
                  q_lengths: Optional[torch.Tensor] = None, order_window: int = 0,
                  q_order_out: Optional[torch.Tensor] = None, persistent: bool = False):
    """vb_attn_fwd: softmax over (block-masked keys of k/v) ∪ (pooled keys kp/vp + bias).
    q,k,v [B,H,L,D]; block_mask [B,H,ceil(Lq/128),ceil(Lk/128)] bool/uint8; rows int32.
    ``order``: dispatch each XCD's q-blocks longest first (scheduling only; ``q_lengths`` [B,H,nbq]
    int32 kept blocks per mask row from mask_predict(rows_kept=...), else counted on the device;
    ``order_window`` > 0 re-orders only the last that many q-blocks of each XCD's range;
    ``q_order_out``: int32 [B*H*ceil(Lq/128)] to receive the dispatch permutation, for tests).
    ``persistent``: a resident-sized launch whose workgroups pull q-blocks from per-XCD queues
    (work_queue(); scheduling only, the same outputs).
    Returns out [B,H,Lq,D] (and lse fp32 [B,H,Lq] when need_lse)."""
    dev = _require_gpu(q, k, v, block_mask, q_rows, kv_rows, kp, vp, q_lengths, q_order_out)
    q = _aligned_bhld(q)
    B, H, Lq, D = q.shape
    if use_main:
        k, v = _aligned_bhld(k), _aligned_bhld(v)
        Lk = k.shape[2]
    else:
        Lk = 0
    if kp is not None:
        kp, vp = _aligned_bhld(kp), _aligned_bhld(vp)
    if out is None:
        out = torch.empty(B, H, Lq, D, device=dev, dtype=q.dtype)
    lse = torch.empty(B, H, Lq, device=dev, dtype=torch.float32) if need_lse else None
    a = AttnArgs()
    a.q = q.data_ptr()
    a.q_stride = _s3(q)
    if use_main:
        a.k, a.v = k.data_ptr(), v.data_ptr()
        a.k_stride, a.v_stride = _s3(k), _s3(v)
    a.q_rows, a.kv_rows = _ptr(q_rows), _ptr(kv_rows)
    a.use_main = 1 if use_main else 0
    if block_mask is not None:
        if block_mask.dtype == torch.bool:
            block_mask = block_mask.view(torch.uint8)
        nbq, nbk = (Lq + BLOCK - 1) // BLOCK, (Lk + BLOCK - 1) // BLOCK
        if block_mask.shape[2] < nbq or block_mask.shape[3] < nbk:
            raise ValueError(f"block_mask {tuple(block_mask.shape)} too small for {nbq}x{nbk} blocks")
        if block_mask.stride(3) != 1:
            block_mask = block_mask.contiguous()
        a.block_mask = block_mask.data_ptr()
        a.mask_stride = (ctypes.c_int64 * 3)(block_mask.stride(0), block_mask.stride(1),
                                             block_mask.stride(2))
    if kp is not None:
        a.kp, a.vp = kp.data_ptr(), vp.data_ptr()
        a.kp_stride, a.vp_stride = _s3(kp), _s3(vp)
        a.Lkp = kp.shape[2]
        a.kp_log_bias = float(kp_log_bias)
    a.out = out.data_ptr()
    a.out_stride = _s3(out)
    a.lse = _ptr(lse)
    a.B, a.H, a.Lq, a.Lk, a.D = B, H, Lq, Lk, D
    a.scale = float(scale) if scale else 0.0
    a.dtype = _dtype_code(q)
    a.heavy_rows = int(heavy_rows)
    if persistent:
        a.work_queue = work_queue(dev).data_ptr()
    if order and block_mask is not None and use_main:
        nbq = (Lq + BLOCK - 1) // BLOCK
        q_order = q_order_out if q_order_out is not None else torch.empty(B * H * nbq, device=dev, dtype=torch.int32)
        if q_order.dtype != torch.int32 or q_order.numel() < B * H * nbq or not q_order.is_contiguous() or q_order.device != dev:
            raise ValueError("attention_fwd: q_order_out must be a contiguous int32 tensor of B*H*ceil(Lq/128) on q's device")
        a.q_order = q_order.data_ptr()
        a.order_window = int(order_window)
        if q_lengths is not None:
            if q_lengths.dtype != torch.int32 or q_lengths.numel() != B * H * nbq or not q_lengths.is_contiguous():
                raise ValueError("attention_fwd: q_lengths must be contiguous int32 [B,H,ceil(Lq/128)]")
            _check_dev("attention_fwd: q_lengths", q_lengths, dev)
            a.q_lengths = q_lengths.data_ptr()
    check(_lib.load().vb_attn_fwd(ctypes.byref(a), _stream(dev)), "vb_attn_fwd")
    return (out, lse) if need_lse else out


MASK_HEAD_MODES = {"per_head": 0, "shared_head0": 1}   # vb_mask_head_mode


def mask_head_mode_code(mode: str) -> int:
    if mode not in MASK_HEAD_MODES:
        raise ValueError(f"mask_head_mode must be one of {sorted(MASK_HEAD_MODES)}, got {mode!r}")
    return MASK_HEAD_MODES[mode]


def block_sparse_attn_fwd(q_unpad, k_unpad, v_unpad, cu_seqlens_q, cu_seqlens_k, head_mask_type,
                          streaming_info, base_blockmask, max_seqlen_q, max_seqlen_k,
                          p_dropout=0.0, deterministic=False, softmax_scale=None,
                          is_causal=False, exact_streaming=False, mask_head_mode="per_head"):
    """Forward of block_sparse_attn_func through vb_block_sparse_attn_fwd (varlen layout).
    Returns (out_unpad [total_q,H,D], softmax_lse fp32 [B,H,max_seqlen_q]). ``mask_head_mode``:
    how head_mask_type's ones address base_blockmask's heads ("per_head": renumbered 1..H, one
    mask per head; "shared_head0": read literally, every such head uses mask head 0)."""
    mode = mask_head_mode_code(mask_head_mode)
    dev = _require_gpu(q_unpad, k_unpad, v_unpad, cu_seqlens_q, cu_seqlens_k, base_blockmask)
    q_unpad, k_unpad, v_unpad = q_unpad.contiguous(), k_unpad.contiguous(), v_unpad.contiguous()
    B = cu_seqlens_q.numel() - 1
    H, D = q_unpad.shape[1], q_unpad.shape[2]
    nbq = (max_seqlen_q + BLOCK - 1) // BLOCK
    nbk = (max_seqlen_k + BLOCK - 1) // BLOCK
    mask = None
    if base_blockmask is not None:
        mask = base_blockmask[:, :, :nbq, :nbk]
        if mask.dtype == torch.bool:
            mask = mask.contiguous().view(torch.uint8)
        mask = mask.to(torch.uint8).contiguous()
    hmt = head_mask_type.to(device=dev, dtype=torch.int32).contiguous() if head_mask_type is not None else None
    out = torch.empty_like(q_unpad)
    lse = torch.empty(B, H, max_seqlen_q, device=dev, dtype=torch.float32)
    check(_lib.load().vb_block_sparse_attn_fwd(
        q_unpad.data_ptr(), k_unpad.data_ptr(), v_unpad.data_ptr(),
        cu_seqlens_q.to(torch.int32).contiguous().data_ptr(),
        cu_seqlens_k.to(torch.int32).contiguous().data_ptr(),
        _ptr(hmt), _ptr(streaming_info), _ptr(mask), B, H, D, int(max_seqlen_q),
        int(max_seqlen_k), float(p_dropout), int(bool(deterministic)),
        float(softmax_scale) if softmax_scale else 0.0, int(bool(is_causal)),
        int(bool(exact_streaming)), _dtype_code(q_unpad), out.data_ptr(), lse.data_ptr(),
        mode, _stream(dev)), "vb_block_sparse_attn_fwd")
    return out, lse


# ----------------------------------------------------------------------------------------------
# backward
# ----------------------------------------------------------------------------------------------
def _mask_u8(block_mask, Lq, Lk):
    if block_mask is None:
        return None
    if block_mask.dtype == torch.bool:
        block_mask = block_mask.view(torch.uint8)
    nbq, nbk = (Lq + BLOCK - 1) // BLOCK, (Lk + BLOCK - 1) // BLOCK
    if block_mask.shape[2] < nbq or block_mask.shape[3] < nbk:
        raise ValueError(f"block_mask {tuple(block_mask.shape)} too small for {nbq}x{nbk} blocks")
    if block_mask.stride(3) != 1:
        block_mask = block_mask.contiguous()
    return block_mask


def attention_bwd(dout, q, k, v, out, lse, *, block_mask=None, q_rows=None, kv_rows=None,
                  kp=None, vp=None, out2=None, lse2=None, alpha=None, gap: int = 0,
                  scale: Optional[float] = None, heavy_rows: int = 0, dk_rows: Optional[int] = None,
                  kernel_select: int = 0, kernels_ran: Optional[list] = None):
    """vb_attn_bwd: gradients (dq, dk, dv) of the block-sparse attention, optionally of the
    adaptive two-branch form (kp/vp/out2/lse2/alpha/gap: alpha detached, pooled grads folded back
    through the mean pool). k/v hold keys in reordered order; dk/dv rows are written at
    kv_rows[g] (dk_rows = number of rows of dk/dv, default Lk). Returns bf16/fp16 tensors.
    ``kernel_select``: _lib.VB_BWD_SEL_* bits (0: the default kernels); ``kernels_ran`` (a list)
    receives the _lib.VB_BWD_RAN_* bits of the kernels the call launched."""
    dev = _require_gpu(dout, q, k, v, out, lse, block_mask, q_rows, kv_rows, kp, vp, out2, lse2,
                       alpha)
    q, k, v, out, dout = (_aligned_bhld(t) for t in (q, k, v, out, dout))
    B, H, Lq, D = q.shape
    Lk = k.shape[2]
    nrows = Lk if dk_rows is None else int(dk_rows)
    dq = torch.empty(B, H, Lq, D, device=dev, dtype=q.dtype)
    dk = torch.empty(B, H, nrows, D, device=dev, dtype=q.dtype)
    dv = torch.empty(B, H, nrows, D, device=dev, dtype=q.dtype)
    a = BwdArgs()
    a.q, a.q_stride = q.data_ptr(), _s3(q)
    a.k, a.v, a.k_stride, a.v_stride = k.data_ptr(), v.data_ptr(), _s3(k), _s3(v)
    a.q_rows, a.kv_rows = _ptr(q_rows), _ptr(kv_rows)
    m = _mask_u8(block_mask, Lq, Lk)
    if m is not None:
        a.block_mask = m.data_ptr()
        a.mask_stride = (ctypes.c_int64 * 3)(m.stride(0), m.stride(1), m.stride(2))
    a.out, a.out_stride = out.data_ptr(), _s3(out)
    lse = lse.float().contiguous()
    a.lse = lse.data_ptr()
    if kp is not None:
        kp, vp, out2 = _aligned_bhld(kp), _aligned_bhld(vp), _aligned_bhld(out2)
        lse2 = lse2.float().contiguous()
        alpha = alpha.float().contiguous()
        a.kp, a.vp, a.kp_stride, a.vp_stride = kp.data_ptr(), vp.data_ptr(), _s3(kp), _s3(vp)
        a.Lkp = kp.shape[2]
        a.out2, a.out2_stride = out2.data_ptr(), _s3(out2)
        a.lse2, a.alpha = lse2.data_ptr(), alpha.data_ptr()
        a.pool_gap = int(gap)
    a.dout, a.dout_stride = dout.data_ptr(), _s3(dout)
    a.dq, a.dq_stride = dq.data_ptr(), _s3(dq)
    a.dk, a.dv, a.dk_stride, a.dv_stride = dk.data_ptr(), dv.data_ptr(), _s3(dk), _s3(dv)
    a.B, a.H, a.Lq, a.Lk, a.D = B, H, Lq, Lk, D
    a.scale = float(scale) if scale else 0.0
    a.dtype = _dtype_code(q)
    a.heavy_rows = int(heavy_rows)
    a.kernel_select = int(kernel_select)
    ran = ctypes.c_int32(0)
    a.kernels_ran = ctypes.pointer(ran)
    lib = _lib.load()
    nbytes = int(lib.vb_attn_bwd_workspace_size(ctypes.byref(a)))
    ws = torch.empty(max(nbytes, 16), device=dev, dtype=torch.uint8)
    a.workspace, a.workspace_bytes = ws.data_ptr(), nbytes
    check(lib.vb_attn_bwd(ctypes.byref(a), _stream(dev)), "vb_attn_bwd")
    if kernels_ran is not None:
        kernels_ran.append(ran.value)
    return dq, dk, dv


def block_sparse_attn_bwd(dout, q_unpad, k_unpad, v_unpad, out_unpad, softmax_lse, cu_seqlens_q,
                          cu_seqlens_k, head_mask_type, streaming_info, base_blockmask,
                          max_seqlen_q, max_seqlen_k, p_dropout=0.0, softmax_scale=None,
                          is_causal=False, exact_streaming=False, deterministic=True,
                          mask_head_mode="per_head"):
    """Backward of block_sparse_attn_func (vb_block_sparse_attn_bwd, varlen layout).
    Returns (dq, dk, dv) [total, H, D]. ``mask_head_mode`` as block_sparse_attn_fwd."""
    mode = mask_head_mode_code(mask_head_mode)
    dev = _require_gpu(dout, q_unpad, k_unpad, v_unpad, out_unpad, softmax_lse, base_blockmask)
    dout, q_unpad, k_unpad, v_unpad, out_unpad = (t.contiguous() for t in
                                                  (dout, q_unpad, k_unpad, v_unpad, out_unpad))
    B = cu_seqlens_q.numel() - 1
    H, D = q_unpad.shape[1], q_unpad.shape[2]
    nbq = (max_seqlen_q + BLOCK - 1) // BLOCK
    nbk = (max_seqlen_k + BLOCK - 1) // BLOCK
    mask = None
    if base_blockmask is not None:
        mask = base_blockmask[:, :, :nbq, :nbk]
        if mask.dtype == torch.bool:
            mask = mask.contiguous().view(torch.uint8)
        mask = mask.to(torch.uint8).contiguous()
    hmt = head_mask_type.to(device=dev, dtype=torch.int32).contiguous() if head_mask_type is not None else None
    cu_q = cu_seqlens_q.to(torch.int32).contiguous()
    cu_k = cu_seqlens_k.to(torch.int32).contiguous()
    lse = softmax_lse.float().contiguous()
    dq, dk, dv = torch.empty_like(q_unpad), torch.empty_like(k_unpad), torch.empty_like(v_unpad)
    lib = _lib.load()
    nbytes = int(lib.vb_block_sparse_attn_bwd_workspace_size(B, H, int(max_seqlen_q)))
    ws = torch.empty(max(nbytes, 16), device=dev, dtype=torch.uint8)
    check(lib.vb_block_sparse_attn_bwd(
        dout.data_ptr(), q_unpad.data_ptr(), k_unpad.data_ptr(), v_unpad.data_ptr(),
        out_unpad.data_ptr(), lse.data_ptr(), cu_q.data_ptr(), cu_k.data_ptr(), _ptr(hmt),
        _ptr(streaming_info), _ptr(mask), B, H, D, int(max_seqlen_q), int(max_seqlen_k),
        float(p_dropout), float(softmax_scale) if softmax_scale else 0.0, int(bool(is_causal)),
        int(bool(exact_streaming)), int(bool(deterministic)), _dtype_code(q_unpad),
        dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), ws.data_ptr(), nbytes, mode, _stream(dev)),
        "vb_block_sparse_attn_bwd")
    return dq, dk, dv


# ----------------------------------------------------------------------------------------------
# mask predictor, energy rule, pooling, combine
# ----------------------------------------------------------------------------------------------
def mask_predict(q, k, q_off=None, k_off=None, *, rows=None, energy_threshold=0.95, min_keep=1,
                 max_keep=1, force_tail=0, scale=None, mask_count=None, want_mask=True,
                 staged_event=None, rand=None, philox=None, pool=None, pyr=None, level=None,
                 rows_kept=None):
    """vb_mask_predict. q,k [B,H,L,D]; q_off/k_off int32 [B,H,32]. Returns (po, mask) with
    po [B,H,nb,nb] in q.dtype and mask uint8 [B,H,nb,nb] (None with want_mask=False: the scores
    only, no energy rule). ``staged_event`` (a torch.cuda.Event) is recorded once the sampled
    rows are staged, before the score kernel: work waiting on it overlaps the score kernel.

    ``rand=(rand_q, rand_k)``: the fp32 uniforms [B,H,1,block] of random_sample_tokens instead of
    q_off/k_off; the topk offsets are drawn inside the sampling launch.
    ``philox=(seed, offset)`` (from claim_rand_draws): those two draws generated inside the
    sampling launch too, equal to the values torch.rand would return at that generator state.
    ``pool=(v, gap, outs)``: the pooled K/V pass (vb_pool_kv of k, v through ``rows``) run by extra
    workgroups of the score kernel's launch on the current stream; ``outs`` = pool_kv_outputs(k,
    gap, reordered) receives kp, vp[, k_r, v_r].
    ``pyr=(v, outs)``: the multi-level KV pyramid pass (vb_kv_pyramid of k, v through ``rows``)
    run the same way; ``outs`` = kv_pyramid_outputs(k). Excludes ``pool``.
    ``level=mask_ratios``: the returned mask is the multi-level rank-band mask (level_mask's rule
    on the scores, computed by the score kernel's epilogue) instead of the energy mask.
    ``rows_kept``: int32 [B,H,nb] receiving the energy rule's kept-block count per mask row."""
    try:
        return _mask_predict(q, k, q_off, k_off, rows=rows, energy_threshold=energy_threshold,
                             min_keep=min_keep, max_keep=max_keep, force_tail=force_tail, scale=scale,
                             mask_count=mask_count, want_mask=want_mask, staged_event=staged_event,
                             rand=rand, philox=philox, pool=pool, pyr=pyr, level=level,
                             rows_kept=rows_kept)
    except Exception as e:
        # the claimed draws go back to the generator only when nothing was launched: a Python-side
        # error (validation, or a host-side VBladeError such as the library failing to load, code
        # None), or the library refusing the call (VB_ERR_INVALID / _UNSUPPORTED, returned before
        # any launch). After a VB_ERR_LAUNCH the sampling launch may already have consumed them, and
        # rewinding would make the next torch.rand repeat those Philox values.
        launched = isinstance(e, _lib.VBladeError) and e.code not in (None, _lib.VB_ERR_INVALID,
                                                                      _lib.VB_ERR_UNSUPPORTED)
        if philox is not None and not launched:
            release_rand_draws(q.device, philox)
        raise


def _mask_predict(q, k, q_off, k_off, *, rows, energy_threshold, min_keep, max_keep, force_tail,
                  scale, mask_count, want_mask, staged_event, rand, philox, pool, pyr, level, rows_kept):
    if k.shape != q.shape:
        raise ValueError(f"mask_predict: k and v must have q's shape {tuple(q.shape)}, "
                         f"got k {tuple(k.shape)}")
    dev = _require_gpu(q, k, q_off, k_off, rows, rows_kept)
    q, k = _aligned_bhld(q), _aligned_bhld(k)
    B, H, L, D = q.shape
    nb = (L + BLOCK - 1) // BLOCK
    if rows_kept is not None and (level is not None or not want_mask):
        raise ValueError("mask_predict: rows_kept is written by the energy rule only (not with level= "
                         "or want_mask=False)")
    po = torch.empty(B, H, nb, nb, device=dev, dtype=q.dtype)
    mask = torch.empty(B, H, nb, nb, device=dev, dtype=torch.uint8) if want_mask else None
    if rand is not None and philox is not None:
        raise ValueError("mask_predict: rand and philox are exclusive")
    if rand is not None or philox is not None:
        if rand is not None:
            rand_q, rand_k = (r.float().contiguous() for r in rand)
        q_off = torch.empty(B, H, 32, device=dev, dtype=torch.int32)
        k_off = torch.empty(B, H, 32, device=dev, dtype=torch.int32)
    q_off = q_off.to(torch.int32).contiguous()
    k_off = k_off.to(torch.int32).contiguous()
    a = PredictArgs()
    a.q, a.k = q.data_ptr(), k.data_ptr()
    a.q_stride, a.k_stride = _s3(q), _s3(k)
    a.rows, a.q_off, a.k_off = _ptr(rows), q_off.data_ptr(), k_off.data_ptr()
    a.B, a.H, a.L, a.D, a.block, a.num_keep = B, H, L, D, BLOCK, q_off.shape[-1]
    a.scale = float(scale) if scale else 0.0
    a.energy_threshold = float(energy_threshold)
    a.min_keep, a.max_keep, a.force_tail = int(min_keep), int(max_keep), int(force_tail)
    a.po, a.mask, a.mask_count = po.data_ptr(), _ptr(mask), _ptr(mask_count)
    a.dtype = _dtype_code(q)
    lib = _lib.load()
    nbytes = int(lib.vb_mask_predict_workspace_size(ctypes.byref(a)))
    ws = torch.empty(max(nbytes, 16), device=dev, dtype=torch.uint8)
    a.workspace, a.workspace_bytes = ws.data_ptr(), nbytes
    a.staged_event = staged_event.cuda_event if staged_event is not None else None
    if rand is not None:
        if rand_q.shape[-1] != BLOCK or rand_q.numel() != B * H * BLOCK or rand_k.numel() != B * H * BLOCK:
            raise ValueError("mask_predict: rand draws must be [B,H,1,block]")
        a.rand_q, a.rand_k = rand_q.data_ptr(), rand_k.data_ptr()
    if philox is not None:
        a.philox, a.philox_seed, a.philox_offset = 1, int(philox[0]), int(philox[1])
    if pool is not None:
        v, gap, outs = pool
        v = _aligned_bhld(v)
        if v.shape != k.shape:
            raise ValueError(f"mask_predict: k and v must have q's shape {tuple(q.shape)}, "
                             f"got v {tuple(v.shape)}")
        if outs[0].shape != (B, H, (L + int(gap) - 1) // int(gap), D):
            raise ValueError("mask_predict: pool outputs must come from pool_kv_outputs(k, gap)")
        a.pool_v, a.pool_v_stride, a.pool_gap = v.data_ptr(), _s3(v), int(gap)
        a.pool_kp, a.pool_vp = outs[0].data_ptr(), outs[1].data_ptr()
        if len(outs) > 2:
            a.pool_k_r, a.pool_v_r = outs[2].data_ptr(), outs[3].data_ptr()
    if pyr is not None:
        if pool is not None:
            raise ValueError("mask_predict: pool and pyr are exclusive")
        v, outs = pyr
        v = _aligned_bhld(v)
        if v.shape != k.shape:
            raise ValueError(f"mask_predict: k and v must have q's shape {tuple(q.shape)}, "
                             f"got v {tuple(v.shape)}")
        if outs[0].shape != (B, H, kv_pyramid_rows(L), D) or outs[1].shape != outs[0].shape:
            raise ValueError("mask_predict: pyramid outputs must come from kv_pyramid_outputs(k)")
        a.pool_v, a.pool_v_stride = v.data_ptr(), _s3(v)
        a.pyr_k, a.pyr_v = outs[0].data_ptr(), outs[1].data_ptr()
    if level is not None:
        if mask is None:
            raise ValueError("mask_predict: level needs want_mask=True")
        vals, st, en = _level_bands(level)
        a.mask_level, a.level_bands = 1, len(vals)
        a.level_band_value, a.level_band_start, a.level_band_end = (
            vals.ctypes.data, st.ctypes.data, en.ctypes.data)
    if rows_kept is not None:
        if rows_kept.dtype != torch.int32 or rows_kept.numel() != B * H * nb or not rows_kept.is_contiguous():
            raise ValueError("mask_predict: rows_kept must be contiguous int32 [B,H,nb]")
        _check_dev("mask_predict: rows_kept", rows_kept, dev)
        a.mask_rows_kept = rows_kept.data_ptr()
    check(lib.vb_mask_predict(ctypes.byref(a), _stream(dev)), "vb_mask_predict")
    return po, mask


# torch.rand's launch on ROCm (ATen/native/hip/DistributionTemplates.h, calc_execution_policy and
# distribution_elementwise_grid_stride_kernel): 256-thread blocks, grid = min(ceil(numel / 256),
# CUs * maxThreadsPerMultiProcessor / 256); thread i draws one hiprand_uniform4 per pass and element
# li = i + pass_stride * c takes component c. Element i is the x component of thread i exactly while
# numel <= CUs * maxThreadsPerMultiProcessor (every element has a thread of its own; 524288 on an
# unpartitioned MI355X, fewer on a partitioned device or a smaller GPU). Each call then advances the
# generator's Philox offset by 4.
RAND_ONE_PASS_NUMEL = 524288   # the MI355X value; rand_one_pass_numel(device) is the per-device bound
PHILOX_DRAWS = os.environ.get("VB_PHILOX_DRAWS", "1") != "0"   # off: the callers use torch.rand
_ONE_PASS = {}


def rand_one_pass_numel(device) -> int:
    """Largest torch.rand numel whose element i is the x of Philox subsequence i on ``device``."""
    if not torch.cuda.is_available():
        return 0
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    n = _ONE_PASS.get(idx)
    if n is None:
        pr = torch.cuda.get_device_properties(idx)
        n = _ONE_PASS[idx] = int(pr.multi_processor_count) * int(pr.max_threads_per_multi_processor)
    return n


def claim_rand_draws(device, numel: int, draws: int = 2):
    """Reserve ``draws`` consecutive torch.rand(numel) calls on ``device``'s default generator for
    a kernel that generates them itself: returns (seed, offset) and advances the generator's offset
    as those calls would, or None when the draw is too large for one x-only pass on this device or
    the stream is being captured into a graph (then call torch.rand). mask_predict gives the draws
    back (release_rand_draws) when it raises before its launch."""
    if not PHILOX_DRAWS or numel > rand_one_pass_numel(device):
        return None
    # under HIP-graph capture torch.rand draws from a per-replay offset; a seed/offset read here
    # would be baked into the graph, so captured calls keep torch.rand
    if torch.cuda.is_current_stream_capturing():
        return None
    dev = torch.device(device)
    gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    seed, off = gen.initial_seed(), gen.get_offset()
    gen.set_offset(off + 4 * draws)
    return seed, off


def release_rand_draws(device, philox, draws: int = 2):
    """Undo claim_rand_draws when the launch it was made for did not run: the generator's offset
    goes back to the claimed one if nothing has drawn from it since."""
    dev = torch.device(device)
    gen = torch.cuda.default_generators[dev.index if dev.index is not None else torch.cuda.current_device()]
    if gen.initial_seed() == philox[0] and gen.get_offset() == philox[1] + 4 * draws:
        gen.set_offset(philox[1])


def sample_offsets(rand_q, rand_k, keep: int = 32):
    """vb_sample_offsets: topk(keep) indices (descending value, ties lower index first) of each
    row of the uniform draws rand_q/rand_k [..., n] -> int32 [..., keep] (q, k)."""
    dev = _require_gpu(rand_q, rand_k)
    rand_q, rand_k = rand_q.float().contiguous(), rand_k.float().contiguous()
    n = rand_q.shape[-1]
    rows = rand_q.numel() // n
    shape = tuple(rand_q.shape[:-1]) + (keep,)
    oq = torch.empty(shape, device=dev, dtype=torch.int32)
    ok = torch.empty(shape, device=dev, dtype=torch.int32)
    check(_lib.load().vb_sample_offsets(rand_q.data_ptr(), rand_k.data_ptr(), rows, n, keep,
                                        oq.data_ptr(), ok.data_ptr(), _stream(dev)),
          "vb_sample_offsets")
    return oq, ok


def energy_mask(po, *, energy_threshold=0.95, min_keep=1, max_keep=1, force_tail=0, mask_count=None):
    """vb_energy_mask on scores po [B,H,nr,nc] (bf16/fp16) -> uint8 mask."""
    dev = _require_gpu(po)
    po = po.contiguous()
    B, H, nr, nc = po.shape
    mask = torch.empty(B, H, nr, nc, device=dev, dtype=torch.uint8)
    check(_lib.load().vb_energy_mask(po.data_ptr(), B, H, nr, nc, float(energy_threshold),
                                     int(min_keep), int(max_keep), int(force_tail),
                                     _dtype_code(po), mask.data_ptr(), _ptr(mask_count),
                                     _stream(dev)), "vb_energy_mask")
    return mask


def pool_kv_outputs(k, gap: int, reordered: bool = False):
    """Allocate pool_kv's outputs (kp, vp[, k_r, v_r]) on the current stream. A caller that launches
    pool_kv on a side stream allocates them BEFORE enqueueing other work whose temporaries could
    otherwise be recycled into them while that work still runs."""
    B, H, L, D = k.shape
    Lp = (L + gap - 1) // gap
    kw = dict(device=k.device, dtype=k.dtype)
    outs = [torch.empty(B, H, Lp, D, **kw), torch.empty(B, H, Lp, D, **kw)]
    if reordered:
        outs += [torch.empty(B, H, L, D, **kw), torch.empty(B, H, L, D, **kw)]
    return tuple(outs)


def pool_kv(k, v, gap: int, rows=None, reordered: bool = False, stream=None, out=None):
    """vb_pool_kv: mean over `gap` consecutive reordered tokens (replicate pad) -> kp, vp; with
    reordered=True also returns the Gilbert-ordered contiguous copies (k_r, v_r) written in the
    same pass. ``stream`` (a torch.cuda.Stream) launches there instead of the current stream; the
    outputs are still allocated on the current stream, which must wait for ``stream`` before
    using them."""
    if v.shape != k.shape:
        raise ValueError(f"pool_kv: k and v must have the same shape, got {tuple(k.shape)} and "
                         f"{tuple(v.shape)}")
    if rows is not None and rows.numel() != k.shape[2]:
        raise ValueError(f"pool_kv: rows has {rows.numel()} entries for {k.shape[2]} keys")
    dev = _require_gpu(k, v, rows)
    k, v = _aligned_bhld(k), _aligned_bhld(v)
    if stream is not None:   # read (and written) on the side stream: no reuse before it is done
        for t in (k, v, rows) + tuple(out or ()):
            if t is not None:
                t.record_stream(stream)
    B, H, L, D = k.shape
    if out is None:
        out = pool_kv_outputs(k, gap, reordered)
    kp, vp = out[0], out[1]
    k_r, v_r = (out[2], out[3]) if reordered else (None, None)
    check(_lib.load().vb_pool_kv(k.data_ptr(), v.data_ptr(), ctypes.cast(_s3(k), ctypes.c_void_p),
                                 ctypes.cast(_s3(v), ctypes.c_void_p), _ptr(rows), B, H, L, D,
                                 int(gap), _dtype_code(k), kp.data_ptr(), vp.data_ptr(),
                                 _ptr(k_r), _ptr(v_r),
                                 stream.cuda_stream if stream is not None else _stream(dev)), "vb_pool_kv")
    if reordered:
        return kp, vp, k_r, v_r
    return kp, vp


def lse_combine(out1, lse1, out2, lse2, gap: float):
    """vb_lse_combine (reference-faithful eager rounding). Returns (out, alpha fp32 [B,H,L])."""
    dev = _require_gpu(out1, lse1, out2, lse2)
    out1, out2 = out1.contiguous(), out2.contiguous()
    lse1, lse2 = lse1.float().contiguous(), lse2.float().contiguous()
    B, H, L, D = out1.shape
    out = torch.empty_like(out1)
    alpha = torch.empty(B, H, L, device=dev, dtype=torch.float32)
    check(_lib.load().vb_lse_combine(out1.data_ptr(), lse1.data_ptr(), out2.data_ptr(),
                                     lse2.data_ptr(), B, H, L, D, float(gap), _dtype_code(out1),
                                     out.data_ptr(), alpha.data_ptr(), _stream(dev)),
          "vb_lse_combine")
    return out, alpha


# ----------------------------------------------------------------------------------------------
# multi-level path (Triton/cogvideo_newattn.py + kernels/block_sparse_attn_kernel_with_backward_9_10.py)
# ----------------------------------------------------------------------------------------------
# Triton/cogvideo_newattn.py:12-18
ML_MASK_RATIOS = {1: (0.0, 0.05), 2: (0.05, 0.15), 4: (0.15, 0.25), 8: (0.25, 0.5), 0: (0.5, 1.0)}


def kv_pyramid_rows(L: int) -> int:
    return int(_lib.load().vb_kv_pyramid_rows(int(L)))


def kv_pyramid_outputs(k):
    """Allocate kv_pyramid's outputs on the current stream (see pool_kv_outputs)."""
    B, H, L, D = k.shape
    R = kv_pyramid_rows(L)
    return (torch.empty(B, H, R, D, device=k.device, dtype=k.dtype),
            torch.empty(B, H, R, D, device=k.device, dtype=k.dtype))


def kv_pyramid(k, v, rows=None, stream=None, out=None):
    """vb_kv_pyramid: K/V [B,H,L,D] (reordered through `rows`) -> pyramids [B,H,15*Lpad/8,D]:
    level-1 rows (zero beyond L), then the 2x, 4x, 8x mean-pooled rows (replicate padding).
    ``stream``: as pool_kv."""
    if v.shape != k.shape:
        raise ValueError(f"kv_pyramid: k and v must have the same shape, got {tuple(k.shape)} and "
                         f"{tuple(v.shape)}")
    if rows is not None and rows.numel() != k.shape[2]:
        raise ValueError(f"kv_pyramid: rows has {rows.numel()} entries for {k.shape[2]} keys")
    dev = _require_gpu(k, v, rows)
    k, v = _aligned_bhld(k), _aligned_bhld(v)
    if stream is not None:   # see pool_kv
        for t in (k, v, rows) + tuple(out or ()):
            if t is not None:
                t.record_stream(stream)
    B, H, L, D = k.shape
    kpyr, vpyr = out if out is not None else kv_pyramid_outputs(k)
    check(_lib.load().vb_kv_pyramid(k.data_ptr(), v.data_ptr(), ctypes.cast(_s3(k), ctypes.c_void_p),
                                    ctypes.cast(_s3(v), ctypes.c_void_p), _ptr(rows), B, H, L, D,
                                    _dtype_code(k), kpyr.data_ptr(), vpyr.data_ptr(),
                                    stream.cuda_stream if stream is not None else _stream(dev)),
          "vb_kv_pyramid")
    return kpyr, vpyr


def pyramid_levels(pyr: torch.Tensor, L: int):
    """Views [level1, level2, level4, level8] of a pyramid tensor (for tests and the backward)."""
    Lpad = (L + BLOCK - 1) // BLOCK * BLOCK
    offs = [0, Lpad, Lpad + Lpad // 2, Lpad + Lpad // 2 + Lpad // 4, 15 * Lpad // 8]
    return [pyr[:, :, offs[i]:offs[i + 1]] for i in range(4)]


def _level_bands(ratios):
    """mask_ratios {level: (start, end)} -> (int32 values, float64 starts, float64 ends), dict order."""
    ratios = ML_MASK_RATIOS if ratios is None else ratios
    vals = np.array([int(v) for v in ratios], dtype=np.int32)
    st = np.array([float(r[0]) for r in ratios.values()], dtype=np.float64)
    en = np.array([float(r[1]) for r in ratios.values()], dtype=np.float64)
    if len(vals) > 8:
        raise ValueError("level mask: at most 8 bands")
    return vals, st, en


def level_mask(po, ratios=None):
    """vb_level_mask: transfer_attn_to_mask (Triton/cogvideo_newattn.py:154-207) on scores po
    [B,H,nr,nc] -> uint8 levels (ties: lower column first)."""
    dev = _require_gpu(po)
    po = po.contiguous()
    B, H, nr, nc = po.shape
    vals, st, en = _level_bands(ratios)
    mask = torch.empty(B, H, nr, nc, device=dev, dtype=torch.uint8)
    check(_lib.load().vb_level_mask(po.data_ptr(), B, H, nr, nc, len(vals), vals.ctypes.data,
                                    st.ctypes.data, en.ctypes.data, _dtype_code(po), mask.data_ptr(),
                                    _stream(dev)), "vb_level_mask")
    return mask


def ml_attention_fwd(q, kpyr, vpyr, level_mask_u8, *, q_rows=None, scale=None, ref_tail=True,
                     want_lse=False, heavy_rows=2, out=None, persistent: bool = False):
    """vb_ml_attn_fwd: multi-level attention of q [B,H,L,D] over the KV pyramids. Returns out
    (rows through q_rows) and, if want_lse, the fp32 natural-log LSE [B,H,L] (reordered rows)."""
    dev = _require_gpu(q, kpyr, vpyr, level_mask_u8, q_rows)
    q = _aligned_bhld(q)
    B, H, L, D = q.shape
    nb = (L + BLOCK - 1) // BLOCK
    if tuple(level_mask_u8.shape) != (B, H, nb, nb) or level_mask_u8.dtype != torch.uint8:
        raise ValueError(f"vblade: level mask must be uint8 [B,H,{nb},{nb}]")
    R = kv_pyramid_rows(L)
    for t in (kpyr, vpyr):
        if tuple(t.shape) != (B, H, R, D) or not t.is_contiguous() or t.dtype != q.dtype:
            raise ValueError(f"vblade: pyramids must be contiguous [B,H,{R},D] in q's dtype")
    m = level_mask_u8
    if m.stride(-1) != 1:
        m = m.contiguous()
    if out is None:
        out = torch.empty_like(q) if q.is_contiguous() else torch.empty(B, H, L, D, device=dev, dtype=q.dtype)
    lse = torch.empty(B, H, L, device=dev, dtype=torch.float32) if want_lse else None
    a = MlAttnArgs()
    a.q, a.q_stride, a.q_rows = q.data_ptr(), _s3(q), _ptr(q_rows)
    a.kpyr, a.vpyr = kpyr.data_ptr(), vpyr.data_ptr()
    a.level_mask = m.data_ptr()
    a.mask_stride = (ctypes.c_int64 * 3)(m.stride(0), m.stride(1), m.stride(2))
    a.out, a.out_stride, a.lse = out.data_ptr(), _s3(out), _ptr(lse)
    a.B, a.H, a.L, a.D = B, H, L, D
    a.scale = float(scale) if scale else 0.0
    a.ref_tail = 1 if ref_tail else 0
    a.dtype = _dtype_code(q)
    a.heavy_rows = int(heavy_rows)
    if persistent:
        a.work_queue = work_queue(dev).data_ptr()
    check(_lib.load().vb_ml_attn_fwd(ctypes.byref(a), _stream(dev)), "vb_ml_attn_fwd")
    return (out, lse) if want_lse else out


def ml_attention_bwd(dout, q, kpyr, vpyr, level_mask_u8, out, lse, *, rows=None, scale=None,
                     ref_tail=True, heavy_rows=2, kernel_select: int = 0, kernels_ran: Optional[list] = None):
    """vb_ml_attn_bwd: gradients of the multi-level attention. q/out/dout [B,H,L,D] (rows through
    ``rows``), pyramids and mask as the forward; lse as ml_attention_fwd(want_lse=True) wrote it.
    Returns (dq, dk, dv) [B,H,L,D] in q's dtype (dk/dv at the caller's rows). ``kernel_select`` /
    ``kernels_ran`` as attention_bwd (VB_BWD_SEL_DQ_RING4 is refused here)."""
    dev = _require_gpu(dout, q, kpyr, vpyr, level_mask_u8, out, lse, rows)
    q, out, dout = _aligned_bhld(q), _aligned_bhld(out), _aligned_bhld(dout)
    B, H, L, D = q.shape
    m = level_mask_u8 if level_mask_u8.stride(-1) == 1 else level_mask_u8.contiguous()
    lse = lse.float().contiguous()
    dq = torch.empty(B, H, L, D, device=dev, dtype=q.dtype)
    dk = torch.empty(B, H, L, D, device=dev, dtype=q.dtype)
    dv = torch.empty(B, H, L, D, device=dev, dtype=q.dtype)
    a = MlBwdArgs()
    a.q, a.q_stride, a.rows = q.data_ptr(), _s3(q), _ptr(rows)
    a.kpyr, a.vpyr = kpyr.data_ptr(), vpyr.data_ptr()
    a.level_mask = m.data_ptr()
    a.mask_stride = (ctypes.c_int64 * 3)(m.stride(0), m.stride(1), m.stride(2))
    a.out, a.out_stride, a.lse = out.data_ptr(), _s3(out), lse.data_ptr()
    a.dout, a.dout_stride = dout.data_ptr(), _s3(dout)
    a.dq, a.dq_stride = dq.data_ptr(), _s3(dq)
    a.dk, a.dv, a.dk_stride, a.dv_stride = dk.data_ptr(), dv.data_ptr(), _s3(dk), _s3(dv)
    a.B, a.H, a.L, a.D = B, H, L, D
    a.scale = float(scale) if scale else 0.0
    a.ref_tail = 1 if ref_tail else 0
    a.dtype = _dtype_code(q)
    a.heavy_rows = int(heavy_rows)
    a.kernel_select = int(kernel_select)
    ran = ctypes.c_int32(0)
    a.kernels_ran = ctypes.pointer(ran)
    lib = _lib.load()
    nbytes = int(lib.vb_ml_attn_bwd_workspace_size(ctypes.byref(a)))
    ws = torch.empty(max(nbytes, 16), device=dev, dtype=torch.uint8)
    a.workspace, a.workspace_bytes = ws.data_ptr(), nbytes
    check(lib.vb_ml_attn_bwd(ctypes.byref(a), _stream(dev)), "vb_ml_attn_bwd")
    if kernels_ran is not None:
        kernels_ran.append(ran.value)
    return dq, dk, dv


def default_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
