"""Backward entry points used by the autograd Functions (vblade/autograd.py).

Both run entirely in libvblade_hip.so (vb_attn_bwd / vb_block_sparse_attn_bwd):
* ``block_sparse_attn_bwd`` — the backward of the reference op block_sparse_attn_func
  (FlashAttention-2 semantics: the LSE output carries no gradient), varlen layout.
* ``adaptive_split_bwd`` — the reference autograd through adaptive_block_sparse_attn
  (cogvideo_blocksparseattn.py:366-393): alpha detached, dO1 = alpha*dO,
  dO2 = (1-alpha)*dO, per-branch FA2 backward, pooled K/V grads through the mean pool and the
  Gilbert gather.
"""
from __future__ import annotations

from . import ops


def block_sparse_attn_bwd(dout, q, k, v, out, lse, cu_q, cu_k, head_mask_type, mask, max_q, max_k,
                          scale):
    return ops.block_sparse_attn_bwd(dout, q, k, v, out, lse, cu_q, cu_k, head_mask_type, None,
                                     mask, max_q, max_k, softmax_scale=scale)


def adaptive_split_bwd(dout, q, k_r, v_r, mask, rows, out1, lse1, out2, lse2, alpha, kp, vp, gap,
                       heavy_rows=0):
    """k_r/v_r: the reordered K/V the forward attended to; rows: reordered -> caller row (or
    None). Returns (dq, dk, dv) in the caller's row order."""
    return ops.attention_bwd(dout, q, k_r, v_r, out1, lse1, block_mask=mask, q_rows=rows,
                             kv_rows=rows, kp=kp, vp=vp, out2=out2, lse2=lse2, alpha=alpha,
                             gap=gap, heavy_rows=heavy_rows)
