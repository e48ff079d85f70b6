"""autograd.Function wrappers with the reference's gradient semantics.

* ``block_sparse_attn_func`` — drop-in for mit-han-lab/Block-Sparse-Attention's function of the
  same name as called at cogvideo_blocksparseattn.py:316-320 (differentiable in q, k, v; the
  returned LSE carries no gradient, FlashAttention-2 convention).
* ``adaptive_split_attention`` — adaptive_block_sparse_attn's two-branch form (:366-393): block-
  sparse branch + pooled dense branch + bf16 LSE combine. Under autograd alpha is a constant
  (both LSEs are detached), so dO1 = alpha*dO, dO2 = (1-alpha)*dO and each branch back-propagates
  with its own output and LSE; pooled-branch K/V gradients flow back through the mean pool.
"""
from __future__ import annotations

import torch

from . import ops

# The training forward's pooled-only branch (every query against the pooled keys) on a side stream
# beside the block-sparse branch: the two launches share only their inputs, so they can fill each
# other's last rounds. Scheduling only: the same bits (tools/ab.py --what trainfwd,
# profiles/r06_trainfwd_fork_ab.log): Wan (D=128) 1.031-1.034x, CogVideoX 0.989-0.992x, so D=128 only.
FORK_POOLED_BRANCH = True
_SIDE_STREAMS = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _SIDE_STREAMS.get(idx)
    if st is None:
        st = _SIDE_STREAMS[idx] = torch.cuda.Stream(device=idx)
    return st


class _BlockSparseAttnFunc(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, cu_q, cu_k, head_mask_type, streaming_info, base_blockmask,
                max_q, max_k, p_dropout, deterministic, softmax_scale, is_causal, exact_streaming,
                mask_head_mode):
        out, lse = ops.block_sparse_attn_fwd(q, k, v, cu_q, cu_k, head_mask_type, streaming_info,
                                             base_blockmask, max_q, max_k, p_dropout,
                                             deterministic, softmax_scale, is_causal,
                                             exact_streaming, mask_head_mode=mask_head_mode)
        ctx.save_for_backward(q, k, v, out, lse, cu_q, cu_k, head_mask_type, base_blockmask)
        ctx.meta = (max_q, max_k, softmax_scale, mask_head_mode)
        ctx.mark_non_differentiable(lse)
        return out, lse

    @staticmethod
    def backward(ctx, dout, _dlse):
        q, k, v, out, lse, cu_q, cu_k, hmt, mask = ctx.saved_tensors
        max_q, max_k, scale, mode = ctx.meta
        dq, dk, dv = ops.block_sparse_attn_bwd(dout, q, k, v, out, lse, cu_q, cu_k, hmt, None,
                                               mask, max_q, max_k, softmax_scale=scale,
                                               mask_head_mode=mode)
        return (dq, dk, dv) + (None,) * 13


def block_sparse_attn_func(q_unpad, k_unpad, v_unpad, cu_seqlens_q, cu_seqlens_k, head_mask_type,
                           streaming_info, base_blockmask, max_seqlen_q_, max_seqlen_k_, p_dropout,
                           deterministic=False, softmax_scale=None, is_causal=False,
                           exact_streaming=False, return_attn_probs=False, mask_head_mode="per_head"):
    """Same signature and return convention as the reference's external op. ``mask_head_mode``
    (keyword, not in the reference's signature): the reading of head_mask_type's ones that SURVEY
    Appendix B leaves open offline ("per_head" default, "shared_head0")."""
    out, lse = _BlockSparseAttnFunc.apply(q_unpad, k_unpad, v_unpad, cu_seqlens_q, cu_seqlens_k,
                                          head_mask_type, streaming_info, base_blockmask,
                                          max_seqlen_q_, max_seqlen_k_, p_dropout, deterministic,
                                          softmax_scale, is_causal, exact_streaming, mask_head_mode)
    if return_attn_probs:
        return out, lse, None
    return out


class _AdaptiveSplitFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask, rows, gap, heavy_rows):
        kp, vp, k_r, v_r = ops.pool_kv(k, v, gap, rows, reordered=True)
        # the persistent (work-queue) launch at D=128: Wan's LSE forward 1.024-1.030x, CogVideoX's
        # 0.98x (profiles/r06_persist_unscoped_ab.log); bit-identical either way
        fork = FORK_POOLED_BRANCH and q.is_cuda and q.shape[-1] == 128
        if fork:
            cur = torch.cuda.current_stream(q.device)
            side = _side_stream(q.device)
            side.wait_stream(cur)   # kp/vp and q are ready
            with torch.cuda.stream(side):
                out2, lse2 = ops.attention_fwd(q, None, None, use_main=False, q_rows=rows, kp=kp,
                                               vp=vp, need_lse=True)
        else:
            out2, lse2 = ops.attention_fwd(q, None, None, use_main=False, q_rows=rows, kp=kp, vp=vp,
                                           need_lse=True)
        out1, lse1 = ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True,
                                       heavy_rows=heavy_rows, persistent=q.shape[-1] == 128)
        if fork:
            cur.wait_stream(side)
            for t in (q, kp, vp, rows):   # read on the side stream: not reused before it is done
                if t is not None:
                    t.record_stream(side)
            out2.record_stream(cur)
            lse2.record_stream(cur)
        out, alpha = ops.lse_combine(out1, lse1, out2, lse2, gap)
        ctx.save_for_backward(q, k_r, v_r, mask, rows, out1, lse1, out2, lse2, alpha, kp, vp)
        ctx.gap = gap
        ctx.heavy_rows = heavy_rows
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k_r, v_r, mask, rows, out1, lse1, out2, lse2, alpha, kp, vp = ctx.saved_tensors
        # per-branch FA2 backward with dO1 = alpha*dO, dO2 = (1-alpha)*dO; pooled-branch K/V grads
        # through the mean pool and the Gilbert gather, returned in the caller's row order
        dq, dk, dv = ops.attention_bwd(dout.contiguous(), q, k_r, v_r, out1, lse1, block_mask=mask,
                                       q_rows=rows, kv_rows=rows, kp=kp, vp=vp, out2=out2,
                                       lse2=lse2, alpha=alpha, gap=ctx.gap, heavy_rows=ctx.heavy_rows)
        return dq, dk, dv, None, None, None, None


def adaptive_split_attention(q, k, v, mask, rows, gap, heavy_rows=2):
    """heavy_rows: forced-dense tail rows dispatched first (CogVideoX 2, Wan 0); scheduling only."""
    return _AdaptiveSplitFn.apply(q, k, v, mask, rows, gap, heavy_rows)
