"""Monkey-patch surface: attention processors and the two setter functions.

Mirrors cogvideox/train/modify_cogvideo.py:11-91 and wanx/train/modify_wan.py:75-168. The
processors are the callers of the hot path (QKV projections, norms and RoPE stay in PyTorch);
``attn.inner_attention(q, k, v)`` is the vblade module. diffusers is imported lazily and only
for its RoPE helper; nothing here needs it at import time.
"""
from __future__ import annotations

from typing import Optional

import torch

from .attention import AdaptiveBlockSparseAttn


def _apply_rotary_emb_real(x: torch.Tensor, freqs_cis) -> torch.Tensor:
    """diffusers.models.embeddings.apply_rotary_emb with use_real=True, unbind_dim=-1 (the form
    CogVideoX's processor uses): x * cos + rotate_half(x) * sin over interleaved pairs."""
    try:  # prefer the library's own implementation when present
        from diffusers.models.embeddings import apply_rotary_emb
        return apply_rotary_emb(x, freqs_cis)
    except Exception:  # noqa: BLE001 - diffusers absent in this image
        cos, sin = freqs_cis
        cos, sin = cos[None, None].to(x.device), sin[None, None].to(x.device)
        x_real, x_imag = x.reshape(*x.shape[:-1], -1, 2).unbind(-1)
        x_rot = torch.stack([-x_imag, x_real], dim=-1).flatten(3)
        return (x.float() * cos + x_rot.float() * sin).to(x.dtype)


class CogVideoXBlockSparseAttnProcessor:
    """SageAttnCogVideoXAttnProcessor (modify_cogvideo.py:11-76): joint text+video self-attention
    whose inner attention is ``attn.inner_attention``. Text tokens come FIRST in the sequence."""

    def __init__(self, idx: int = 0):
        self.idx = idx

    def __call__(self, attn, hidden_states, encoder_hidden_states, attention_mask=None,
                 image_rotary_emb=None):
        assert attention_mask is None, "Attention mask is not supported"
        text_seq_length = encoder_hidden_states.size(1)
        hidden_states = torch.cat([encoder_hidden_states, hidden_states], dim=1)
        batch_size = encoder_hidden_states.shape[0]
        query = attn.to_q(hidden_states)
        key = attn.to_k(hidden_states)
        value = attn.to_v(hidden_states)
        head_dim = key.shape[-1] // attn.heads
        query = query.view(batch_size, -1, attn.heads, head_dim).transpose(1, 2)
        key = key.view(batch_size, -1, attn.heads, head_dim).transpose(1, 2)
        value = value.view(batch_size, -1, attn.heads, head_dim).transpose(1, 2)
        if getattr(attn, "norm_q", None) is not None:
            query = attn.norm_q(query).to(dtype=value.dtype)
        if getattr(attn, "norm_k", None) is not None:
            key = attn.norm_k(key).to(dtype=value.dtype)
        if image_rotary_emb is not None:
            query[:, :, text_seq_length:] = _apply_rotary_emb_real(query[:, :, text_seq_length:], image_rotary_emb)
            if not getattr(attn, "is_cross_attention", False):
                key[:, :, text_seq_length:] = _apply_rotary_emb_real(key[:, :, text_seq_length:], image_rotary_emb)
        hidden_states = attn.inner_attention(query, key, value.contiguous())
        hidden_states = hidden_states.transpose(1, 2).reshape(batch_size, -1, attn.heads * head_dim)
        hidden_states = attn.to_out[0](hidden_states)
        hidden_states = attn.to_out[1](hidden_states)
        encoder_hidden_states, hidden_states = hidden_states.split(
            [text_seq_length, hidden_states.size(1) - text_seq_length], dim=1)
        return hidden_states, encoder_hidden_states


def set_block_sparse_attn_cogvideox(model, verbose: bool = False, **attn_kwargs):
    """modify_cogvideo.py:79-91: ONE shared inner-attention module on every transformer block's
    attn1, processor swapped, the original kept as ``origin_processor``. Returns the module."""
    inner_attn = AdaptiveBlockSparseAttn("cog", **attn_kwargs)
    for idx, block in enumerate(model.transformer_blocks):
        block.attn1.verbose = verbose
        block.attn1.inner_attention = inner_attn
        origin = block.attn1.get_processor() if hasattr(block.attn1, "get_processor") else None
        block.attn1.set_processor(CogVideoXBlockSparseAttnProcessor(idx))
        if not hasattr(block.attn1, "origin_processor"):
            block.attn1.origin_processor = origin
    return inner_attn


class WanBlockSparseAttnProcessor:
    """WanAttnProcessor2_0 (modify_wan.py:75-148): video self-attention (attn1) with the
    complex-valued RoPE in float64; the I2V image branch also goes through inner_attention."""

    def __call__(self, attn, hidden_states, encoder_hidden_states=None, attention_mask=None,
                 rotary_emb: Optional[torch.Tensor] = None):
        encoder_hidden_states_img = None
        if getattr(attn, "add_k_proj", None) is not None:
            encoder_hidden_states_img = encoder_hidden_states[:, :257]
            encoder_hidden_states = encoder_hidden_states[:, 257:]
        if encoder_hidden_states is None:
            encoder_hidden_states = hidden_states
        query = attn.to_q(hidden_states)
        key = attn.to_k(encoder_hidden_states)
        value = attn.to_v(encoder_hidden_states)
        if getattr(attn, "norm_q", None) is not None:
            query = attn.norm_q(query)
        if getattr(attn, "norm_k", None) is not None:
            key = attn.norm_k(key)
        query = query.unflatten(2, (attn.heads, -1)).transpose(1, 2)
        key = key.unflatten(2, (attn.heads, -1)).transpose(1, 2)
        value = value.unflatten(2, (attn.heads, -1)).transpose(1, 2)
        if rotary_emb is not None:
            def apply_rotary_emb(hs, freqs):
                x_rotated = torch.view_as_complex(hs.to(torch.float64).unflatten(3, (-1, 2)))
                return torch.view_as_real(x_rotated * freqs).flatten(3, 4).type_as(hs)
            query = apply_rotary_emb(query, rotary_emb)
            key = apply_rotary_emb(key, rotary_emb)
        hidden_states_img = None
        if encoder_hidden_states_img is not None:
            key_img = attn.norm_added_k(attn.add_k_proj(encoder_hidden_states_img))
            value_img = attn.add_v_proj(encoder_hidden_states_img)
            key_img = key_img.unflatten(2, (attn.heads, -1)).transpose(1, 2)
            value_img = value_img.unflatten(2, (attn.heads, -1)).transpose(1, 2)
            hidden_states_img = attn.inner_attention(query, key_img, value_img)
            hidden_states_img = hidden_states_img.transpose(1, 2).flatten(2, 3).type_as(query)
        hidden_states = attn.inner_attention(query, key, value)
        hidden_states = hidden_states.transpose(1, 2).flatten(2, 3).type_as(query)
        if hidden_states_img is not None:
            hidden_states = hidden_states + hidden_states_img
        hidden_states = attn.to_out[0](hidden_states)
        hidden_states = attn.to_out[1](hidden_states)
        return hidden_states


def set_adaptive_block_sparse_attn_wanx(model, verbose: bool = False, **attn_kwargs):
    """modify_wan.py:150-168: patch attn1 (self-attention) of every block; attn2 (cross-attention
    to the T5 tokens) keeps stock SDPA. Returns the shared module."""
    inner_attn = AdaptiveBlockSparseAttn("wan", **attn_kwargs)
    for block in model.blocks:
        block.attn1.verbose = verbose
        block.attn1.inner_attention = inner_attn
        origin = block.attn1.get_processor() if hasattr(block.attn1, "get_processor") else None
        block.attn1.set_processor(WanBlockSparseAttnProcessor())
        if not hasattr(block.attn1, "origin_processor"):
            block.attn1.origin_processor = origin
    return inner_attn
