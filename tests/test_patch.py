"""CPU: the monkey-patch surface — processors and setters of vblade/patch.py
against hand-written statements of the reference processors, with SDPA standing in for
``attn.inner_attention`` (the layout around the op is what is checked here; the op itself is
checked on the GPU in test_gpu_module.py).

References:
  CogVideoX  cogvideox/train/modify_cogvideo.py:22-76 (processor), :79-91 (setter)
  Wan2.1     wanx/train/modify_wan.py:95-148 (processor), :150-168 (setter)

The hand-written statements below spell RoPE out per element pair (not with the reshape/stack
form patch.py uses), so a transposed pair, a wrong sign or RoPE on the text rows shows up.
"""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import vblade
from vblade import patch

SDPA = F.scaled_dot_product_attention


class FakeAttention(nn.Module):
    """The attributes the processors read from diffusers' Attention."""

    def __init__(self, dim, heads, qk_norm="head", i2v=False, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.heads = heads
        hd = dim // heads
        self.to_q, self.to_k, self.to_v = (nn.Linear(dim, dim) for _ in range(3))
        # CogVideoX normalises per head after the split; Wan over the whole projection before it
        nd = hd if qk_norm == "head" else dim
        self.norm_q = nn.LayerNorm(nd) if qk_norm else None
        self.norm_k = nn.LayerNorm(nd) if qk_norm else None
        self.to_out = nn.ModuleList([nn.Linear(dim, dim), nn.Dropout(0.0)])
        self.is_cross_attention = False
        self.add_k_proj = nn.Linear(dim, dim) if i2v else None
        self.add_v_proj = nn.Linear(dim, dim) if i2v else None
        self.norm_added_k = nn.LayerNorm(dim) if i2v else None
        self.processor = "stock"
        self.inner_attention = SDPA

    def get_processor(self):
        return self.processor

    def set_processor(self, p):
        self.processor = p


def rope_real_pairs(x, cos, sin):
    """diffusers apply_rotary_emb(use_real=True, unbind_dim=-1), written per pair:
    y[2i] = x[2i] cos[2i] - x[2i+1] sin[2i];  y[2i+1] = x[2i+1] cos[2i+1] + x[2i] sin[2i+1]."""
    xf = x.float()
    y = torch.empty_like(xf)
    y[..., 0::2] = xf[..., 0::2] * cos[..., 0::2] - xf[..., 1::2] * sin[..., 0::2]
    y[..., 1::2] = xf[..., 1::2] * cos[..., 1::2] + xf[..., 0::2] * sin[..., 1::2]
    return y.to(x.dtype)


def cog_reference(attn, hidden, text, rope):
    """modify_cogvideo.py:33-76, statement by statement (text first, RoPE on the video rows)."""
    T = text.size(1)
    B = text.shape[0]
    hs = torch.cat([text, hidden], dim=1)
    q, k, v = attn.to_q(hs), attn.to_k(hs), attn.to_v(hs)
    hd = k.shape[-1] // attn.heads
    q = q.view(B, -1, attn.heads, hd).transpose(1, 2)
    k = k.view(B, -1, attn.heads, hd).transpose(1, 2)
    v = v.view(B, -1, attn.heads, hd).transpose(1, 2)
    q = attn.norm_q(q).to(v.dtype)
    k = attn.norm_k(k).to(v.dtype)
    cos, sin = rope
    q = torch.cat([q[:, :, :T], rope_real_pairs(q[:, :, T:], cos, sin)], 2)
    k = torch.cat([k[:, :, :T], rope_real_pairs(k[:, :, T:], cos, sin)], 2)
    o = SDPA(q, k, v.contiguous())
    o = o.transpose(1, 2).reshape(B, -1, attn.heads * hd)
    o = attn.to_out[1](attn.to_out[0](o))
    return o[:, T:], o[:, :T]


def wan_rope_pairs(x, freqs):
    """The float64 complex product of modify_wan.py:106-110, written on real pairs."""
    xd = x.double()
    a, b = xd[..., 0::2], xd[..., 1::2]
    c, s = freqs.real, freqs.imag
    y = torch.empty_like(xd)
    y[..., 0::2] = a * c - b * s
    y[..., 1::2] = a * s + b * c
    return y.to(x.dtype)


def wan_reference(attn, hidden, enc, freqs):
    """modify_wan.py:95-148 (I2V: the first 257 context tokens are the image's)."""
    img = None
    if attn.add_k_proj is not None:
        img, enc = enc[:, :257], enc[:, 257:]
    if enc is None:
        enc = hidden
    q, k, v = attn.to_q(hidden), attn.to_k(enc), attn.to_v(enc)
    q, k = attn.norm_q(q), attn.norm_k(k)
    sp = lambda t: t.unflatten(2, (attn.heads, -1)).transpose(1, 2)  # noqa: E731
    q, k, v = sp(q), sp(k), sp(v)
    q, k = wan_rope_pairs(q, freqs), wan_rope_pairs(k, freqs)
    extra = None
    if img is not None:
        ki = sp(attn.norm_added_k(attn.add_k_proj(img)))
        vi = sp(attn.add_v_proj(img))
        extra = SDPA(q, ki, vi).transpose(1, 2).flatten(2, 3).type_as(q)
    o = SDPA(q, k, v).transpose(1, 2).flatten(2, 3).type_as(q)
    if extra is not None:
        o = o + extra
    return attn.to_out[1](attn.to_out[0](o))


def _rope_tables(S, hd, seed=3):
    g = torch.Generator().manual_seed(seed)
    ang = torch.rand(S, hd // 2, generator=g, dtype=torch.float64) * 6.28
    ang2 = ang.repeat_interleave(2, -1)      # CogVideoX's real form repeats each angle per pair
    return (ang2.cos().float(), ang2.sin().float()), torch.polar(torch.ones_like(ang), ang)[None, None]


@torch.no_grad()
def test_cog_processor_matches_reference_statement():
    B, T, N, heads, dim = 2, 7, 40, 4, 64
    attn = FakeAttention(dim, heads)
    g = torch.Generator().manual_seed(1)
    hidden = torch.randn(B, N, dim, generator=g)
    text = torch.randn(B, T, dim, generator=g)
    rope, _ = _rope_tables(N, dim // heads)
    proc = patch.CogVideoXBlockSparseAttnProcessor(0)
    got_v, got_t = proc(attn, hidden, text, image_rotary_emb=rope)
    ref_v, ref_t = cog_reference(attn, hidden, text, rope)
    assert got_v.shape == (B, N, dim) and got_t.shape == (B, T, dim)
    torch.testing.assert_close(got_v, ref_v, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(got_t, ref_t, rtol=1e-5, atol=1e-5)


@torch.no_grad()
def test_cog_processor_rope_touches_video_rows_only():
    """inner_attention sees the text rows of q/k un-rotated and the video rows rotated."""
    B, T, N, heads, dim = 1, 5, 12, 2, 32
    attn = FakeAttention(dim, heads, qk_norm=None)
    seen = {}

    def spy(q, k, v):
        seen["q"], seen["k"] = q.clone(), k.clone()
        return SDPA(q, k, v)

    attn.inner_attention = spy
    g = torch.Generator().manual_seed(2)
    hidden, text = torch.randn(B, N, dim, generator=g), torch.randn(B, T, dim, generator=g)
    rope, _ = _rope_tables(N, dim // heads)
    patch.CogVideoXBlockSparseAttnProcessor(0)(attn, hidden, text, image_rotary_emb=rope)
    hs = torch.cat([text, hidden], 1)
    q0 = attn.to_q(hs).view(B, -1, heads, dim // heads).transpose(1, 2)
    assert torch.equal(seen["q"][:, :, :T], q0[:, :, :T])
    torch.testing.assert_close(seen["q"][:, :, T:], rope_real_pairs(q0[:, :, T:], *rope))


@pytest.mark.parametrize("i2v", [False, True])
@torch.no_grad()
def test_wan_processor_matches_reference_statement(i2v):
    B, N, heads, dim = 2, 36, 4, 64
    attn = FakeAttention(dim, heads, qk_norm="full", i2v=i2v)
    g = torch.Generator().manual_seed(4)
    hidden = torch.randn(B, N, dim, generator=g)
    _, freqs = _rope_tables(N, dim // heads)
    # I2V: 257 image tokens, then a context as long as the video (the reference rotates k by the
    # video's RoPE table, so the lengths must match for the product to broadcast)
    enc = torch.randn(B, 257 + N, dim, generator=g) if i2v else None
    got = patch.WanBlockSparseAttnProcessor()(attn, hidden, enc, rotary_emb=freqs)
    ref = wan_reference(attn, hidden, enc, freqs)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


class _Block(nn.Module):
    def __init__(self, dim=64, heads=1):
        super().__init__()
        self.attn1 = FakeAttention(dim, heads)


class _CogModel(nn.Module):
    def __init__(self, n=3):
        super().__init__()
        self.transformer_blocks = nn.ModuleList([_Block() for _ in range(n)])


class _WanModel(nn.Module):
    def __init__(self, n=3):
        super().__init__()
        self.blocks = nn.ModuleList([_Block() for _ in range(n)])


def test_cog_setter_installs_one_shared_module():
    m = _CogModel()
    inner = vblade.set_block_sparse_attn_cogvideox(m, verbose=True)
    assert isinstance(inner, vblade.AdaptiveBlockSparseAttnTrain)
    assert inner.variant == "cog" and inner.gilbert_rearranger.seq_len == 17776
    for idx, b in enumerate(m.transformer_blocks):
        assert b.attn1.inner_attention is inner
        assert isinstance(b.attn1.processor, patch.CogVideoXBlockSparseAttnProcessor)
        assert b.attn1.processor.idx == idx
        assert b.attn1.origin_processor == "stock" and b.attn1.verbose is True
    # a second call keeps the first origin_processor (modify_cogvideo.py:90-91)
    vblade.set_block_sparse_attn_cogvideox(m)
    assert all(b.attn1.origin_processor == "stock" for b in m.transformer_blocks)


def test_wan_setter_installs_one_shared_module():
    m = _WanModel()
    inner = vblade.set_adaptive_block_sparse_attn_wanx(m)
    assert inner.variant == "wan" and inner.gilbert_rearranger.seq_len == 32760
    for b in m.blocks:
        assert b.attn1.inner_attention is inner
        assert isinstance(b.attn1.processor, patch.WanBlockSparseAttnProcessor)
        assert b.attn1.origin_processor == "stock"


def test_module_rejects_mismatched_kv_before_any_launch():
    """The reference's index_select raises on a k/v shorter than q (e.g. the Wan I2V image keys
    through the sparse module); vblade raises ValueError up front, on CPU tensors too."""
    mod = vblade.AdaptiveBlockSparseAttn("cog", width=12, height=8, depth=6, text_length=26)
    L = mod.gilbert_rearranger.seq_len
    q = torch.zeros(1, 2, L, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError, match="k and v"):
        mod(q, q[:, :, :257], q[:, :, :257])
    with pytest.raises(ValueError, match="k and v"):
        mod(q, q, q[:, :1])
