"""GPU parity of the whole inner_attention module (AdaptiveBlockSparseAttn) against
(a) the reference-generated end-to-end goldens (fp16 cases; the reference glue run in this
container, tests/golden/make_golden.py) and (b) the oracle at the real CogVideoX / Wan sizes
through size-independent properties."""
import math
import os

import numpy as np
import pytest
import torch

import bsa_oracle as O
from conftest import GOLDEN, record

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    peak = ref.double().abs().max().item()
    return 99.0 if mse == 0 else 10 * math.log10(peak * peak / mse)


def _module_for(z, case, combine):
    import vblade
    B, H, w, h, d, text, D = z[case + "_meta"].tolist()
    rmin, rmax, gap = z[case + "_ratios"].tolist()
    variant = str(z[case + "_variant"])
    m = vblade.AdaptiveBlockSparseAttn(variant, combine=combine, width=w, height=h, depth=d,
                                       text_length=text, min_retain_ratio=rmin,
                                       max_retain_ratio=rmax, sample_gap=int(gap), log_every=0)
    return m, variant


@pytest.mark.parametrize("case", ["cog_f16", "wan_f16"])
@pytest.mark.parametrize("combine", ["reference", "fused"])
def test_module_matches_reference_e2e_golden(case, combine):
    z = np.load(os.path.join(GOLDEN, "adaptive_e2e.npz"))
    m, variant = _module_for(z, case, combine)
    q, k, v = (torch.from_numpy(z[case + s]).to(torch.float16).to(DEV) for s in ("_q", "_k", "_v"))
    qo = torch.from_numpy(z[case + "_qoff"]).to(DEV)
    ko = torch.from_numpy(z[case + "_koff"]).to(DEV)
    with torch.no_grad():
        out = m(q, k, v, q_off=qo, k_off=ko)
    ref_mask = torch.from_numpy(z[case + "_mask"])
    ref_po = torch.from_numpy(z[case + "_po"])
    nb = ref_mask.shape[-1]
    from vblade.attention import retain_counts
    lo, hi = retain_counts(nb, m.min_retain_ratio, m.max_retain_ratio, variant)
    kk = O.energy_keep_counts(ref_po, lo, hi, store_dtype=torch.float16)
    assert O.mask_is_valid_topk(m.last_mask.bool().cpu(), ref_po, kk, m.force_tail)
    ref = torch.from_numpy(z[case + "_out"].astype(np.float32))
    got = out.float().cpu()
    tol = 3e-3 if combine == "reference" else 6e-3
    same_mask = torch.equal(m.last_mask.bool().cpu(), ref_mask)
    record("e2e golden: predicted mask == reference mask bit for bit",
           f"{case}/{combine}: {same_mask} ({int((m.last_mask.bool().cpu() != ref_mask).sum())} "
           f"of {ref_mask.numel()} blocks differ)")
    if same_mask:
        assert (got - ref).abs().max() <= tol
        assert abs(m.sparsity - float(z[case + "_sparsity"])) < 1e-6
    assert psnr(got, ref) >= 40
    # unconditional: the same module on the reference's own mask (the fixture's, from the same
    # offsets) reproduces the reference output to the stated tolerance whatever the tie-breaking
    # of the prediction above did (mask_head_mode per_head, the default)
    m2, _ = _module_for(z, case, combine)
    assert m2.mask_head_mode == "per_head"
    with torch.no_grad():
        out2 = m2(q, k, v, q_off=qo, k_off=ko, block_mask=ref_mask.to(DEV))
    err = (out2.float().cpu() - ref).abs().max().item()
    record("e2e golden: max|out - ref| on the reference mask", f"{case}/{combine}: {err:.2e} (tol {tol})")
    assert err <= tol


def _realistic_qkv(B, H, L, D, seed, dtype=torch.bfloat16):
    """BASELINE/SURVEY §8d realistic-input option: q,k = N(0,1) + 2*c[token // 128]."""
    g = torch.Generator().manual_seed(seed)
    cent = torch.randn(B, H, L // 128 + 1, D, generator=g).repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(B, H, L, D, generator=g) + 2 * cent).to(dtype)
    k = (torch.randn(B, H, L, D, generator=g) + 2 * cent).to(dtype)
    v = torch.randn(B, H, L, D, generator=g).to(dtype)
    return q, k, v


@pytest.mark.parametrize("variant,H,D", [("cog", 2, 64), ("wan", 1, 128)])
def test_full_size_module_against_oracle(variant, H, D):
    """Real sequence lengths (17776 / 32760), a subset of heads; the oracle recomputes the
    reference combine on the GPU's own mask and must agree to PSNR >= 40 dB (north_star)."""
    import vblade
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    q, k, v = _realistic_qkv(1, H, L, D, seed=5)
    torch.manual_seed(3)
    with torch.no_grad():
        out_fused = m(q.to(DEV), k.to(DEV), v.to(DEV))
    mask = m.last_mask.bool().cpu()
    nb = mask.shape[-1]
    kept_rows = mask.sum(-1)
    from vblade.attention import retain_counts
    lo, hi = retain_counts(nb, m.min_retain_ratio, m.max_retain_ratio, variant)
    body = kept_rows[..., : nb - m.force_tail] if m.force_tail else kept_rows
    assert body.min() >= lo and body.max() <= hi + m.force_tail
    if m.force_tail:
        assert mask[..., -2:, :].all() and mask[..., -2:].all()
    cfg = (O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan())
    ref = O.adaptive_attention(q, k, v, cfg, None, None, mask=mask, store_dtype=torch.bfloat16)
    assert psnr(out_fused.float().cpu(), ref["out"]) >= 40
    m2 = vblade.AdaptiveBlockSparseAttn(variant, combine="reference", log_every=0)
    with torch.no_grad():
        out_ref = m2(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=m.last_mask)
    assert psnr(out_ref.float().cpu(), ref["out"]) >= 45
    assert 0.0 < m.sparsity < 1.0


def test_sparsity_statistic_is_device_side_and_matches_mask():
    import vblade
    m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0, width=8, height=6, depth=10,
                                       text_length=30, min_retain_ratio=0.2, max_retain_ratio=0.5)
    L = m.gilbert_rearranger.seq_len
    vals = []
    for s in range(3):
        q, k, v = _realistic_qkv(1, 2, L, 64, seed=s)
        with torch.no_grad():
            m(q.to(DEV), k.to(DEV), v.to(DEV))
        vals.append(1 - m.last_mask.float().mean().item() - 1 / 15)
    assert abs(m.sparsity - sum(vals) / 3) < 1e-9


@pytest.mark.parametrize("variant,D", [("cog", 64), ("wan", 128)])
def test_fused_sampling_and_pool_launches_match_separate_launches(variant, D):
    """The module's launch structure (topk offsets drawn inside the sampling launch, the pooled
    K/V pass run by extra workgroups of the score kernel's launch) gives the same offsets, mask,
    pooled K/V, Gilbert copies and output, bit for bit, as the separate launches (vb_sample_offsets,
    vb_mask_predict with given offsets, vb_pool_kv) on the same RNG draws."""
    import vblade
    from vblade import ops
    kw = dict(width=12, height=8, depth=6, text_length=26) if variant == "cog" else dict(width=13, height=6, depth=7)
    fused = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **kw)
    sep = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, overlap=False, **kw)
    L = fused.gilbert_rearranger.seq_len
    H = 3
    g = torch.Generator(device=DEV).manual_seed(11)
    q, k, v = (torch.randn(1, H, L, D, generator=g, device=DEV).bfloat16() for _ in range(3))
    with torch.no_grad():
        torch.manual_seed(5)
        out_f = fused(q, k, v)
        torch.manual_seed(5)
        rq = torch.rand(1, H, 1, 128, device=DEV)
        rk = torch.rand(1, H, 1, 128, device=DEV)
        qo, ko = ops.sample_offsets(rq, rk, 32)
        out_s = sep(q, k, v, q_off=qo[:, :, 0], k_off=ko[:, :, 0])
        rows = fused._rows(q.device)
        outs = ops.pool_kv_outputs(k, fused.sample_gap, reordered=True)
        _, mask_p = ops.mask_predict(q, k, rows=rows, energy_threshold=0.95, min_keep=1, max_keep=4,
                                     rand=(rq, rk), pool=(v, fused.sample_gap, outs))
        _, mask_r = ops.mask_predict(q, k, qo[:, :, 0], ko[:, :, 0], rows=rows, energy_threshold=0.95,
                                     min_keep=1, max_keep=4)
        ref_pool = ops.pool_kv(k, v, fused.sample_gap, rows, reordered=True)
    torch.cuda.synchronize()
    assert torch.equal(fused.last_mask, sep.last_mask)
    assert torch.equal(out_f, out_s)
    assert torch.equal(mask_p, mask_r)
    for a, b in zip(outs, ref_pool):
        assert torch.equal(a, b)


@pytest.mark.parametrize("variant,D,B,H,strided", [("cog", 64, 1, 3, False), ("cog", 64, 2, 2, True),
                                                     ("wan", 128, 1, 2, False), ("wan", 128, 2, 1, True)])
def test_fused_pooled_pass_matches_pool_kv_at_full_length(variant, D, B, H, strided):
    """At the real sequence lengths, the pooled K/V pass run by the extra workgroups of the score
    kernel's launch: pooled K/V and the Gilbert-order copies must equal the stand-alone
    vb_pool_kv bit for bit, and the mask and scores must equal the predictor run without the pass.
    Batched and on the processors' strided [B,L,H,D].transpose(1,2) views."""
    import vblade
    from vblade import ops
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    g = torch.Generator(device=DEV).manual_seed(77)
    shape = (B, L, H, D) if strided else (B, H, L, D)
    q, k, v = (torch.randn(*shape, generator=g, device=DEV).bfloat16() for _ in range(3))
    if strided:
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    rows = m._rows(q.device)
    rq = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    rk = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    with torch.no_grad():
        for copies in (True, False):
            outs = ops.pool_kv_outputs(k, m.sample_gap, reordered=copies)
            po_p, mask_p = ops.mask_predict(q, k, rows=rows, energy_threshold=0.95, min_keep=6,
                                            max_keep=13, force_tail=m.force_tail, rand=(rq, rk),
                                            pool=(v, m.sample_gap, outs))
            po_r, mask_r = ops.mask_predict(q, k, rows=rows, energy_threshold=0.95, min_keep=6,
                                            max_keep=13, force_tail=m.force_tail, rand=(rq, rk))
            ref = ops.pool_kv(k, v, m.sample_gap, rows, reordered=copies)
            torch.cuda.synchronize()
            assert torch.equal(mask_p, mask_r) and torch.equal(po_p, po_r)
            assert len(outs) == len(ref)
            for a, b in zip(outs, ref):
                assert torch.equal(a, b)


@pytest.mark.parametrize("variant,D", [("cog", 64), ("wan", 128)])
def test_gathered_kv_rows_equal_gilbert_copies(variant, D):
    """The attention kernel gathering K/V rows through the Gilbert index (gather_kv=True) and
    streaming the pooled pass's Gilbert-ordered copies (gather_kv=False) read the same keys in the
    same order: bit-identical outputs, on shapes with a partial last key block."""
    import vblade
    kw = dict(width=12, height=8, depth=6, text_length=26) if variant == "cog" else dict(width=13, height=6, depth=7)
    mods = [vblade.AdaptiveBlockSparseAttn(variant, log_every=0, gather_kv=gk, **kw) for gk in (True, False)]
    L = mods[0].gilbert_rearranger.seq_len
    g = torch.Generator(device=DEV).manual_seed(21)
    q, k, v = (torch.randn(1, 4, L, D, generator=g, device=DEV).bfloat16() for _ in range(3))
    outs = []
    with torch.no_grad():
        for m in mods:
            torch.manual_seed(9)
            outs.append(m(q, k, v))
    torch.cuda.synchronize()
    assert torch.equal(mods[0].last_mask, mods[1].last_mask)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("variant,D", [("cog", 64), ("wan", 128)])
def test_module_takes_the_processors_strided_layout(variant, D):
    """The diffusers processors hand inner_attention views `[B,L,H,D].transpose(1, 2)` (row stride
    H*D, not D). Every kernel reads through strides (sampled rows, pooled pass, gathered K/V), so
    the module's output on those views must equal its output on contiguous copies, bit for bit."""
    import vblade
    kw = dict(width=12, height=8, depth=6, text_length=26) if variant == "cog" else dict(width=13, height=6, depth=7)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **kw)
    L = m.gilbert_rearranger.seq_len
    H = 3
    g = torch.Generator(device=DEV).manual_seed(33)
    q, k, v = (torch.randn(1, L, H, D, generator=g, device=DEV).bfloat16().transpose(1, 2) for _ in range(3))
    assert not q.is_contiguous()
    outs, masks = [], []
    with torch.no_grad():
        for args in ((q, k, v), tuple(t.contiguous() for t in (q, k, v))):
            torch.manual_seed(5)
            outs.append(m(*args))
            masks.append(m.last_mask.clone())
    torch.cuda.synchronize()
    assert torch.equal(masks[0], masks[1])
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("variant,D", [("cog", 64), ("wan", 128)])
def test_batched_call_equals_per_sample_calls(variant, D):
    """Classifier-free guidance runs the module on B=2 (and TDM training on B=5). With the same
    sampled offsets, the batched call equals one call per batch element, bit for bit: the batch
    index only selects slices (no cross-batch reduction anywhere on the path)."""
    import vblade
    from vblade import attention
    kw = dict(width=12, height=8, depth=6, text_length=26) if variant == "cog" else dict(width=13, height=6, depth=7)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **kw)
    L = m.gilbert_rearranger.seq_len
    B, H = 2, 3
    g = torch.Generator(device=DEV).manual_seed(44)
    q, k, v = (torch.randn(B, H, L, D, generator=g, device=DEV).bfloat16() for _ in range(3))
    q_off, k_off = attention.draw_sample_offsets_qk(B, H, DEV, generator=g)
    with torch.no_grad():
        out = m(q, k, v, q_off=q_off, k_off=k_off)
        mask = m.last_mask.clone()
        for b in range(B):
            sl = slice(b, b + 1)
            ob = m(q[sl], k[sl], v[sl], q_off=q_off[sl], k_off=k_off[sl])
            assert torch.equal(m.last_mask, mask[sl])
            assert torch.equal(ob, out[sl])


def test_full_size_wan_gather_path_is_deterministic():
    """The default Wan call (gathered K/V rows, fused sampling + pooling launch) at the real sequence
    length returns bit-identical outputs on repeated calls with the same RNG state."""
    import vblade
    m = vblade.AdaptiveBlockSparseAttn("wan", log_every=0)
    L = m.gilbert_rearranger.seq_len
    q, k, v = (t.to(DEV) for t in _realistic_qkv(1, 2, L, 128, seed=8))
    outs = []
    with torch.no_grad():
        for _ in range(2):
            torch.manual_seed(12)
            outs.append(m(q, k, v))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("variant", ["cog", "wan"])
def test_patched_processor_end_to_end_through_hip_module(variant):
    """a11 on the GPU: the setter patches a fake transformer, the block's processor runs the
    projections/norm/RoPE around the HIP module, and the result equals the same processor with
    the oracle's adaptive path (same mask) as inner_attention."""
    import torch.nn as nn
    import vblade
    from test_patch import FakeAttention, _rope_tables

    heads, hd = 2, (64 if variant == "cog" else 128)
    dim = heads * hd
    geo = dict(width=12, height=8, depth=6, log_every=0)
    text = 26 if variant == "cog" else 0

    class Block(nn.Module):
        def __init__(self):
            super().__init__()
            self.attn1 = FakeAttention(dim, heads, qk_norm="head" if variant == "cog" else "full")

    model = nn.Module()
    blocks = nn.ModuleList([Block(), Block()])
    if variant == "cog":
        model.transformer_blocks = blocks
        inner = vblade.set_block_sparse_attn_cogvideox(model, text_length=text, **geo)
    else:
        model.blocks = blocks
        inner = vblade.set_adaptive_block_sparse_attn_wanx(model, **geo)
    model = model.to(DEV).to(torch.bfloat16)
    attn = blocks[0].attn1
    N = 12 * 8 * 6
    g = torch.Generator().manual_seed(9)
    hidden = torch.randn(1, N, dim, generator=g).to(DEV, torch.bfloat16)
    cos_sin, freqs = _rope_tables(N, hd)
    with torch.no_grad():
        if variant == "cog":
            enc = torch.randn(1, text, dim, generator=g).to(DEV, torch.bfloat16)
            rope = tuple(t.to(DEV) for t in cos_sin)
            got = attn.processor(attn, hidden, enc, image_rotary_emb=rope)[0]
        else:
            got = attn.processor(attn, hidden, None, rotary_emb=freqs.to(DEV))
        mask = inner.last_mask.bool().cpu()
        cfg = (O.AdaptiveConfig.cogvideox(width=12, height=8, depth=6, text_length=text)
               if variant == "cog" else O.AdaptiveConfig.wan(width=12, height=8, depth=6))

        class OracleInner(nn.Module):
            def forward(self, q, k, v):
                r = O.adaptive_attention(q.cpu(), k.cpu(), v.cpu(), cfg, None, None, mask=mask,
                                         store_dtype=torch.bfloat16)["out"]
                return r.to(q.device, q.dtype)

        for b in blocks:
            b.attn1.inner_attention = OracleInner()
        if variant == "cog":
            ref = attn.processor(attn, hidden, enc, image_rotary_emb=rope)[0]
        else:
            ref = attn.processor(attn, hidden, None, rotary_emb=freqs.to(DEV))
    assert psnr(got.float().cpu(), ref.float().cpu()) >= 40


@pytest.mark.parametrize("grad", [False, True])
def test_mask_head_mode_shared_head0_reads_head0_mask(grad):
    """head_mask_type = ones(H) (:313) read literally gives every head
    base_blockmask head 0. The module's shared_head0 mode on a per-head mask equals the default
    per_head mode on a mask whose every head is head 0's, bit for bit (fused inference and the
    training path's forward and gradients)."""
    z = np.load(os.path.join(GOLDEN, "adaptive_e2e.npz"))
    case = "cog_f16"
    q, k, v = (torch.from_numpy(z[case + s]).to(torch.float16).to(DEV) for s in ("_q", "_k", "_v"))
    B, H, L, D = q.shape
    nb = (L + 127) // 128
    g = torch.Generator().manual_seed(7)
    bm = (torch.rand(B, H, nb, nb, generator=g) < 0.4).to(DEV)
    bm[..., :, -1] = True
    head0 = bm[:, :1].expand(B, H, nb, nb).contiguous()
    outs, grads = [], []
    for mode, mask in (("shared_head0", bm), ("per_head", head0)):
        m, _ = _module_for(z, case, "fused")
        m.mask_head_mode = mode
        qq, kk, vv = (t.clone().requires_grad_(grad) for t in (q, k, v))
        with torch.set_grad_enabled(grad):
            out = m(qq, kk, vv, block_mask=mask)
            if grad:
                out.float().square().sum().backward()
                grads.append([t.grad for t in (qq, kk, vv)])
        outs.append(out.detach())
        assert torch.equal(m.last_mask.bool(), mask.bool())   # the statistic sees the predicted mask
    assert torch.equal(outs[0], outs[1])
    if grad:
        for a, b in zip(*grads):
            assert torch.equal(a, b)


def test_reference_signature_mask_head_mode():
    """block_sparse_attn_func with head_mask_type = ones(H): shared_head0 equals per_head on a
    base_blockmask whose every head is head 0's (forward and backward, bit for bit), and differs
    from per_head on the per-head mask."""
    import vblade
    H, D, Lq = 3, 64, 400
    g = torch.Generator().manual_seed(3)
    q, k, v = (torch.randn(Lq, H, D, generator=g).to(torch.bfloat16).to(DEV) for _ in range(3))
    cu = torch.tensor([0, Lq], dtype=torch.int32, device=DEV)
    nb = (Lq + 127) // 128
    base = (torch.rand(1, H, nb, nb, generator=g) < 0.5)
    base[..., -1] = True
    base[:, 1:] = ~base[:, :1]
    base[..., -1] = True
    hmt = torch.ones(H, dtype=torch.int32, device=DEV)
    res = {}
    for name, mode, b in (("shared", "shared_head0", base), ("per0", "per_head", base[:, :1].repeat(1, H, 1, 1)),
                          ("per", "per_head", base)):
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
        out = vblade.block_sparse_attn_func(qq, kk, vv, cu, cu, hmt, None, b.to(DEV), Lq, Lq, 0.0,
                                            deterministic=True, mask_head_mode=mode)
        out.float().square().sum().backward()
        res[name] = (out.detach(), qq.grad, kk.grad, vv.grad)
    for a, b in zip(res["shared"], res["per0"]):
        assert torch.equal(a, b)
    assert not torch.equal(res["shared"][0], res["per"][0])
    with pytest.raises(ValueError, match="mask_head_mode"):
        vblade.block_sparse_attn_func(q, k, v, cu, cu, hmt, None, base.to(DEV), Lq, Lq, 0.0,
                                      mask_head_mode="head0")
