"""GPU parity: the HIP forward path (through the C ABI) against the oracle on the same inputs.

Tolerances (bf16/fp16 inputs, fp32 accumulate; the oracle computes in fp64):
  attention outputs   max|err| <= 2.5e-2 (bf16) / 4e-3 (fp16) on O(1) outputs,
                      PSNR >= 40 dB (BASELINE.json north_star)
  LSE                 max|err| <= 2e-3 (natural log, fp32 out)
  pooled scores / pooled K,V / combine: storage-dtype rounding of the reference reproduced;
                      differences limited to single-ulp flips from fp32 summation order.
"""
import math
import os

import numpy as np
import pytest
import torch

import bsa_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rand(*shape, dtype=torch.bfloat16, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    peak = ref.double().abs().max().item()
    return 99.0 if mse == 0 else 10 * math.log10(peak * peak / mse)


def _tol(dtype):
    return 2.5e-2 if dtype == torch.bfloat16 else 4e-3


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vblade
    vblade.load_library()


def _ops():
    from vblade import ops
    return ops


@pytest.mark.parametrize("L,D,dtype", [(128, 64, torch.bfloat16), (300, 64, torch.bfloat16),
                                       (1000, 128, torch.bfloat16), (517, 64, torch.float16),
                                       (260, 128, torch.float16)])
def test_dense_matches_oracle_and_sdpa(L, D, dtype):
    q, k, v = (_rand(1, 2, L, D, dtype=dtype, seed=s) for s in range(3))
    out, lse = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), need_lse=True)
    ref, ref_lse = O.block_sparse_attention(q, k, v, None)
    assert (out.float().cpu() - ref).abs().max() <= _tol(dtype)
    assert (lse.cpu() - ref_lse).abs().max() <= 2e-3
    sd = torch.nn.functional.scaled_dot_product_attention(q.to(DEV), k.to(DEV), v.to(DEV))
    assert psnr(out.float().cpu(), sd.float().cpu()) >= 40


@pytest.mark.parametrize("B,H,L,D,density", [(2, 3, 1000, 64, 0.3), (1, 4, 17776 // 8, 64, 0.5),
                                             (1, 2, 1500, 128, 0.2), (2, 2, 640, 64, 0.05)])
def test_block_mask_matches_oracle(B, H, L, D, density):
    q, k, v = (_rand(B, H, L, D, seed=10 + s) for s in range(3))
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(B, H, nb, nb, density, seed=L)
    out, lse = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV),
                                    need_lse=True)
    ref, ref_lse = O.block_sparse_attention(q, k, v, mask)
    assert (out.float().cpu() - ref).abs().max() <= _tol(torch.bfloat16)
    assert (lse.cpu() - ref_lse).abs().max() <= 2e-3
    assert psnr(out.float().cpu(), ref) >= 40


def test_empty_row_outputs_zero_and_neg_inf_lse():
    q, k, v = (_rand(1, 1, 384, 64, seed=s) for s in range(3))
    mask = torch.ones(1, 1, 3, 3, dtype=torch.bool)
    mask[0, 0, 1] = False
    out, lse = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV),
                                    need_lse=True)
    assert torch.all(out[0, 0, 128:256] == 0)
    assert torch.all(torch.isneginf(lse[0, 0, 128:256]))
    ref, _ = O.block_sparse_attention(q, k, v, mask)
    assert (out.float().cpu()[0, 0, :128] - ref[0, 0, :128]).abs().max() <= 2.5e-2


def test_reference_signature_empty_row_lse_is_pos_inf():
    """block_sparse_attn_func (the FlashAttention-2-based op) reports +inf LSE for a query row
    with no kept key block and a zero output row; the module path keeps -inf (above)."""
    import vblade
    q, k, v = (_rand(384, 1, 64, seed=s) for s in range(3))
    mask = torch.ones(1, 1, 3, 3, dtype=torch.bool)
    mask[0, 0, 1] = False
    cu = torch.tensor([0, 384], dtype=torch.int32, device=DEV)
    out, lse, _ = vblade.block_sparse_attn_func(
        q.to(DEV), k.to(DEV), v.to(DEV), cu, cu, torch.ones(1, dtype=torch.int32, device=DEV),
        None, mask.to(DEV), 384, 384, 0.0, deterministic=True, return_attn_probs=True)
    assert torch.all(out[128:256] == 0)
    assert torch.all(torch.isposinf(lse[0, 0, 128:256]))
    assert torch.all(torch.isfinite(lse[0, 0, :128]))


def test_online_softmax_rescale_branch_is_exercised():
    """Spike one key late in the key order so the running max jumps (guide §5.4 rule 26)."""
    q, k, v = (_rand(1, 1, 700, 64, seed=20 + s) for s in range(3))
    k[0, 0, 650] = q[0, 0, 5] * 4   # query 5's max jumps at the last tile
    k[0, 0, 64] = -q[0, 0, 70] * 3
    out = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV))
    ref, _ = O.block_sparse_attention(q, k, v, None)
    assert (out.float().cpu() - ref).abs().max() <= 2.5e-2


@pytest.mark.parametrize("D", [64, 128])
def test_huge_late_scores_rescale_both_kernels(D):
    """Scores ~100-300 log2-units above the first tile's max (keys = 6-20 x a query) in the first
    and second 32-key half of a tile, in the tail tile and for several queries of one wave.
    need_lse=True runs the training kernel (unscaled Q): exact to bf16 rounding. The inference
    kernel (kCBias: Q pre-scaled by scale*log2(e) and rounded to bf16) is checked against the
    oracle run on that same pre-scaled query, and against the exact oracle by PSNR: with keys of
    this norm the pre-scale rounding alone moves outputs by ~3 bf16 ulps."""
    L = 700
    q, k, v = (_rand(1, 1, L, D, seed=40 + s) for s in range(3))
    for qi, ki, mult in ((5, 650, 12.0), (6, 300, 12.0), (7, 690, 14.0), (40, 70, 12.0),
                         (41, 200, 6.0), (130, 10, 20.0)):
        k[0, 0, ki] = q[0, 0, qi] * mult
    ref, _ = O.block_sparse_attention(q, k, v, None)
    out_t, _ = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), need_lse=True)
    assert (out_t.float().cpu() - ref).abs().max() <= 2.5e-2
    out = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV)).float().cpu()
    assert torch.isfinite(out).all()
    qs = (q.float() * (D ** -0.5 * 1.4426950408889634)).to(q.dtype)
    ref_s, _ = O.block_sparse_attention(qs, k, v, None, sm_scale=math.log(2.0))
    assert (out - ref_s).abs().max() <= 2.5e-2
    assert psnr(out, ref) >= 40


def test_row_index_gather_scatter_equals_permuted_oracle():
    B, H, L, D = 1, 2, 900, 64
    q, k, v = (_rand(B, H, L, D, seed=30 + s) for s in range(3))
    g = torch.Generator().manual_seed(4)
    P = torch.randperm(L, generator=g)
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(B, H, nb, nb, 0.4, seed=9)
    out, lse = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV),
                                    q_rows=P.int().to(DEV), kv_rows=P.int().to(DEV), need_lse=True)
    ref_r, lse_r = O.block_sparse_attention(q[:, :, P], k[:, :, P], v[:, :, P], mask)
    ref = torch.empty_like(ref_r)
    ref[:, :, P] = ref_r
    ref_lse = torch.empty_like(lse_r)
    ref_lse[:, :, P] = lse_r
    assert (out.float().cpu() - ref).abs().max() <= 2.5e-2
    assert (lse.cpu() - ref_lse).abs().max() <= 2e-3


def test_strided_views_need_no_copy():
    """q/k as [B,L,H,D] storage viewed as [B,H,L,D] (the processors' transpose(1,2))."""
    B, L, H, D = 1, 400, 3, 64
    qs, ks, vs = (_rand(B, L, H, D, seed=40 + s) for s in range(3))
    q, k, v = (t.to(DEV).transpose(1, 2) for t in (qs, ks, vs))
    assert not q.is_contiguous()
    out = _ops().attention_fwd(q, k, v)
    ref, _ = O.block_sparse_attention(qs.transpose(1, 2), ks.transpose(1, 2), vs.transpose(1, 2), None)
    assert (out.float().cpu() - ref).abs().max() <= 2.5e-2


@pytest.mark.parametrize("D,gap", [(64, 15), (128, 30)])
def test_fused_pooled_branch_equals_joint_softmax(D, gap):
    B, H, L = 1, 2, 1100
    q, k, v = (_rand(B, H, L, D, seed=50 + s) for s in range(3))
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(B, H, nb, nb, 0.25, seed=3)
    kp = O.simple_pooling(k, gap)
    vp = O.simple_pooling(v, gap)
    out, lse = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV),
                                    kp=kp.to(DEV), vp=vp.to(DEV), kp_log_bias=math.log(gap),
                                    need_lse=True)
    o1, l1 = O.block_sparse_attention(q, k, v, mask)
    o2, l2 = O.block_sparse_attention(q, kp, vp, None, key_bias=math.log(gap))
    lj = torch.logaddexp(l1, l2)
    a = torch.exp(l1 - lj)[..., None]
    ref = o1 * a + o2 * (1 - a)
    assert (out.float().cpu() - ref).abs().max() <= 2.5e-2
    assert (lse.cpu() - lj).abs().max() <= 2e-3
    # pooled-only (the reference's standard_attn call, bias 0)
    out2, lse2 = _ops().attention_fwd(q.to(DEV), None, None, use_main=False, kp=kp.to(DEV),
                                      vp=vp.to(DEV), need_lse=True)
    r2, rl2 = O.block_sparse_attention(q, kp, vp, None)
    assert (out2.float().cpu() - r2).abs().max() <= 2.5e-2
    assert (lse2.cpu() - rl2).abs().max() <= 2e-3


def test_reference_signature_varlen_and_head_mask_type():
    """block_sparse_attn_func(q_unpad, ..., head_mask_type, ..., base_blockmask, ...) as called at
    cogvideo_blocksparseattn.py:316-320, with two sequences of different lengths, one dense head
    (type 0) and two block-sparse heads (type 1 -> base masks 0 and 1)."""
    import vblade
    H, D = 3, 64
    lens = [300, 555]
    cu = torch.tensor([0, 300, 855], dtype=torch.int32)
    tot = 855
    q, k, v = (_rand(tot, H, D, seed=60 + s) for s in range(3))
    nb = (max(lens) + 127) // 128
    base = O.block_mask_from_density(2, 2, nb, nb, 0.4, seed=11)
    hmt = torch.tensor([1, 0, 1], dtype=torch.int32)
    out, lse, _ = vblade.block_sparse_attn_func(
        q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV), cu.to(DEV), hmt.to(DEV),
        torch.zeros(2 * H, dtype=torch.int32, device=DEV), base.to(DEV), max(lens), max(lens), 0.0,
        deterministic=True, softmax_scale=None, is_causal=False, exact_streaming=False,
        return_attn_probs=True)
    assert lse.shape == (2, H, max(lens))
    for b, (s0, n) in enumerate(zip([0, 300], lens)):
        qb = q[s0:s0 + n].transpose(0, 1)[None]
        kb = k[s0:s0 + n].transpose(0, 1)[None]
        vb = v[s0:s0 + n].transpose(0, 1)[None]
        nbb = (n + 127) // 128
        m = torch.ones(1, H, nbb, nbb, dtype=torch.bool)
        m[0, 0] = base[b, 0, :nbb, :nbb]
        m[0, 2] = base[b, 1, :nbb, :nbb]
        ref, ref_lse = O.block_sparse_attention(qb, kb, vb, m)
        got = out[s0:s0 + n].transpose(0, 1)[None].float().cpu()
        assert (got - ref).abs().max() <= 2.5e-2
        assert (lse[b, :, :n].cpu() - ref_lse[0]).abs().max() <= 2e-3


# -------------------------------------------------------------------------------- predictor
def _exact_inputs(B, H, L, D, seed):
    """bf16 values with few mantissa bits: every fp32 partial dot product is exact, so GPU and
    CPU pooled scores agree to the bit regardless of summation order."""
    g = torch.Generator().manual_seed(seed)
    cent = torch.randint(-2, 3, (B, H, L // 64 + 1, D), generator=g).repeat_interleave(64, 2)[:, :, :L]
    x = torch.randint(-2, 3, (B, H, L, D), generator=g) + cent
    return (x.float() / 4).to(torch.bfloat16)


@pytest.mark.parametrize("variant,L,D,H", [("cog", 17776, 64, 2), ("wan", 32760, 128, 1),
                                          ("cog", 1000, 64, 3),
                                          ("wan", 40960, 128, 1)])   # the largest supported: nb = 320
def test_mask_predict_matches_oracle(variant, L, D, H):
    import vblade
    from vblade.attention import retain_counts
    B = 1
    q = _exact_inputs(B, H, L, D, 1)
    k = _exact_inputs(B, H, L, D, 2)
    g = torch.Generator().manual_seed(7)
    qo = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0]
    ko = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0]
    nb = (L + 127) // 128
    mn, mx = (0.05, 0.1) if variant == "cog" else (0.05, 0.17)
    lo, hi = retain_counts(nb, mn, mx, variant)
    ft = 2 if variant == "cog" else 0
    perm = torch.randperm(L, generator=g)
    cnt = torch.zeros(1, dtype=torch.int64, device=DEV)
    po, mask = _ops().mask_predict(q.to(DEV), k.to(DEV), qo.int().to(DEV), ko.int().to(DEV),
                                   rows=perm.int().to(DEV), min_keep=lo, max_keep=hi,
                                   force_tail=ft, mask_count=cnt)
    qr, kr = q[:, :, perm], k[:, :, perm]
    qs = O.sample_tokens(O.pad_replicate(qr, 128), qo)
    ks = O.sample_tokens(O.pad_replicate(kr, 128), ko)
    ref_po = O.pooled_scores(qs, ks, 1.0 / D ** 0.5, 32, torch.bfloat16)
    po_c = po.float().cpu()
    exact = (po_c == ref_po).float().mean().item()
    assert exact >= 0.999, exact
    assert (po_c - ref_po).abs().max().item() <= 2 ** -7
    # the energy rule applied by the oracle to the GPU's own scores reproduces the GPU mask exactly
    ref_mask = O.energy_mask(po_c, lo, hi, 0.95, ft)
    assert torch.equal(mask.bool().cpu(), ref_mask)
    assert cnt.item() == int(ref_mask.sum())
    del vblade


@pytest.mark.parametrize("case,variant,ft", [("cog", "cog", 2), ("wan", "wan", 0), ("cog_small", "cog", 2)])
def test_energy_mask_kernel_on_reference_goldens(case, variant, ft):
    from vblade.attention import retain_counts
    z = np.load(os.path.join(GOLDEN, "energy_masks.npz"))
    po = torch.from_numpy(z[case + "_po"]).bfloat16()
    nb = po.shape[-1]
    lo, hi = retain_counts(nb, 0.05, 0.1 if variant == "cog" else 0.17, variant)
    m = _ops().energy_mask(po.to(DEV), min_keep=lo, max_keep=hi, force_tail=ft).bool().cpu()
    assert torch.equal(m, O.energy_mask(po, lo, hi, 0.95, ft))
    k = O.energy_keep_counts(po, lo, hi)
    assert O.mask_is_valid_topk(torch.from_numpy(z[case + "_mask"]), po, k, ft)
    assert O.mask_is_valid_topk(m, po, k, ft)


@pytest.mark.parametrize("L,gap,D", [(17776, 15, 64), (1000, 30, 128), (33, 15, 64)])
def test_pool_kv_matches_oracle(L, gap, D):
    k, v = _rand(2, 2, L, D, seed=70), _rand(2, 2, L, D, seed=71)
    perm = torch.randperm(L, generator=torch.Generator().manual_seed(1))
    kp, vp = _ops().pool_kv(k.to(DEV), v.to(DEV), gap, rows=perm.int().to(DEV))
    rk = O.simple_pooling(k[:, :, perm], gap).float()
    rv = O.simple_pooling(v[:, :, perm], gap).float()
    for got, ref in ((kp, rk), (vp, rv)):
        got = got.float().cpu()
        ulp = ref.abs().clamp_min(2 ** -126) * 2 ** -7
        assert torch.all((got - ref).abs() <= ulp + 1e-30)
        assert (got == ref).float().mean() >= 0.99


@pytest.mark.parametrize("B,H,L,gap,with_rows", [(1, 3, 1237, 1, True), (1, 3, 1237, 7, False), (1, 3, 1237, 8, True),
                                                (1, 3, 1237, 9, False), (1, 3, 1237, 16, True), (1, 3, 1237, 30, False),
                                                (2, 24, 17776, 1, True), (2, 24, 17776, 15, False)])
def test_pool_kv_pipeline_steps_and_copies(B, H, L, gap, with_rows):
    """The pooled pass's pipelined steps (vb_pool.hpp: groups of 8 rows, the next step's rows entries
    loaded one step ahead, two entry sets): gaps below, at and above the group size, with and without
    the row table; the two large shapes give every thread several items (the launch is capped at
    kPoolWgsDefault workgroups), so steps chain across items. The Gilbert-order copies are exact."""
    D = 64
    k, v = _rand(B, H, L, D, seed=72), _rand(B, H, L, D, seed=73)
    perm = torch.randperm(L, generator=torch.Generator().manual_seed(2))
    rows = perm.int().to(DEV) if with_rows else None
    kp, vp, k_r, v_r = _ops().pool_kv(k.to(DEV), v.to(DEV), gap, rows=rows, reordered=True)
    src_k, src_v = (k[:, :, perm], v[:, :, perm]) if with_rows else (k, v)
    assert torch.equal(k_r.cpu(), src_k) and torch.equal(v_r.cpu(), src_v)
    for got, x in ((kp, src_k), (vp, src_v)):
        ref = O.simple_pooling(x, gap).float()
        got = got.float().cpu()
        ulp = ref.abs().clamp_min(2 ** -126) * 2 ** -7
        assert torch.all((got - ref).abs() <= ulp + 1e-30)
        assert (got == ref).float().mean() >= 0.99


def test_lse_combine_matches_reference_rounding():
    B, H, L, D = 2, 3, 333, 64
    o1, o2 = _rand(B, H, L, D, seed=80), _rand(B, H, L, D, seed=81)
    l1 = torch.randn(B, H, L) * 3 + 5
    l2 = torch.randn(B, H, L) * 3 + 3
    out, alpha = _ops().lse_combine(o1.to(DEV), l1.to(DEV), o2.to(DEV), l2.to(DEV), 15)
    ref, ra = O.combine_reference(o1, l1, o2, l2, 15)
    assert (alpha.cpu() - ra[..., 0]).abs().max() <= 2 ** -8
    assert ((out.float().cpu() - ref).abs() <= ref.abs() * 2 ** -7 + 2 ** -14).all()
    assert (out.float().cpu() == ref).float().mean() >= 0.99


@pytest.mark.parametrize("variant,H,D", [("cog", 48, 64), ("wan", 12, 128)])
def test_forward_is_bitwise_deterministic_at_full_size(variant, H, D):
    """Repeated launches on identical inputs give identical bits (no read of an MFMA result or LDS
    slot before it is ready). Full CogVideoX / Wan shapes, so every tile/tail path runs."""
    import vblade
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    g = torch.Generator(device=DEV).manual_seed(11)
    q, k, v = (torch.randn(1, H, L, D, generator=g, device=DEV).to(torch.bfloat16) for _ in range(3))
    with torch.no_grad():
        outs = [m(q, k, v, q_off=torch.zeros(1, H, 32, dtype=torch.int32, device=DEV) + torch.arange(32, dtype=torch.int32, device=DEV),
                  k_off=torch.zeros(1, H, 32, dtype=torch.int32, device=DEV) + torch.arange(32, dtype=torch.int32, device=DEV))
                for _ in range(4)]
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("variant,H,D", [("cog", 48, 64), ("wan", 12, 128)])
def test_longest_first_dispatch_order_is_bit_identical(variant, H, D):
    """Round 5 scheduling: with ``order`` the attention launch dispatches each XCD's q-blocks head by
    head, most kept key blocks first (vb_attn_args.q_order; lengths from the predictor's
    mask_rows_kept or counted on the device). Outputs must equal the kernel's own order bit for
    bit, and the predictor's kept counts must equal the mask rows' counts."""
    import vblade
    from vblade import ops
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    g = torch.Generator(device=DEV).manual_seed(5)
    q, k, v = (torch.randn(1, H, L, D, generator=g, device=DEV).to(torch.bfloat16) for _ in range(3))
    offs = torch.zeros(1, H, 32, dtype=torch.int32, device=DEV) + torch.arange(32, dtype=torch.int32, device=DEV)
    with torch.no_grad():
        m.order = False
        ref = m(q, k, v, q_off=offs, k_off=offs)
        m.order = True
        got = m(q, k, v, q_off=offs, k_off=offs)
        assert torch.equal(got, ref)
        # the predictor's kept counts are the mask rows' counts
        nb = (L + 127) // 128
        kept = torch.full((1, H, nb), -1, dtype=torch.int32, device=DEV)
        _, mask = m.predict_mask(q, k, offs, offs, rows_kept=kept)
        assert torch.equal(kept, (mask != 0).sum(-1).to(torch.int32))
        # the op level: lengths counted on the device, and given
        rows = m._rows(q.device)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
        kw = dict(block_mask=mask, q_rows=rows, kp=kp, vp=vp, kp_log_bias=m._log_gap(q.dtype),
                  heavy_rows=m.force_tail)
        a = ops.attention_fwd(q, k_r, v_r, **kw)
        b = ops.attention_fwd(q, k_r, v_r, order=True, **kw)
        c = ops.attention_fwd(q, k_r, v_r, order=True, q_lengths=kept, **kw)
        assert torch.equal(a, b) and torch.equal(a, c)
        # the permutation itself (attn_order_kernel), restated: per XCD range of the non-heavy
        # rows, a permutation of the range whose (head, -kept) keys never decrease (equal keys may
        # come in any order: the bins are filled with LDS atomics); with a window, the range's
        # first count - window items keep their place
        kc = kept.view(-1).cpu()
        hr = min(m.force_tail, nb)
        rows_left = nb - hr
        nwg = rows_left * H
        q8, r8 = nwg // 8, nwg % 8
        for window in (0, 16):
            qo = torch.full((H * nb,), -1, dtype=torch.int32, device=DEV)
            ops.attention_fwd(q, k_r, v_r, order=True, q_lengths=kept, order_window=window, q_order_out=qo, **kw)
            qo = qo.cpu()
            for x in range(8):
                start = x * (q8 + 1) if x < r8 else r8 * (q8 + 1) + (x - r8) * q8
                count = q8 + (1 if x < r8 else 0)
                skip = count - window if 0 < window < count else 0
                seg = qo[start:start + count].tolist()
                assert sorted(seg) == list(range(start, start + count)), (x, "not a permutation")
                assert seg[:skip] == list(range(start, start + skip))
                def key(lin):
                    bh, qb = lin // rows_left, rows_left - 1 - lin % rows_left
                    return (bh, -int(kc[bh * nb + qb]))
                keys = [key(lin) for lin in seg[skip:]]
                assert keys == sorted(keys), (x, "not longest first within each head")


@pytest.mark.parametrize("variant,H,D", [("cog", 8, 64), ("wan", 4, 128)])
def test_persistent_dispatch_is_bit_identical(variant, H, D):
    """Round 6 scheduling: with ``persistent`` the attention launch is resident-sized and its
    workgroups pull q-blocks from per-XCD queues (vb_attn_args.work_queue), then from the other
    XCDs' queues. Every launch form (module, op with and without the longest-first order, gathered
    K/V, the LSE-returning training launch) gives the one-workgroup-per-q-block bits, the queue is
    zero again after every launch, and two streams with their own queues run concurrently."""
    import vblade
    from vblade import ops
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    g = torch.Generator(device=DEV).manual_seed(11)
    q, k, v = (torch.randn(1, H, L, D, generator=g, device=DEV).to(torch.bfloat16) for _ in range(3))
    offs = torch.zeros(1, H, 32, dtype=torch.int32, device=DEV) + torch.arange(32, dtype=torch.int32, device=DEV)
    with torch.no_grad():
        m.persistent = False
        ref = m(q, k, v, q_off=offs, k_off=offs)
        m.persistent = True
        for _ in range(3):
            assert torch.equal(m(q, k, v, q_off=offs, k_off=offs), ref)
        rows = m._rows(q.device)
        _, mask = m.predict_mask(q, k, offs, offs)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
        kw = dict(block_mask=mask, q_rows=rows, kp=kp, vp=vp, kp_log_bias=m._log_gap(q.dtype),
                  heavy_rows=m.force_tail)
        a = ops.attention_fwd(q, k_r, v_r, **kw)
        for order in (False, True):
            assert torch.equal(ops.attention_fwd(q, k_r, v_r, order=order, persistent=True, **kw), a)
        assert torch.equal(ops.attention_fwd(q, k, v, kv_rows=rows, persistent=True, **kw),
                           ops.attention_fwd(q, k, v, kv_rows=rows, **kw))
        o1, l1 = ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True)
        o2, l2 = ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True, persistent=True)
        assert torch.equal(o1, o2) and torch.equal(l1, l2)
        assert int(ops.work_queue(q.device).abs().sum()) == 0
        # two streams, each its own queue, launched back to back so they overlap
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        outs = []
        for st in (s1, s2):
            with torch.cuda.stream(st):
                outs.append(ops.attention_fwd(q, k_r, v_r, persistent=True, **kw))
        torch.cuda.synchronize()
        assert all(torch.equal(o, a) for o in outs)
        for st in (s1, s2):
            with torch.cuda.stream(st):
                assert int(ops.work_queue(q.device).abs().sum()) == 0


def test_order_launch_sorts_by_length_when_a_range_spans_too_many_heads():
    """attn_order_kernel bins (head, kept) keys in LDS; an XCD range spanning more heads than the
    bins hold (here 2752 heads x 3 lengths > 8192) is sorted by kept count alone (longest first over
    the range). Outputs stay bit-identical and each range is a permutation in that order."""
    from vblade import ops
    B, H, L, D = 4, 5504, 256, 64
    g = torch.Generator(device=DEV).manual_seed(3)
    q, k, v = (torch.randn(B, H, L, D, generator=g, device=DEV).to(torch.bfloat16) for _ in range(3))
    mask = (torch.rand(B, H, 2, 2, generator=g, device=DEV) < 0.5)
    mask[..., 0] = True
    mask = mask.to(torch.uint8)
    with torch.no_grad():
        a = ops.attention_fwd(q, k, v, block_mask=mask)
        qo = torch.full((B * H * 2,), -1, dtype=torch.int32, device=DEV)
        b = ops.attention_fwd(q, k, v, block_mask=mask, order=True, q_order_out=qo)
        assert torch.equal(a, b)
    kept = (mask != 0).sum(-1).view(-1).cpu()
    qo = qo.cpu()
    nwg = B * H * 2
    q8, r8 = nwg // 8, nwg % 8
    for x in range(8):
        start = x * (q8 + 1) if x < r8 else r8 * (q8 + 1) + (x - r8) * q8
        count = q8 + (1 if x < r8 else 0)
        seg = qo[start:start + count]
        assert torch.equal(seg.sort().values, torch.arange(start, start + count, dtype=torch.int32))
        bh, qb = seg // 2, 1 - seg % 2
        lens = kept[bh * 2 + qb]
        assert bool((lens[:-1] >= lens[1:]).all()), (x, "not longest first")


def test_sample_offsets_match_torch_topk_and_rng_order():
    """vb_sample_offsets == torch.topk(rand, 32).indices (the reference's random_sample_tokens,
    :45-46), and the module draws q then k from the same generator stream as the reference."""
    from vblade import attention, ops
    g = torch.Generator(device=DEV).manual_seed(123)
    rq = torch.rand(2, 5, 1, 128, device=DEV, generator=g)
    rk = torch.rand(2, 5, 1, 128, device=DEV, generator=g)
    oq, ok = ops.sample_offsets(rq, rk, 32)
    assert torch.equal(oq.long(), torch.topk(rq, 32, dim=3).indices)
    assert torch.equal(ok.long(), torch.topk(rk, 32, dim=3).indices)
    g1 = torch.Generator(device=DEV).manual_seed(7)
    q_off, k_off = attention.draw_sample_offsets_qk(2, 5, DEV, generator=g1)
    g2 = torch.Generator(device=DEV).manual_seed(7)
    ref_q = attention.draw_sample_offsets(2, 5, DEV, generator=g2)
    ref_k = attention.draw_sample_offsets(2, 5, DEV, generator=g2)
    assert torch.equal(q_off, ref_q) and torch.equal(k_off, ref_k)


@pytest.mark.parametrize("B,H,L,D,pre", [(1, 2, 1000, 64, 0), (2, 48, 17776, 64, 3000),
                                          (1, 12, 32760, 128, 700000), (5, 48, 4096, 64, 17)])
def test_philox_draws_in_the_sampling_launch_equal_torch_rand(B, H, L, D, pre):
    """The two draws generated inside the sampling launch (vb_predict_args.philox) are the values
    torch.rand(B,H,1,128) returns twice on the device's default generator (q first): the scores and
    mask equal those of the same launch given torch.topk(torch.rand(...)) offsets, and the generator
    ends at the same state. ``pre`` draws before move the Philox offset off zero (700000 > one
    grid-stride pass of torch.rand: the offset advances by more than 4)."""
    from vblade import ops
    g = torch.Generator().manual_seed(B * 1000 + H)
    q = torch.randn(B, H, L, D, generator=g).to(torch.bfloat16).to(DEV)
    k = torch.randn(B, H, L, D, generator=g).to(torch.bfloat16).to(DEV)
    kw = dict(energy_threshold=0.9, min_keep=2, max_keep=(L + 127) // 128, force_tail=1)

    torch.manual_seed(41)
    if pre:
        torch.rand(pre, device=DEV)
    rq = torch.rand(B, H, 1, 128, device=DEV)
    rk = torch.rand(B, H, 1, 128, device=DEV)
    after_ref = torch.rand(7, device=DEV)
    q_off = torch.topk(rq, 32, dim=3).indices[:, :, 0].to(torch.int32)
    k_off = torch.topk(rk, 32, dim=3).indices[:, :, 0].to(torch.int32)
    po_ref, mask_ref = ops.mask_predict(q, k, q_off, k_off, **kw)

    torch.manual_seed(41)
    if pre:
        torch.rand(pre, device=DEV)
    philox = ops.claim_rand_draws(DEV, B * H * 128)
    assert philox is not None
    po, mask = ops.mask_predict(q, k, philox=philox, **kw)
    after = torch.rand(7, device=DEV)
    assert torch.equal(after, after_ref)
    assert torch.equal(po, po_ref) and torch.equal(mask, mask_ref)


def test_philox_claim_declines_draws_past_one_pass():
    from vblade import ops
    assert ops.claim_rand_draws(DEV, ops.RAND_ONE_PASS_NUMEL + 128) is None


def test_module_call_captures_into_a_hip_graph_with_torch_rand_draws():
    """Under HIP-graph capture the module keeps torch.rand (graph-safe per-replay offsets) instead of
    the in-kernel draws, and a captured call replays: finite outputs of the right shape, and the
    graph's outputs equal an eager call's given the same mask."""
    import vblade
    from vblade import ops
    m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0, width=8, height=6, depth=10,
                                       text_length=30, min_retain_ratio=0.2, max_retain_ratio=0.5)
    B, H, L, D = 1, 2, m.gilbert_rearranger.seq_len, 64
    g = torch.Generator().manual_seed(77)
    q, k, v = (torch.randn(B, H, L, D, generator=g).bfloat16().to(DEV) for _ in range(3))
    with torch.no_grad():
        m(q, k, v)                                   # warm up outside the capture
        torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                assert ops.claim_rand_draws(DEV, B * H * 128) is None
                out = m(q, k, v)
        torch.cuda.current_stream().wait_stream(s)
        for _ in range(2):
            graph.replay()
        torch.cuda.synchronize()
        assert out.shape == q.shape and bool(torch.isfinite(out.float()).all())
        mask = m.last_mask.clone()
        eager = m(q, k, v, block_mask=mask)
        torch.cuda.synchronize()
        assert (eager.float() - out.float()).abs().max().item() <= 2.5e-2


@pytest.mark.parametrize("n,keep", [(128, 32), (131, 32), (61, 7), (256, 256)])
def test_sample_offsets_ties_and_ragged_row_lengths(n, keep):
    """The rank loop reads four draws per LDS broadcast with a scalar tail: rows whose length is
    not a multiple of 4 and tie-heavy draws (a quarter of the values repeated) must still give the
    stable descending order (ties -> lower index first, topk_wave's rule)."""
    from vblade import ops
    g = torch.Generator().manual_seed(n * 7 + keep)
    r = torch.rand(2, 3, 2, n, generator=g)
    dup = torch.rand(2, 3, 2, n, generator=g) < 0.25
    r = torch.where(dup, torch.round(r * 8) / 8, r)              # many exact ties
    rk = torch.rand(2, 3, 2, n, generator=g)
    oq, ok = ops.sample_offsets(r.to(DEV), rk.to(DEV), keep)
    want_q = torch.from_numpy(np.argsort(-r.numpy(), axis=-1, kind="stable")[..., :keep].copy())
    want_k = torch.from_numpy(np.argsort(-rk.numpy(), axis=-1, kind="stable")[..., :keep].copy())
    assert torch.equal(oq.cpu().long(), want_q.long())
    assert torch.equal(ok.cpu().long(), want_k.long())


def test_mask_predict_rejects_sequences_past_its_block_limit():
    """nb = 321 sampled blocks exceeds the predictor's LDS row buffers: a loud error, no launch."""
    L, D = 321 * 128, 64
    q = torch.zeros(1, 1, L, D, dtype=torch.bfloat16, device=DEV)
    off = torch.arange(32, dtype=torch.int32, device=DEV).view(1, 1, 32)
    with pytest.raises(RuntimeError, match="too long"):
        _ops().mask_predict(q, q, off, off, min_keep=1, max_keep=4)


@pytest.mark.parametrize("D", [64, 128])
def test_forward_at_its_largest_key_count(D):
    """Lk = 131072 keys (1024 key blocks, the kernel's list limit). A q-block's output depends only
    on its mask row, so the oracle checks four q-blocks against their own rows; 1025 blocks raise."""
    L = 1024 * 128
    q, k, v = (_rand(1, 1, L, D, seed=80 + s) for s in range(3))
    mask = O.block_mask_from_density(1, 1, 1024, 1024, 0.01, seed=D)
    mask[0, 0, :, -1] = True   # the last key block on every row (its DMA ends at the slice's end)
    out = _ops().attention_fwd(q.to(DEV), k.to(DEV), v.to(DEV), block_mask=mask.to(DEV))
    out = out.float().cpu()
    for i in (0, 1, 511, 1023):
        rows = slice(i * 128, (i + 1) * 128)
        ref, _ = O.block_sparse_attention(q[:, :, rows], k, v, mask[:, :, i:i + 1])
        assert (out[:, :, rows] - ref).abs().max() <= _tol(torch.bfloat16)
    big = torch.zeros(1, 1, L + 128, D, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(RuntimeError, match="too long"):
        _ops().attention_fwd(big, big, big, block_mask=torch.ones(1, 1, 1025, 1025, dtype=torch.bool, device=DEV))


def test_reference_signature_varlen_with_an_empty_sequence():
    """A zero-length sequence between two others (cu_seqlens [0, 300, 300, 855]): its workgroups
    exit at once and the neighbours' rows match the oracle."""
    import vblade
    H, D = 3, 64
    starts, lens = [0, 300, 300], [300, 0, 555]
    cu = torch.tensor([0, 300, 300, 855], dtype=torch.int32)
    q, k, v = (_rand(855, H, D, seed=90 + s) for s in range(3))
    nb = (max(lens) + 127) // 128
    base = O.block_mask_from_density(3, 2, nb, nb, 0.4, seed=12)
    hmt = torch.tensor([1, 0, 1], dtype=torch.int32)
    out, lse, _ = vblade.block_sparse_attn_func(
        q.to(DEV), k.to(DEV), v.to(DEV), cu.to(DEV), cu.to(DEV), hmt.to(DEV),
        torch.zeros(3 * H, dtype=torch.int32, device=DEV), base.to(DEV), max(lens), max(lens), 0.0,
        deterministic=True, softmax_scale=None, is_causal=False, exact_streaming=False,
        return_attn_probs=True)
    for b, (s0, n) in enumerate(zip(starts, lens)):
        if n == 0:
            continue
        qb, kb, vb = (t[s0:s0 + n].transpose(0, 1)[None] for t in (q, k, v))
        nbb = (n + 127) // 128
        m = torch.ones(1, H, nbb, nbb, dtype=torch.bool)
        m[0, 0] = base[b, 0, :nbb, :nbb]
        m[0, 2] = base[b, 1, :nbb, :nbb]
        ref, ref_lse = O.block_sparse_attention(qb, kb, vb, m)
        got = out[s0:s0 + n].transpose(0, 1)[None].float().cpu()
        assert (got - ref).abs().max() <= 2.5e-2
        assert (lse[b, :, :n].cpu() - ref_lse[0]).abs().max() <= 2e-3


@pytest.mark.parametrize("B,H,L,D,heavy,window", [(2, 3, 300, 64, 0, 0), (2, 3, 1000, 128, 2, 0),
                                                  (1, 5, 777, 64, 2, 3), (3, 2, 520, 64, 9, 1000),
                                                  (1, 1, 100, 128, 0, 0)])
def test_dispatch_order_small_shapes_batches_and_windows(B, H, L, D, heavy, window):
    """The ordered launch at small, ragged, batched shapes: heavy rows beyond nbq, windows larger
    than an XCD range, ranges with one or no item. Same output as the kernel's own order (bit for
    bit) and a valid permutation of every range (head-major, longest first within a head)."""
    from vblade import ops
    q, k, v = (_rand(B, H, L, D, seed=s).to(DEV) for s in (80, 81, 82))
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(B, H, nb, nb, 0.5, seed=83).to(DEV)
    kept = (mask != 0).sum(-1).to(torch.int32).contiguous()
    ref = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy)
    qo = torch.full((B * H * nb,), -1, dtype=torch.int32, device=DEV)
    got = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy, order=True, q_lengths=kept,
                            order_window=window, q_order_out=qo)
    got2 = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy, order=True, order_window=window)
    assert torch.equal(got, ref) and torch.equal(got2, ref)
    # the persistent launch at the same shapes: fewer items than resident workgroups (most exit on
    # their first claim), ragged last q-blocks, heavy rows beyond nbq; the queue is zero afterwards
    for order in (False, True):
        got3 = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy, order=order,
                                 order_window=window, persistent=True)
        assert torch.equal(got3, ref), order
    o1, l1 = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy, need_lse=True)
    o2, l2 = ops.attention_fwd(q, k, v, block_mask=mask, heavy_rows=heavy, need_lse=True, persistent=True)
    assert torch.equal(o1, o2) and torch.equal(l1, l2)
    assert int(ops.work_queue(q.device).abs().sum()) == 0
    qo, kc = qo.cpu(), kept.view(-1).cpu()
    rows_left = nb - min(heavy, nb)
    nwg = rows_left * B * H
    q8, r8 = nwg // 8, nwg % 8
    for x in range(8):
        start = x * (q8 + 1) if x < r8 else r8 * (q8 + 1) + (x - r8) * q8
        count = q8 + (1 if x < r8 else 0)
        if count <= 0:
            continue
        skip = count - window if 0 < window < count else 0
        seg = qo[start:start + count].tolist()
        assert sorted(seg) == list(range(start, start + count)), (x, seg)
        assert seg[:skip] == list(range(start, start + skip))
        keys = [(lin // rows_left, -int(kc[(lin // rows_left) * nb + rows_left - 1 - lin % rows_left]))
                for lin in seg[skip:]]
        assert keys == sorted(keys), (x, keys)


@pytest.mark.parametrize("D,gather,lse", [(64, False, False), (64, True, True), (128, False, True),
                                          (128, True, False)])
def test_persistent_fp16_launch_forms(D, gather, lse):
    """The fp16 instantiations of the persistent forward (each launch form is a separate kernel:
    head dim, gathered or contiguous K/V, with or without the LSE): the same bits as the
    one-workgroup-per-q-block launch on ragged batched inputs with a pooled branch, and the queue
    left zero."""
    from vblade import ops
    B, H, L = 2, 3, 900
    q, k, v = (_rand(B, H, L, D, dtype=torch.float16, seed=s).to(DEV) for s in (60, 61, 62))
    nb = (L + 127) // 128
    mask = O.block_mask_from_density(B, H, nb, nb, 0.4, seed=63).to(DEV)
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(64)).to(torch.int32).to(DEV)
    kp, vp = (_rand(B, H, 60, D, dtype=torch.float16, seed=s).to(DEV) for s in (65, 66))
    kw = dict(block_mask=mask, q_rows=rows, kp=kp, vp=vp, kp_log_bias=math.log(15.0), heavy_rows=1,
              need_lse=lse)
    if gather:
        kw["kv_rows"] = rows
    ref = ops.attention_fwd(q, k, v, **kw)
    got = ops.attention_fwd(q, k, v, persistent=True, **kw)
    if lse:
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])
    else:
        assert torch.equal(got, ref)
    assert int(ops.work_queue(q.device).abs().sum()) == 0
