"""GPU parity of the multi-level path (vb_kv_pyramid, vb_level_mask, vb_ml_attn_fwd) against the
oracle (oracle/ml_oracle.py, itself pinned to the reference Triton kernel's fixtures) and against
the reference's own fixtures directly.

Tolerances: outputs max|err| <= 2.5e-2 (bf16) / 4e-3 (fp16) on O(1) outputs and PSNR >= 40 dB at
full size; LSE max|err| <= 2e-3; the pyramid is bit-exact (same fp32 pair sums, same rounding);
level masks are exact against the oracle's stable tie order and valid against the reference's
unstable torch.sort (ml_oracle.level_mask_is_valid)."""
import math
import os

import numpy as np
import pytest
import torch

import ml_oracle as ML
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vblade
    vblade.load_library()


def _ops():
    from vblade import ops
    return ops


def _rand(*shape, dtype=torch.bfloat16, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def _tol(dtype):
    return 2.5e-2 if dtype == torch.bfloat16 else 4e-3


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    peak = ref.double().abs().max().item()
    return 99.0 if mse == 0 else 10 * math.log10(peak * peak / mse)


def _random_levels(B, H, nb, seed, p=(0.1, 0.1, 0.1, 0.2, 0.5)):
    """Random level masks (values 1,2,4,8,0 with probabilities p) plus the forced last column."""
    g = torch.Generator().manual_seed(seed)
    lv = torch.tensor([1, 2, 4, 8, 0], dtype=torch.int32)
    idx = torch.multinomial(torch.tensor(p), B * H * nb * nb, replacement=True, generator=g)
    m = lv[idx].reshape(B, H, nb, nb)
    m[..., -1] = 1
    return m


def _tie_heavy_po(B, H, nb, seed):
    g = torch.Generator().manual_seed(seed)
    po = torch.rand(B, H, nb, nb, generator=g) ** 4
    ties = (torch.rand(B, H, nb, nb, generator=g) < 0.15).float()
    po = torch.where(torch.rand(B, H, nb, 1, generator=g) < 0.5, po, torch.maximum(po, ties))
    return (po / po.sum(-1, keepdim=True)).bfloat16()


# ------------------------------------------------------------------------------------- pyramid
@pytest.mark.parametrize("L,D,dtype", [(300, 64, torch.bfloat16), (17776, 64, torch.bfloat16),
                                       (1000, 128, torch.float16), (32760, 128, torch.bfloat16)])
def test_kv_pyramid_bit_exact(L, D, dtype):
    B, H = 1, 2
    k = _rand(B, H, L, D, dtype=dtype, seed=1, scale=2.0)
    v = _rand(B, H, L, D, dtype=dtype, seed=2)
    perm = torch.randperm(L, generator=torch.Generator().manual_seed(3))
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV), perm.int().to(DEV))
    Lpad = (L + 127) // 128 * 128
    for x, pyr in ((k, kp), (v, vp)):
        ref = ML.kv_pyramid(x[:, :, perm])
        got = _ops().pyramid_levels(pyr.cpu(), L)
        assert torch.equal(got[0][:, :, :L], ref[0][:, :, :L])
        assert bool((got[0][:, :, L:] == 0).all())          # tail rows zero (masked loads)
        for lv in (1, 2, 3):
            assert torch.equal(got[lv], ref[lv]), lv
        assert got[3].shape[2] == Lpad // 8


@pytest.mark.parametrize("L,D,B,H,strided", [(17776, 64, 1, 3, False), (17776, 64, 2, 2, True),
                                             (1000, 128, 1, 2, False), (32760, 128, 1, 2, True)])
def test_kv_pyramid_in_the_predictor_launch_equals_standalone(L, D, B, H, strided):
    """The pyramid pass run by extra workgroups of the score kernel's launch (ops.mask_predict
    pyr=..., the module's inference path) writes the same pyramids, bit for bit, as vb_kv_pyramid,
    and leaves the scores unchanged; batched and on strided [B,L,H,D].transpose(1,2) views."""
    ops = _ops()
    g = torch.Generator(device=DEV).manual_seed(12)
    shape = (B, L, H, D) if strided else (B, H, L, D)
    q, k, v = (torch.randn(*shape, generator=g, device=DEV).bfloat16() for _ in range(3))
    if strided:
        q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(4)).int().to(DEV)
    rq = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    rk = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    outs = ops.kv_pyramid_outputs(k)
    po_p, _ = ops.mask_predict(q, k, rows=rows, want_mask=False, rand=(rq, rk), pyr=(v, outs))
    po_r, _ = ops.mask_predict(q, k, rows=rows, want_mask=False, rand=(rq, rk))
    ref = ops.kv_pyramid(k, v, rows)
    torch.cuda.synchronize()
    assert torch.equal(po_p, po_r)
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)


# ------------------------------------------------------------------------------------- level mask
@pytest.mark.parametrize("case", ["m139", "m256", "m21", "m5"])
def test_level_mask_kernel_on_reference_goldens(case):
    z = np.load(os.path.join(GOLDEN, "multilevel.npz"))
    po = torch.from_numpy(z[f"lm_{case}_po"]).bfloat16()
    mask = _ops().level_mask(po.to(DEV)).cpu().to(torch.int32)
    assert torch.equal(mask, ML.level_mask(po))                         # stable tie order
    assert ML.level_mask_is_valid(mask, po)                             # a valid reference answer
    ref = torch.from_numpy(z[f"lm_{case}_mask"])
    x = po.float()
    untied = (x[..., None, :] == x[..., :, None]).sum(-1) == 1
    assert torch.equal(mask[untied], ref[untied])


@pytest.mark.parametrize("nr,nc", [(139, 139), (256, 256), (3, 70), (1, 1), (40, 1000)])
def test_level_mask_kernel_matches_oracle(nr, nc):
    po = _tie_heavy_po(2, 3, max(nr, nc), seed=nr + nc)[..., :nr, :nc].contiguous()
    mask = _ops().level_mask(po.to(DEV)).cpu().to(torch.int32)
    assert torch.equal(mask, ML.level_mask(po))
    ratios = {8: (0.0, 0.3), 2: (0.2, 0.6), 0: (0.6, 1.0)}                # overlapping: later wins
    mask = _ops().level_mask(po.to(DEV), ratios).cpu().to(torch.int32)
    assert torch.equal(mask, ML.level_mask(po, ratios))


@pytest.mark.parametrize("L,D,B,H,ratios", [(17776, 64, 1, 2, None), (32760, 128, 1, 1, None),
                                             (1000, 64, 2, 3, None), (300, 128, 1, 2, "overlap"),
                                             (17776, 64, 1, 1, "empty")])
def test_level_mask_in_the_score_kernel_equals_vb_level_mask(L, D, B, H, ratios):
    """The level mask written by the score kernel's epilogue (ops.mask_predict level=..., the
    multi-level module's path) equals vb_level_mask on the scores the same launch returns, bit for
    bit: the reference bands, overlapping bands (later wins) and no bands (forced tail only).
    Low-entropy inputs make many exactly tied bf16 scores (ties -> lower column)."""
    ops = _ops()
    r = {None: None, "overlap": {8: (0.0, 0.3), 2: (0.2, 0.6), 0: (0.6, 1.0)}, "empty": {}}[ratios]
    g = torch.Generator(device=DEV).manual_seed(L + H)
    q = (torch.randn(B, H, L, D, generator=g, device=DEV) * 0.05).bfloat16()
    k = (torch.randn(B, H, L, D, generator=g, device=DEV) * 0.05).bfloat16()
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(9)).int().to(DEV)
    rq = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    rk = torch.rand(B, H, 1, 128, device=DEV, generator=g)
    po, mask = ops.mask_predict(q, k, rows=rows, rand=(rq, rk), level=ops.ML_MASK_RATIOS if r is None else r)
    po2, _ = ops.mask_predict(q, k, rows=rows, want_mask=False, rand=(rq, rk))
    assert torch.equal(po, po2)
    assert torch.equal(mask, ops.level_mask(po, r))
    assert torch.equal(mask.cpu().to(torch.int32), ML.level_mask(po.cpu(), r))


# ------------------------------------------------------------------------------------- forward
@pytest.mark.parametrize("case", ["f16_d64", "f16_d128_b2"])
def test_ml_forward_matches_reference_kernel_fixture(case):
    """The reference Triton kernel's own fp16 outputs (generated under the interpreter)."""
    z = np.load(os.path.join(GOLDEN, "multilevel.npz"))
    g = lambda s: torch.from_numpy(z[f"k_{case}_{s}"])
    q, k, v = (g(s).half().to(DEV) for s in ("q", "k", "v"))
    mask = g("mask").to(torch.uint8).to(DEV)
    kp, vp = _ops().kv_pyramid(k, v)
    out, lse = _ops().ml_attention_fwd(q, kp, vp, mask, want_lse=True)
    assert (out.float().cpu() - g("out")).abs().max() <= 4e-3
    ref_lse = g("m") + torch.log(g("l"))
    assert (lse.cpu() - ref_lse).abs().max() <= 2e-3


@pytest.mark.parametrize("L,D,dtype,ref_tail", [(300, 64, torch.bfloat16, True), (300, 64, torch.bfloat16, False),
                                                (1000, 128, torch.bfloat16, True), (1000, 128, torch.float16, False),
                                                (2600, 64, torch.float16, True), (200, 64, torch.bfloat16, True),
                                                (129, 128, torch.bfloat16, False), (1024, 64, torch.bfloat16, True)])
def test_ml_forward_matches_oracle(L, D, dtype, ref_tail):
    B, H = 1, 2
    q, k, v = (_rand(B, H, L, D, dtype=dtype, seed=s) for s in (10, 11, 12))
    nb = (L + 127) // 128
    mask = _random_levels(B, H, nb, seed=L + D)
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV))
    out, lse = _ops().ml_attention_fwd(q.to(DEV), kp, vp, mask.to(torch.uint8).to(DEV),
                                       ref_tail=ref_tail, want_lse=True)
    ref = ML.multilevel_attention(q, k, v, mask, ref_tail=ref_tail)
    assert (out.float().cpu() - ref["out"]).abs().max() <= _tol(dtype)
    assert (lse.cpu() - ref["lse"]).abs().max() <= 2e-3


def test_ml_forward_level_coverage_and_partial_tiles():
    """Rows whose level-4 / level-8 block counts are not multiples of 2 / 4 (masked partial
    tiles), rows with a single level, and an all-skip row (output 0, lse -inf)."""
    B, H, L, D = 1, 1, 1280, 64
    nb = 10
    q, k, v = (_rand(B, H, L, D, seed=s) for s in (20, 21, 22))
    m = torch.zeros(B, H, nb, nb, dtype=torch.int32)
    m[0, 0, 0, :] = 8                      # 10 level-8 blocks -> tiles of 4, 4, 2
    m[0, 0, 1, :3] = 4                     # 3 level-4 blocks -> tiles of 2, 1
    m[0, 0, 2, ::3] = 2
    m[0, 0, 3, 5] = 1
    m[0, 0, 4, :] = torch.tensor([1, 2, 4, 8, 0, 8, 4, 2, 1, 8], dtype=torch.int32)
    m[0, 0, 5, :] = torch.tensor([8, 8, 8, 8, 8, 4, 0, 0, 0, 0], dtype=torch.int32)
    m[0, 0, 6, :] = 1
    m[0, 0, 7, 9] = 8
    m[0, 0, 8, :] = torch.tensor([3, 5, 16, 1, 0, 0, 0, 0, 0, 0], dtype=torch.int32)  # non-levels skip
    # row 9 stays all zero
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV))
    mask_u8 = m.clamp(0, 255).to(torch.uint8)
    out, lse = _ops().ml_attention_fwd(q.to(DEV), kp, vp, mask_u8.to(DEV), want_lse=True)
    ref_mask = m.clone()
    ref_mask[0, 0, 8, :3] = 0
    ref = ML.multilevel_attention(q, k, v, ref_mask)
    got = out.float().cpu()
    assert (got[:, :, :9 * 128] - ref["out"][:, :, :9 * 128]).abs().max() <= 2.5e-2
    assert bool((got[:, :, 9 * 128:] == 0).all())
    assert bool(torch.isinf(lse[0, 0, 9 * 128:]).all())


def test_ml_forward_row_gather_scatter_equals_permuted_oracle():
    B, H, L, D = 1, 2, 866, 64
    q, k, v = (_rand(B, H, L, D, seed=s) for s in (30, 31, 32))
    perm = torch.randperm(L, generator=torch.Generator().manual_seed(33))
    nb = (L + 127) // 128
    mask = _random_levels(B, H, nb, seed=34)
    rows = perm.int().to(DEV)
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV), rows)
    out = _ops().ml_attention_fwd(q.to(DEV), kp, vp, mask.to(torch.uint8).to(DEV), q_rows=rows)
    ref = ML.multilevel_attention(q[:, :, perm], k[:, :, perm], v[:, :, perm], mask)["out"]
    want = torch.empty_like(ref)
    want[:, :, perm] = ref
    assert (out.float().cpu() - want).abs().max() <= 2.5e-2


@pytest.mark.parametrize("L,D,H", [(17776, 64, 2), (32760, 128, 1)])
def test_ml_forward_full_size_psnr_and_determinism(L, D, H):
    B = 1
    q, k, v = (_rand(B, H, L, D, seed=s) for s in (40, 41, 42))
    nb = (L + 127) // 128
    po = _tie_heavy_po(B, H, nb, seed=43)
    mask = _ops().level_mask(po.to(DEV))
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV))
    qd = q.to(DEV)
    out1 = _ops().ml_attention_fwd(qd, kp, vp, mask)
    out2 = _ops().ml_attention_fwd(qd, kp, vp, mask)
    assert torch.equal(out1, out2)
    ref = ML.multilevel_attention(q, k, v, mask.cpu().to(torch.int32))["out"]
    assert psnr(out1.float().cpu(), ref) >= 40.0
    assert (out1.float().cpu() - ref).abs().max() <= 2.5e-2


# ------------------------------------------------------------------------------------- end to end
def test_adaptive_multilevel_on_reference_fixture():
    """adaptive_block_sparse_attn of the sampler module on the fixture's inputs and sampling
    offsets (the RNG draw replayed): the predicted mask is a valid reference answer, and the
    output equals the reference kernel's where the masks coincide (else the oracle on ours)."""
    from vblade import multilevel
    z = np.load(os.path.join(GOLDEN, "multilevel.npz"))
    g = lambda s: torch.from_numpy(z[f"e2e_f16_{s}"])
    q, k, v = (g(s).half() for s in ("q", "k", "v"))
    out, sp, mask, po = multilevel.adaptive_block_sparse_attn(
        q.to(DEV), k.to(DEV), v.to(DEV), q_off=g("qoff").int().to(DEV), k_off=g("koff").int().to(DEV),
        return_mask=True)
    assert abs(sp - float(z["e2e_f16_sparsity"])) < 1e-12
    assert (po.float().cpu() - g("po")).abs().max() <= 2 ** -10
    mask_c = mask.cpu().to(torch.int32)
    assert ML.level_mask_is_valid(mask_c, g("po"))
    if torch.equal(mask_c, g("mask")):
        ref = g("out").float()
    else:
        ref = ML.multilevel_attention(q, k, v, mask_c)["out"]
    assert (out.float().cpu() - ref).abs().max() <= 4e-3


def test_sampler_module_with_gilbert_reorder_matches_oracle():
    from vblade import multilevel
    w, h, d, text = 14, 10, 6, 26
    L = w * h * d + text
    B, H, D = 1, 2, 64
    g = torch.Generator().manual_seed(50)
    cent = torch.randn(B, H, L // 16 + 1, D, generator=g).repeat_interleave(16, 2)[:, :, :L]
    q = (torch.randn(B, H, L, D, generator=g) + 1.5 * cent).bfloat16()
    k = (torch.randn(B, H, L, D, generator=g) + 1.5 * cent).bfloat16()
    v = torch.randn(B, H, L, D, generator=g).bfloat16()
    mod = multilevel.AdaptiveBlockSparseAttnTrain(width=w, height=h, depth=d, text_length=text).to(DEV)
    qo = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0].int()
    ko = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0].int()
    out = mod(q.to(DEV), k.to(DEV), v.to(DEV), q_off=qo.to(DEV), k_off=ko.to(DEV))
    rows = mod.gilbert_rearranger.rows.long().cpu()
    r = ML.adaptive_multilevel_attention(q[:, :, rows], k[:, :, rows], v[:, :, rows], qo.long(), ko.long())
    mask = mod.last_mask.cpu().to(torch.int32)
    assert ML.level_mask_is_valid(mask, r["po"])
    ref = ML.multilevel_attention(q[:, :, rows], k[:, :, rows], v[:, :, rows], mask)["out"]
    want = torch.empty_like(ref)
    want[:, :, rows] = ref
    assert (out.float().cpu() - want).abs().max() <= 2.5e-2
    assert abs(mod.sparsity_acc - 0.84375) < 1e-12


def test_level_mask_draws_offsets_in_the_reference_rng_order():
    """Without offsets the multi-level predictor draws rand(q) then rand(k) (efficient_attn_with_
    pooling :77-78) and ranks them inside the sampling launch: the same scores and level mask as
    explicit offsets from vb_sample_offsets on the same generator state."""
    from vblade import attention, multilevel
    B, H, L, D = 1, 3, 40 * 128 + 17, 64
    g = torch.Generator().manual_seed(61)
    q = torch.randn(B, H, L, D, generator=g).bfloat16().to(DEV)
    k = torch.randn(B, H, L, D, generator=g).bfloat16().to(DEV)
    torch.cuda.manual_seed(5)
    po1, m1 = multilevel.predict_level_mask(q, k)
    torch.cuda.manual_seed(5)
    qo, ko = attention.draw_sample_offsets_qk(B, H, DEV)
    po2, m2 = multilevel.predict_level_mask(q, k, q_off=qo, k_off=ko)
    assert torch.equal(po1, po2) and torch.equal(m1, m2)


# ------------------------------------------------------------------------------------- backward
def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("case", ["f16_d64", "f16_d128_b2"])
def test_ml_backward_matches_reference_kernel_fixture(case):
    """dq/dk/dv against the reference Triton kernel's own backward (fp16, interpreter)."""
    z = np.load(os.path.join(GOLDEN, "multilevel.npz"))
    g = lambda s: torch.from_numpy(z[f"k_{case}_{s}"])
    q, k, v, do = (g(s).half().to(DEV) for s in ("q", "k", "v", "do"))
    mask = g("mask").to(torch.uint8).to(DEV)
    kp, vp = _ops().kv_pyramid(k, v)
    out, lse = _ops().ml_attention_fwd(q, kp, vp, mask, want_lse=True)
    dq, dk, dv = _ops().ml_attention_bwd(do, q, kp, vp, mask, out, lse)
    for name, got in (("dq", dq), ("dk", dk), ("dv", dv)):
        assert _rel(got.float().cpu(), g(name)) <= 5e-3, name


@pytest.mark.parametrize("L,D,dtype,ref_tail,perm", [(300, 64, torch.bfloat16, True, False),
                                                     (300, 64, torch.bfloat16, False, True),
                                                     (1000, 128, torch.bfloat16, True, True),
                                                     (517, 128, torch.float16, False, False),
                                                     (1280, 64, torch.float16, True, True)])
def test_ml_backward_matches_oracle(L, D, dtype, ref_tail, perm):
    B, H = 1, 2
    q, k, v, do = (_rand(B, H, L, D, dtype=dtype, seed=s) for s in (60, 61, 62, 63))
    nb = (L + 127) // 128
    mask = _random_levels(B, H, nb, seed=L + 7 * D, p=(0.15, 0.15, 0.15, 0.25, 0.3))
    rows = torch.randperm(L, generator=torch.Generator().manual_seed(64)) if perm else None
    rd = rows.int().to(DEV) if perm else None
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV), rd)
    md = mask.to(torch.uint8).to(DEV)
    out, lse = _ops().ml_attention_fwd(q.to(DEV), kp, vp, md, q_rows=rd, ref_tail=ref_tail, want_lse=True)
    dq, dk, dv = _ops().ml_attention_bwd(do.to(DEV), q.to(DEV), kp, vp, md, out, lse, rows=rd,
                                         ref_tail=ref_tail)
    P = rows if perm else torch.arange(L)
    qr, kr, vr, dor = q[:, :, P], k[:, :, P], v[:, :, P], do[:, :, P]
    fwd = ML.multilevel_attention(qr, kr, vr, mask, ref_tail=ref_tail)
    rq, rk, rv = ML.multilevel_attention_bwd(qr, kr, vr, mask, out.float().cpu()[:, :, P], fwd["l"],
                                             fwd["m"], dor)
    for name, got, ref in (("dq", dq, rq), ("dk", dk, rk), ("dv", dv, rv)):
        assert _rel(got.float().cpu()[:, :, P], ref) <= 2e-2, name


def test_ml_backward_deterministic_and_module_autograd():
    """Bitwise-reproducible gradients at CogVideoX's sequence length, through the module's
    autograd path (Gilbert reorder inside the op)."""
    from vblade import multilevel
    B, H, D = 1, 2, 64
    mod = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0).to(DEV)
    L = mod.gilbert_rearranger.seq_len
    q, k, v, do = (_rand(B, H, L, D, seed=s).to(DEV) for s in (70, 71, 72, 73))
    nb = (L + 127) // 128
    mask = _ops().level_mask(_tie_heavy_po(B, H, nb, seed=74).to(DEV))
    grads = []
    for _ in range(2):
        qq, kk, vv = (t.clone().requires_grad_() for t in (q, k, v))
        out = mod(qq, kk, vv, level_mask=mask)
        out.backward(do)
        grads.append((qq.grad, kk.grad, vv.grad))
    for a, b in zip(*grads):
        assert torch.equal(a, b)
    # the inference path gives the autograd op's output up to the inference kernel's extra
    # rounding of q * scale * log2(e) to bf16 (vb_attn_fwd.hip, kCBias)
    with torch.no_grad():
        out_inf = mod(q, k, v, level_mask=mask)
    assert (out_inf.float() - out.detach().float()).abs().max().item() <= 2.5e-2
    assert _rel(out_inf.float().cpu(), out.detach().float().cpu()) <= 5e-3


@pytest.mark.parametrize("sel", ["default", "dkdv_round3", "dq_round3"])
def test_ml_backward_kernel_select_matches_oracle(sel):
    """Every selectable multi-level backward path (kernel_select) against the oracle, with the kernels
    that ran asserted from kernels_ran: the default (pipeline level-1 dK/dV and dQ), the round-3
    level-1 dK/dV, the round-3 dQ. dk/dv of the two dK/dV kernels agree to bf16 rounding, dq of the
    two dQ kernels too; the 4-slot dQ ring does not exist here and is refused."""
    from vblade import _lib
    B, H, L, D = 1, 2, 700, 64
    q, k, v, do = (_rand(B, H, L, D, seed=s) for s in (80, 81, 82, 83))
    nb = (L + 127) // 128
    mask = _random_levels(B, H, nb, seed=84, p=(0.15, 0.15, 0.15, 0.25, 0.3))
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV))
    md = mask.to(torch.uint8).to(DEV)
    qd, dod = q.to(DEV), do.to(DEV)
    out, lse = _ops().ml_attention_fwd(qd, kp, vp, md, want_lse=True)
    bits = {"default": 0, "dkdv_round3": _lib.VB_BWD_SEL_DKDV_ROUND3, "dq_round3": _lib.VB_BWD_SEL_DQ_ROUND3}[sel]
    want = _lib.VB_BWD_RAN_ML_PYRAMID
    want |= _lib.VB_BWD_RAN_DKDV_ROUND3 if sel == "dkdv_round3" else _lib.VB_BWD_RAN_DKDV_PIPE
    want |= _lib.VB_BWD_RAN_DQ_ROUND3 if sel == "dq_round3" else _lib.VB_BWD_RAN_DQ_PIPE_RING2
    ran, ran0 = [], []
    g = _ops().ml_attention_bwd(dod, qd, kp, vp, md, out, lse, kernel_select=bits, kernels_ran=ran)
    g0 = _ops().ml_attention_bwd(dod, qd, kp, vp, md, out, lse, kernels_ran=ran0)
    assert ran == [want]
    for a, b in zip(g, g0):
        assert _rel(a.float().cpu(), b.float().cpu()) <= 5e-3
    fwd = ML.multilevel_attention(q, k, v, mask)
    ref = ML.multilevel_attention_bwd(q, k, v, mask, out.float().cpu(), fwd["l"], fwd["m"], do)
    for name, got, r in zip(("dq", "dk", "dv"), g, ref):
        assert _rel(got.float().cpu(), r) <= 2e-2, name
    with pytest.raises(_lib.VBladeError):
        _ops().ml_attention_bwd(dod, qd, kp, vp, md, out, lse, kernel_select=_lib.VB_BWD_SEL_DQ_RING4)


@pytest.mark.parametrize("L,D,H", [(17776, 64, 4), (32760, 128, 2)])
def test_ml_forward_persistent_is_bit_identical(L, D, H):
    """The persistent (work-queue) multi-level launch gives the one-workgroup-per-q-block launch's
    bits, twice in a row on the same queue (which each launch leaves zero)."""
    q, k, v = (_rand(1, H, L, D, seed=s) for s in (90, 91, 92))
    nb = (L + 127) // 128
    mask = _ops().level_mask(_tie_heavy_po(1, H, nb, seed=93).to(DEV))
    kp, vp = _ops().kv_pyramid(k.to(DEV), v.to(DEV))
    qd = q.to(DEV)
    ref = _ops().ml_attention_fwd(qd, kp, vp, mask)
    for _ in range(2):
        assert torch.equal(_ops().ml_attention_fwd(qd, kp, vp, mask, persistent=True), ref)
    assert int(_ops().work_queue(qd.device).abs().sum()) == 0
