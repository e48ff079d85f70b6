"""CPU: the multi-level oracle (oracle/ml_oracle.py) against fixtures produced by running the
reference's own multi-level Triton kernel and sampler glue under the Triton interpreter
(tests/golden/make_golden.py gen_multilevel). Reference: cogvideox/sample_evaluate/Triton/
cogvideo_newattn.py and kernels/block_sparse_attn_kernel_with_backward_9_10.py."""
import os

import numpy as np
import pytest
import torch

import ml_oracle as ML
from conftest import GOLDEN

DT = {"torch.float32": torch.float32, "torch.float16": torch.float16}


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(GOLDEN, "multilevel.npz"))


def test_level_bands_reference_values():
    # CogVideoX: nb = ceil(17776/128) = 139; Wan: 256 (TRI/cogvideo_newattn.py:189-192)
    assert ML.level_bands(139) == [(1, 0, 6), (2, 6, 20), (4, 20, 34), (8, 34, 69), (0, 69, 139)]
    assert ML.level_bands(256) == [(1, 0, 12), (2, 12, 38), (4, 38, 64), (8, 64, 128), (0, 128, 256)]
    assert ML.level_bands(5) == [(4, 0, 1), (8, 1, 2), (0, 2, 5)]
    assert abs(ML.density() - 0.15625) < 1e-12      # reported sparsity 0.84375


@pytest.mark.parametrize("case", ["m139", "m256", "m21", "m5"])
def test_level_mask_matches_reference_up_to_ties(z, case):
    po = torch.from_numpy(z[f"lm_{case}_po"])
    ref = torch.from_numpy(z[f"lm_{case}_mask"])
    assert ML.level_mask_is_valid(ref, po)             # the checker accepts the reference
    assert ML.level_mask_is_valid(ML.level_mask(po), po)
    # untied entries agree exactly
    x = po.float()
    eq = (x[..., None, :] == x[..., :, None]).sum(-1) == 1
    mine = ML.level_mask(po)
    assert torch.equal(mine[eq], ref[eq])


def test_level_mask_validity_rejects_wrong_masks(z):
    po = torch.from_numpy(z["lm_m21_po"])
    m = ML.level_mask(po)
    bad = m.clone()
    bad[0, 0, 0, :3] = torch.tensor([8, 8, 8], dtype=torch.int32)
    assert not ML.level_mask_is_valid(bad, po)
    bad = m.clone()
    bad[0, 0, -1, 4] = 0                                # forced row
    assert not ML.level_mask_is_valid(bad, po)


def test_kv_pyramid_bit_exact(z):
    x = torch.from_numpy(z["pyr_x"]).half()
    for name, t in zip(["pad", "p2", "p4", "p8"], ML.kv_pyramid(x)):
        assert torch.equal(t.float(), torch.from_numpy(z["pyr_" + name])), name


@pytest.mark.parametrize("case", ["f32_d64", "f16_d64", "f32_d128", "f16_d128_b2"])
def test_multilevel_forward_matches_reference_kernel(z, case):
    g = lambda s: torch.from_numpy(z[f"k_{case}_{s}"])
    dt = DT[str(z[f"k_{case}_dtype"])]
    q, k, v = (g(s).to(dt) for s in ("q", "k", "v"))
    r = ML.multilevel_attention(q, k, v, g("mask"))
    tol = 1e-5 if dt == torch.float32 else 2e-3
    assert (r["out"] - g("out")).abs().max() < tol
    assert ((r["l"] - g("l")) / g("l")).abs().max() < 1e-5
    assert (r["m"] - g("m")).abs().max() < 1e-5


@pytest.mark.parametrize("case", ["f32_d64", "f16_d64", "f32_d128", "f16_d128_b2"])
def test_multilevel_backward_matches_reference_kernel(z, case):
    g = lambda s: torch.from_numpy(z[f"k_{case}_{s}"])
    dt = DT[str(z[f"k_{case}_dtype"])]
    q, k, v, do = (g(s).to(dt) for s in ("q", "k", "v", "do"))
    dq, dk, dv = ML.multilevel_attention_bwd(q, k, v, g("mask"), g("out").to(dt), g("l"), g("m"),
                                             do, store_dtype=dt)
    tol = 1e-5 if dt == torch.float32 else 1e-3
    for name, a in (("dq", dq), ("dk", dk), ("dv", dv)):
        ref = g(name)
        assert ((a - ref).norm() / ref.norm()) < tol, name


def test_reference_tail_differs_from_masked_tail(z):
    """L % 128 != 0: the reference's level-1 tail keys are zero vectors with logit 0 (kept by
    default); ref_tail=False masks them. L = 256 has no tail and the two agree."""
    g = lambda c, s: torch.from_numpy(z[f"k_{c}_{s}"])
    q, k, v = (g("f32_d64", s) for s in ("q", "k", "v"))
    a = ML.multilevel_attention(q, k, v, g("f32_d64", "mask"))["out"]
    b = ML.multilevel_attention(q, k, v, g("f32_d64", "mask"), ref_tail=False)["out"]
    assert (a - b).abs().max() > 1e-3
    q, k, v = (g("f32_d128", s) for s in ("q", "k", "v"))
    a = ML.multilevel_attention(q, k, v, g("f32_d128", "mask"))["out"]
    b = ML.multilevel_attention(q, k, v, g("f32_d128", "mask"), ref_tail=False)["out"]
    assert torch.equal(a, b)


@pytest.mark.parametrize("case", ["e2e_f32", "e2e_f16"])
def test_adaptive_multilevel_end_to_end(z, case):
    g = lambda s: torch.from_numpy(z[f"{case}_{s}"])
    dt = DT[str(z[f"{case}_dtype"])]
    q, k, v = (g(s).to(dt) for s in ("q", "k", "v"))
    r = ML.adaptive_multilevel_attention(q, k, v, g("qoff").long(), g("koff").long(), store_dtype=dt)
    assert (r["po"] - g("po")).abs().max() <= (1e-6 if dt == torch.float32 else 0)
    assert ML.level_mask_is_valid(r["mask"], g("po"))
    # the kernel output on the reference's own mask
    out = ML.multilevel_attention(q, k, v, g("mask"))["out"]
    assert (out - g("out")).abs().max() < (1e-5 if dt == torch.float32 else 2e-3)
    assert abs(r["sparsity"] - float(z[f"{case}_sparsity"])) < 1e-12
