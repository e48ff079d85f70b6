"""CPU: the oracle's block-sparse attention (restatement of the external block_sparse_attn_func)
against the reference's own CPU attention path — F.scaled_dot_product_attention with the block
mask expanded to a token mask (blocksparseattn.py:93-94) — on BASELINE config 1's inputs.

This pins the op's forward semantics for arbitrary masks, beyond the all-ones identity with
dense SDPA: the masked SDPA is the reference's code path, run here on the same inputs.
"""
import torch

import bsa_oracle as O
import ref_cpu_path as R


def test_token_mask_expands_blocks():
    bm = torch.tensor([[[[1, 0], [0, 1]]]], dtype=torch.bool)
    tm = R.token_mask(bm, 200, 150)
    assert tm.shape == (1, 1, 200, 150)
    assert tm[0, 0, :128, :128].all() and not tm[0, 0, :128, 128:].any()
    assert not tm[0, 0, 128:, :128].any() and tm[0, 0, 128:, 128:].all()


def test_config1_inputs_follow_baseline_plan():
    q, k, v, m = R.config1_inputs("cog", heads=2)
    assert q.shape == (1, 2, 17776, 64) and q.dtype == torch.bfloat16
    assert m.shape == (1, 2, 139, 139)
    assert bool(torch.diagonal(m[0, 0]).all())
    assert 0.48 < m.float().mean().item() < 0.53
    # a head slice is the same data as the first heads of the full draw
    q1, _, _, m1 = R.config1_inputs("cog", heads=1)
    assert torch.equal(q1, q[:, :1]) and torch.equal(m1, m[:, :1])


def test_oracle_matches_reference_masked_sdpa_small():
    g = torch.Generator().manual_seed(7)
    q, k, v = (torch.randn(2, 3, 700, 64, generator=g).bfloat16() for _ in range(3))
    m = O.block_mask_from_density(2, 3, 6, 6, 0.5, seed=5)
    ref, _ = O.block_sparse_attention(q, k, v, m)
    sd = R.masked_sdpa(q, k, v, m).float()
    assert (ref - sd).abs().max().item() <= 4e-3   # bf16 output rounding of the SDPA result


def test_oracle_matches_reference_masked_sdpa_config1_one_head():
    q, k, v, m = R.config1_inputs("cog", heads=1)
    ref, _ = O.block_sparse_attention(q, k, v, m)
    sd = R.masked_sdpa(q, k, v, m).float()
    assert (ref - sd).abs().max().item() <= 4e-3


def test_host_threads_respects_cgroup_quota():
    n = R.host_threads()
    assert 1 <= n <= (__import__("os").cpu_count() or 1)
