"""TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of Video-BLADE's MULTI-LEVEL block-sparse
attention, the op the VBench sampler uses.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker. The product path is the HIP library (csrc/vb_ml.hip and the
multi-level instantiation of csrc/vb_attn_fwd.hip); it never calls into this file.

Reference files (paths relative to the reference root), abbreviated:
  TRI/ = cogvideox/sample_evaluate/Triton/
  KML  = TRI/kernels/block_sparse_attn_kernel_with_backward_9_10.py

Semantics restated here:
  * level mask      transfer_attn_to_mask (TRI/cogvideo_newattn.py:154-207): per row, the block
                    ranked r (descending pooled score) gets the value of the band [int(nc*start),
                    int(nc*end)) that holds r (dict order, later bands overwrite), else 0; then
                    the last two columns and the last two rows are forced to 1.
  * KV pyramid      KML:1239-1270 and :1311-1320: K/V replicate-padded to a multiple of 128, then
                    mean-pooled by 2 three times (each level rounded to the storage dtype).
  * forward         KML:338-692: one softmax per query row over, for every key block j with level
                    p > 0, the 128/p level-p keys of block j, each with logit q.k*scale + ln p.
                    Level-1 keys beyond L (the last block when L % 128 != 0) are loaded as ZERO
                    vectors (masked loads, KML:111,126): logit 0, value 0 — the reference's tail
                    behaviour, kept by default (``ref_tail=True``); ``ref_tail=False`` masks them.
                    Stores l (row sum) and m (row max, natural log domain) for the backward.
  * backward        KML:696-731 (preprocess: dO/l rounded to dO's dtype, Delta = rowsum(O*dO/l)),
                    :732-1237 (per-level dK/dV/dQ with the same biases, tail keys masked), and
                    :1375-1576 (dK = dK1 + up(dK2)/2 + up(dK4)/4 + up(dK8)/8 truncated to L: the
                    gradient that reaches replicate-padded rows is dropped, as the reference does).

Pinning: the reference's own Triton kernel and glue run under TRITON_INTERPRET=1 in the build
container generate the fixtures (tests/golden/make_golden.py -> tests/golden/multilevel.npz);
tests/test_oracle_golden.py checks this restatement against them.
"""
from __future__ import annotations

import math

import torch

# TRI/cogvideo_newattn.py:12-18 (the sampler's module-level mask_ratios)
ML_MASK_RATIOS = {1: (0.0, 0.05), 2: (0.05, 0.15), 4: (0.15, 0.25), 8: (0.25, 0.5), 0: (0.5, 1.0)}
LEVELS = (1, 2, 4, 8)
BLOCK = 128


def level_bands(nc: int, ratios=None):
    """TRI/cogvideo_newattn.py:189-192: [(value, start_idx, end_idx)] in dict order (Python float
    arithmetic, as the reference computes int(seq * ratio))."""
    ratios = ML_MASK_RATIOS if ratios is None else ratios
    out = []
    for v, (s, e) in ratios.items():
        a = max(0, int(nc * s))
        b = min(nc, int(nc * e))
        if a < b:
            out.append((int(v), a, b))
    return out


def rank_stable_desc(po: torch.Tensor) -> torch.Tensor:
    """rank[j] = #{i: po_i > po_j} + #{i < j: po_i == po_j} (descending, ties to the lower index)."""
    x = po.float()
    gt = (x[..., None, :] > x[..., :, None]).sum(-1)
    n = x.shape[-1]
    lower = torch.tril(torch.ones(n, n, dtype=torch.bool), diagonal=-1)   # i < j
    eq = ((x[..., None, :] == x[..., :, None]) & lower).sum(-1)
    return gt + eq


def level_mask(po: torch.Tensor, ratios=None) -> torch.Tensor:
    """transfer_attn_to_mask (TRI/cogvideo_newattn.py:154-207) with a stable descending sort
    (the reference's torch.sort is unstable; ties are resolved to the lower block index)."""
    nr, nc = po.shape[-2], po.shape[-1]
    rank = rank_stable_desc(po)
    mask = torch.zeros(po.shape, dtype=torch.int32)
    for v, a, b in level_bands(nc, ratios):
        sel = (rank >= a) & (rank < b)
        mask = torch.where(sel, torch.full_like(mask, v), mask)
    mask[..., -2:] = 1
    mask[..., -2:, :] = 1
    return mask


def level_mask_is_valid(mask: torch.Tensor, po: torch.Tensor, ratios=None) -> bool:
    """True iff ``mask`` equals transfer_attn_to_mask under SOME tie order of ``po`` (the
    reference's torch.sort is unstable, so ties may land in any order): the forced last two
    rows/columns are 1, and for every group of equal scores in a row, occupying ranks
    [g, g + e), the levels of its members outside the forced columns are a sub-multiset of the
    levels those ranks carry (the forced members take the rest)."""
    from collections import Counter
    nr, nc = po.shape[-2], po.shape[-1]
    m = mask.to(torch.int64).reshape(-1, nr, nc)
    x = po.float().reshape(-1, nr, nc)
    if not bool((m[:, :, -2:] == 1).all()) or not bool((m[:, -2:, :] == 1).all()):
        return False
    lvl_of_rank = [0] * nc
    for v, a, b in level_bands(nc, ratios):
        for r in range(a, b):
            lvl_of_rank[r] = v
    forced_col = set(range(max(0, nc - 2), nc))
    for s in range(m.shape[0]):
        for i in range(nr - 2):
            row = x[s, i].tolist()
            order = sorted(range(nc), key=lambda j: -row[j])
            r = 0
            while r < nc:
                e = r + 1
                while e < nc and row[order[e]] == row[order[r]]:
                    e += 1
                avail = Counter(lvl_of_rank[r:e])
                need = Counter(int(m[s, i, j]) for j in order[r:e] if j not in forced_col)
                if any(need[k] > avail[k] for k in need):
                    return False
                r = e
    return True


def pad_replicate(x: torch.Tensor, multiple: int) -> torch.Tensor:
    """KML:1239-1250 (F.pad mode='replicate' on dim 2)."""
    L = x.shape[2]
    rem = L % multiple
    if rem == 0:
        return x
    tail = x[:, :, L - 1:L, :].expand(x.shape[0], x.shape[1], multiple - rem, x.shape[3])
    return torch.cat([x, tail], dim=2)


def pool2(x: torch.Tensor) -> torch.Tensor:
    """KML:1252-1270: mean over consecutive pairs, in the tensor's own dtype (torch.mean)."""
    B, H, L, D = x.shape
    assert L % 2 == 0
    return torch.mean(x.view(B, H, L // 2, 2, D), dim=3)


def kv_pyramid(x: torch.Tensor):
    """KML:1311-1320 -> [x_pad, x_2, x_4, x_8] (x_16 is computed by the reference but unused)."""
    xp = pad_replicate(x, BLOCK)
    x2 = pool2(xp)
    x4 = pool2(x2)
    x8 = pool2(x4)
    return [xp, x2, x4, x8]


def _level_keys(pyr, j: int, p: int, L: int, ref_tail: bool):
    """Keys/values of key block j at level p as the forward kernel loads them."""
    lvl = {1: 0, 2: 1, 4: 2, 8: 3}[p]
    n = BLOCK // p
    k = pyr[0][lvl][:, :, j * n:(j + 1) * n].float()
    v = pyr[1][lvl][:, :, j * n:(j + 1) * n].float()
    valid = torch.ones(n, dtype=torch.bool)
    if p == 1:
        idx = torch.arange(j * n, (j + 1) * n)
        tail = idx >= L
        if tail.any():
            k = k.clone()
            v = v.clone()
            k[:, :, tail] = 0.0     # masked tl.load -> 0 (KML:111, 126)
            v[:, :, tail] = 0.0
            if not ref_tail:
                valid = ~tail
    return k, v, valid


def multilevel_attention(q, k, v, mask, sm_scale=None, ref_tail=True):
    """_fwd_kernel (KML:338-692) in fp32 (softmax exact, no online rescale rounding).
    q, k, v [B,H,L,D] (storage dtype); mask [B,H,nb,nb] int levels.
    Returns dict(out fp32 [B,H,L,D], l [B,H,L], m [B,H,L] (natural-log max), lse)."""
    B, H, L, D = q.shape
    sm_scale = sm_scale if sm_scale is not None else D ** -0.5
    nb = (L + BLOCK - 1) // BLOCK
    pyr = (kv_pyramid(k), kv_pyramid(v))
    qf = q.float()
    out = torch.zeros(B, H, L, D)
    l_out = torch.zeros(B, H, L)
    m_out = torch.zeros(B, H, L)
    for b in range(B):
        for h in range(H):
            for i in range(nb):
                r0, r1 = i * BLOCK, min(L, (i + 1) * BLOCK)
                qs = qf[b, h, r0:r1]
                logits, vals = [], []
                for j in range(nb):
                    p = int(mask[b, h, i, j])
                    if p not in LEVELS:
                        continue
                    kk, vv, valid = _level_keys(pyr, j, p, L, ref_tail)
                    s = qs @ kk[b, h].T * sm_scale + math.log(p)
                    s[:, ~valid] = -math.inf
                    logits.append(s)
                    vals.append(vv[b, h])
                if not logits:
                    continue
                S = torch.cat(logits, 1)
                V = torch.cat(vals, 0)
                m = S.amax(1)
                P = torch.exp(S - m[:, None])
                l = P.sum(1)
                out[b, h, r0:r1] = (P @ V) / l[:, None]
                l_out[b, h, r0:r1] = l
                m_out[b, h, r0:r1] = m
    return dict(out=out, l=l_out, m=m_out, lse=m_out + torch.log(l_out))


def multilevel_attention_bwd(q, k, v, mask, out, l, m, dout, sm_scale=None, store_dtype=None):
    """_backward (KML:1375-1576) with the per-level kernels (:696-1237), fp32 arithmetic.
    ``out`` is the forward output as stored (storage dtype values); dO/l is rounded to
    ``store_dtype`` (NewDO = empty_like(do), :1397) when given. Returns (dq, dk, dv) fp32."""
    B, H, L, D = q.shape
    sm_scale = sm_scale if sm_scale is not None else D ** -0.5
    nb = (L + BLOCK - 1) // BLOCK
    Lpad = nb * BLOCK
    pyr = (kv_pyramid(k), kv_pyramid(v))
    do_s = dout.float() / l[..., None]
    if store_dtype is not None:
        do_s = do_s.to(store_dtype).float()
    delta = (out.float() * do_s).sum(-1)
    qf = q.float()
    dq = torch.zeros(B, H, L, D)
    dkl = [torch.zeros(B, H, Lpad // p, D) for p in LEVELS]
    dvl = [torch.zeros(B, H, Lpad // p, D) for p in LEVELS]
    for b in range(B):
        for h in range(H):
            for i in range(nb):
                r0, r1 = i * BLOCK, min(L, (i + 1) * BLOCK)
                qs, dos = qf[b, h, r0:r1], do_s[b, h, r0:r1]
                mi, di = m[b, h, r0:r1], delta[b, h, r0:r1]
                for j in range(nb):
                    p = int(mask[b, h, i, j])
                    if p not in LEVELS:
                        continue
                    lv = LEVELS.index(p)
                    n = BLOCK // p
                    kk = pyr[0][lv][b, h, j * n:(j + 1) * n].float()
                    vv = pyr[1][lv][b, h, j * n:(j + 1) * n].float()
                    s = qs @ kk.T * sm_scale + math.log(p)
                    if p == 1:
                        idx = torch.arange(j * n, (j + 1) * n)
                        s[:, idx >= L] = -math.inf        # KML:762-763
                    P = torch.exp(s - mi[:, None])
                    dvl[lv][b, h, j * n:(j + 1) * n] += P.T @ dos
                    dp = dos @ vv.T - di[:, None]
                    ds = P * dp * sm_scale
                    dkl[lv][b, h, j * n:(j + 1) * n] += ds.T @ qs
                    dq[b, h, r0:r1] += ds @ kk
    dk = dkl[0].clone()
    dv = dvl[0].clone()
    for lv, p in enumerate(LEVELS[1:], start=1):
        dk += dkl[lv].repeat_interleave(p, dim=2)[:, :, :Lpad] / p
        dv += dvl[lv].repeat_interleave(p, dim=2)[:, :, :Lpad] / p
    return dq, dk[:, :, :L], dv[:, :, :L]


def density(ratios=None) -> float:
    """adaptive_block_sparse_attn's reported density (TRI/cogvideo_newattn.py:227-231)."""
    ratios = ML_MASK_RATIOS if ratios is None else ratios
    return sum((e - s) / v for v, (s, e) in ratios.items() if v != 0)


def adaptive_multilevel_attention(q_r, k_r, v_r, q_off, k_off, ratios=None,
                                  store_dtype=torch.bfloat16, ref_tail=True):
    """adaptive_block_sparse_attn (TRI/cogvideo_newattn.py:210-234) on already-reordered q, k, v:
    efficient_attn_with_pooling (:64-89, the same sampler and Triton pooled scores as the main
    path) -> level mask -> multi-level attention. Returns dict(out, po, mask, sparsity, ...)."""
    import bsa_oracle as O   # oracle dir is on sys.path
    D = q_r.shape[-1]
    qs = O.sample_tokens(O.pad_replicate(q_r, BLOCK), q_off, BLOCK)
    ks = O.sample_tokens(O.pad_replicate(k_r, BLOCK), k_off, BLOCK)
    po = O.pooled_scores(qs, ks, 1.0 / (D ** 0.5), q_off.shape[-1], store_dtype)
    mask = level_mask(po, ratios)
    res = multilevel_attention(q_r, k_r, v_r, mask, ref_tail=ref_tail)
    res.update(po=po, mask=mask, sparsity=1.0 - density(ratios))
    return res
