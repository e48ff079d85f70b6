"""TEST INFRASTRUCTURE ONLY — CPU restatement (oracle) of Video-BLADE's adaptive block-sparse
attention path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline. The product path is the HIP library
``libvblade_hip.so`` (``video-blade_amd/csrc``); it never calls into this file.

Every function cites the reference file:line it restates. Paths are relative to the reference
repo root; ``TR/`` = ``cogvideox/train/special_attentions_local/TrainRelated/`` (the Wan copy
under ``wanx/train/...`` differs only where noted).

Pinning:
  * gilbert permutation, sampled offsets, pooled scores (fp32 and fp16 storage), energy masks,
    simple pooling, the LSE combine and the whole adaptive glue are pinned against the
    reference's own Python/Triton code run in this container (``tests/golden/make_golden.py``,
    Triton interpreter) — fixtures in ``tests/golden/``.
  * the external CUDA op ``block_sparse_attn_func`` (mit-han-lab/Block-Sparse-Attention, an
    un-vendored FlashAttention-2 fork; no version pinned by the reference, README.md:52-61) is
    absent: its restatement here (masked softmax with natural-log LSE) is pinned only by the
    identity with dense SDPA for an all-ones mask and by masked-softmax semantics
    -> "parity unpinned" for that single op, as recorded in DESIGN.md.
"""
from __future__ import annotations

import math

import numpy as np
import torch

LOG2E = 1.44269504  # the literal used by attn_pooling_kernel.py:169


# ----------------------------------------------------------------------------------------------
# rounding helpers
# ----------------------------------------------------------------------------------------------
def rnd(x: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Round an fp32/fp64 tensor to ``dtype`` storage and back to fp32 (no-op for fp32)."""
    return x.to(dtype).to(torch.float32)


# ----------------------------------------------------------------------------------------------
# a3: padding and token sampling for the mask predictor
# ----------------------------------------------------------------------------------------------
def pad_replicate(x: torch.Tensor, multiple: int) -> torch.Tensor:
    """TR/cogvideo_blocksparseattn.py:20-31 — replicate-pad dim -2 up to a multiple."""
    L = x.shape[-2]
    rem = L % multiple
    if rem == 0:
        return x
    tail = x[..., L - 1:L, :].expand(*x.shape[:-2], multiple - rem, x.shape[-1])
    return torch.cat([x, tail], dim=-2)


def draw_sample_offsets(B: int, H: int, block: int = 128, num_keep: int = 32,
                        generator: torch.Generator | None = None, device="cpu") -> torch.Tensor:
    """TR/cogvideo_blocksparseattn.py:45-46 — rand(B,H,1,block) then topk(num_keep) -> [B,H,num_keep]."""
    r = torch.rand(B, H, 1, block, generator=generator, device=device)
    return torch.topk(r, num_keep, dim=3).indices[:, :, 0, :]


def sample_tokens(x_padded: torch.Tensor, offsets: torch.Tensor, block: int = 128) -> torch.Tensor:
    """TR/cogvideo_blocksparseattn.py:32-55 — the same ``num_keep`` offsets in every block of a (b,h)."""
    B, H, L, D = x_padded.shape
    nb = L // block
    xb = x_padded.reshape(B, H, nb, block, D)
    idx = offsets[:, :, None, :, None].expand(B, H, nb, offsets.shape[-1], D)
    return torch.gather(xb, 3, idx).reshape(B, H, nb * offsets.shape[-1], D)


# ----------------------------------------------------------------------------------------------
# a4: pooled scores (restates the Triton kernel attn_pooling_kernel.py:17-84, 87-199, 201-253)
# ----------------------------------------------------------------------------------------------
def pooled_scores(qs: torch.Tensor, ks: torch.Tensor, sm_scale: float, block: int = 32,
                  store_dtype: torch.dtype | None = None) -> torch.Tensor:
    """Po[b,h,i,j] = max_{r in q-block i} exp2(R[r,j] - m_r), row-normalised in ``store_dtype``.

    * qk_scale = fp32(sm_scale) * fp32(1.44269504)                     (:168-169)
    * rowmax_blk = max over the block's keys of fp32 dot products, times qk_scale (:46,52)
    * R = rowmax_blk rounded to the storage dtype (q.dtype)             (:55, R alloc :219)
    * m_r = running max of the UNROUNDED fp32 rowmax_blk                 (:53,56)
    * Po[i,j] = storage(max_r exp2(float(R[r,j]) - m_r))  (l_i == 1)    (:73-82)
    * Po /= Po.sum(-1) in the storage dtype (fp32 accumulation)         (:250-251)
    """
    store_dtype = store_dtype or qs.dtype
    B, H, Ls, D = qs.shape
    n = Ls // block
    qk_scale = float(np.float32(sm_scale) * np.float32(LOG2E))
    S = torch.matmul(qs.float(), ks.float().transpose(-1, -2))             # [B,H,Ls,Ls] fp32
    rowblk = S.reshape(B, H, Ls, n, block).amax(-1) * np.float32(qk_scale)  # fp32
    m = rowblk.amax(-1, keepdim=True)
    R = rnd(rowblk, store_dtype)
    w = torch.exp2(R - m)
    po = rnd(w.reshape(B, H, n, block, n).amax(3), store_dtype)
    tot = rnd(po.sum(-1, keepdim=True), store_dtype)
    return rnd(po / tot, store_dtype)


# ----------------------------------------------------------------------------------------------
# a5: energy rule -> block mask
# ----------------------------------------------------------------------------------------------
def retain_counts(nb: int, min_ratio: float, max_ratio: float, variant: str) -> tuple[int, int]:
    """min/max kept blocks per row.

    cog: clamp((seq * fp32 ratio tensor).to(int), min=1)   (TR/cogvideo_blocksparseattn.py:230-231, 347-348)
    wan: max(1, int(seq * ratio)) in Python floats          (wanx_blocksparseattn.py:215-216)"""
    if variant == "cog":
        lo = int(np.float32(nb) * np.float32(min_ratio))
        hi = int(np.float32(nb) * np.float32(max_ratio))
    else:
        lo = int(nb * min_ratio)
        hi = int(nb * max_ratio)
    return max(1, lo), max(1, hi)


def energy_keep_count(po_row_sorted: np.ndarray, thr: float, store_dtype=torch.bfloat16) -> int:
    """Number of leading sorted blocks kept before clamping (TR/cogvideo_blocksparseattn.py:232-238).

    cumsum accumulates in fp32 and rounds each prefix to the storage dtype (torch CPU cumsum);
    k = first index with cum >= storage(total*fp32(thr)); the crossing block itself is NOT kept;
    never crossing -> k = nb."""
    # torch CPU cumsum for bf16/fp16 accumulates in float: a sequential fp32 running sum,
    # each prefix rounded to the storage dtype
    cums = np.cumsum(po_row_sorted.astype(np.float32), dtype=np.float32)
    cum = rnd(torch.from_numpy(cums), store_dtype)
    total = cum[-1]
    th = rnd(total * np.float32(thr), store_dtype)
    hit = torch.nonzero(cum >= th)
    return int(hit[0]) if hit.numel() else int(cum.numel())


def energy_keep_counts(po: torch.Tensor, min_keep: int, max_keep: int, thr: float = 0.95,
                       store_dtype=torch.bfloat16) -> torch.Tensor:
    """Clamped kept-block count k per row [B,H,nr] (TR/cogvideo_blocksparseattn.py:232-239).
    k depends only on the sorted VALUES, so it is independent of how ties are ordered."""
    p = po.float().cpu().numpy()
    k = np.zeros(p.shape[:3], dtype=np.int64)
    for idx in np.ndindex(*p.shape[:3]):
        row = p[idx]
        kk = energy_keep_count(-np.sort(-row), thr, store_dtype)
        k[idx] = min(max(kk, min_keep), max_keep)
    return torch.from_numpy(k)


def energy_mask(po: torch.Tensor, min_keep: int, max_keep: int, thr: float = 0.95,
                force_tail: int = 0, store_dtype=torch.bfloat16) -> torch.Tensor:
    """transfer_attn_to_mask(mode="energy") (TR/cogvideo_blocksparseattn.py:177-249;
    wanx_blocksparseattn.py:162-233). Ties are broken by LOWER block index first (stable
    descending sort); the reference's torch.sort is unstable, so which of several EQUAL
    boundary blocks it keeps is implementation-defined (``mask_is_valid_topk`` accepts any
    such choice). ``force_tail`` = 2 for CogVideoX (:247-248: last 2 rows and columns forced
    True), 0 for Wan."""
    B, H, nr, nc = po.shape
    p = po.float().cpu().numpy()
    kk = energy_keep_counts(po, min_keep, max_keep, thr, store_dtype).numpy()
    mask = np.zeros((B, H, nr, nc), dtype=bool)
    for idx in np.ndindex(B, H, nr):
        order = np.argsort(-p[idx], kind="stable")
        mask[idx][order[:kk[idx]]] = True
    if force_tail:
        mask[..., -force_tail:] = True
        mask[..., -force_tail:, :] = True
    return torch.from_numpy(mask)


def mask_is_valid_topk(mask: torch.Tensor, po: torch.Tensor, k: torch.Tensor,
                       force_tail: int = 0) -> bool:
    """True when every row of ``mask`` equals T ∪ F for SOME top-k selection T of that row
    (any tie order) and F = the forced tail columns; forced rows must be all True."""
    m = mask.bool().cpu().numpy()
    p = po.float().cpu().numpy()
    kk = k.cpu().numpy()
    nr, nc = m.shape[2], m.shape[3]
    forced = np.zeros(nc, dtype=bool)
    if force_tail:
        forced[-force_tail:] = True
    for idx in np.ndindex(*m.shape[:3]):
        row, val, kr = m[idx], p[idx], int(kk[idx])
        if force_tail and idx[2] >= nr - force_tail:
            if not row.all():
                return False
            continue
        if not row[forced].all():
            return False
        vk = np.sort(val)[::-1][kr - 1]
        required = val > vk
        ties = val == vk
        body = row & ~forced
        if not row[required].all():
            return False
        if (body & ~(required | ties)).any():
            return False
        need = kr - int(required.sum())
        if not (int((body & ties).sum()) <= need <= int((row & ties).sum())):
            return False
    return True


# ----------------------------------------------------------------------------------------------
# a7: block-sparse attention (external block_sparse_attn_func; restated, parity unpinned)
# ----------------------------------------------------------------------------------------------
def block_sparse_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
                           block_mask: torch.Tensor | None, sm_scale: float | None = None,
                           block: int = 128, key_bias: float = 0.0,
                           acc_dtype=torch.float64):
    """out[b,h,r] = softmax over keys c of the kept (row-block, col-block) pairs of
    (q_r . k_c) * scale, times v; lse = natural-log log-sum-exp of the kept scaled scores.

    Replaces block_sparse_attn_func as called at TR/cogvideo_blocksparseattn.py:316-320
    (non-causal, p_dropout 0, softmax_scale None -> D^-1/2, 128x128 blocks, LSE fp32 [B,H,Lq]).
    ``block_mask`` None = dense. Computed per 128-row block in ``acc_dtype``.
    Returns (out fp32 [B,H,Lq,D], lse fp32 [B,H,Lq])."""
    B, H, Lq, D = q.shape
    Lk = k.shape[2]
    scale = sm_scale if sm_scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = q.to(acc_dtype), k.to(acc_dtype), v.to(acc_dtype)
    out = torch.zeros(B, H, Lq, D, dtype=torch.float32)
    lse = torch.full((B, H, Lq), float("-inf"), dtype=torch.float32)
    nbq = (Lq + block - 1) // block
    keycol_block = torch.arange(Lk) // block
    for i in range(nbq):
        r0, r1 = i * block, min(Lq, (i + 1) * block)
        s = torch.matmul(qf[:, :, r0:r1], kf.transpose(-1, -2)) * scale + key_bias  # [B,H,m,Lk]
        if block_mask is not None:
            keep = block_mask[:, :, i, :].bool()[:, :, keycol_block]                   # [B,H,Lk]
            s = s.masked_fill(~keep[:, :, None, :], float("-inf"))
        mx = s.amax(-1, keepdim=True)
        mx_safe = torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))
        p = torch.exp(s - mx_safe)
        l = p.sum(-1, keepdim=True)
        o = torch.matmul(p, vf) / torch.where(l > 0, l, torch.ones_like(l))
        out[:, :, r0:r1] = o.float()
        lse[:, :, r0:r1] = (mx_safe + torch.log(l)).squeeze(-1).float()
    return out, lse


def block_sparse_attention_bwd(q, k, v, out, lse, dout, block_mask, sm_scale=None, block=128,
                               key_bias: float = 0.0, acc_dtype=torch.float64):
    """FlashAttention-2 backward semantics for a7 (LSE treated as a constant, no LSE gradient):
    P = exp(S*scale + bias - lse), Delta = rowsum(dO*O), dS = P*(dO V^T - Delta),
    dQ = scale dS K, dK = scale dS^T Q, dV = P^T dO. Returns fp32 (dq, dk, dv)."""
    B, H, Lq, D = q.shape
    Lk = k.shape[2]
    scale = sm_scale if sm_scale is not None else 1.0 / math.sqrt(D)
    qf, kf, vf = q.to(acc_dtype), k.to(acc_dtype), v.to(acc_dtype)
    of, dof = out.to(acc_dtype), dout.to(acc_dtype)
    dq = torch.zeros(B, H, Lq, D, dtype=acc_dtype)
    dk = torch.zeros(B, H, Lk, D, dtype=acc_dtype)
    dv = torch.zeros(B, H, Lk, D, dtype=acc_dtype)
    nbq = (Lq + block - 1) // block
    keycol_block = torch.arange(Lk) // block
    for i in range(nbq):
        r0, r1 = i * block, min(Lq, (i + 1) * block)
        s = torch.matmul(qf[:, :, r0:r1], kf.transpose(-1, -2)) * scale + key_bias
        if block_mask is not None:
            keep = block_mask[:, :, i, :].bool()[:, :, keycol_block]
            s = s.masked_fill(~keep[:, :, None, :], float("-inf"))
        p = torch.exp(s - lse[:, :, r0:r1, None].to(acc_dtype))
        do = dof[:, :, r0:r1]
        delta = (do * of[:, :, r0:r1]).sum(-1, keepdim=True)
        dp = torch.matmul(do, vf.transpose(-1, -2))
        ds = p * (dp - delta)
        dq[:, :, r0:r1] = torch.matmul(ds, kf) * scale
        dk += torch.matmul(ds.transpose(-1, -2), qf[:, :, r0:r1]) * scale
        dv += torch.matmul(p.transpose(-1, -2), do)
    return dq.float(), dk.float(), dv.float()


# ----------------------------------------------------------------------------------------------
# a8: mean pooling of K/V; a9: LSE combine
# ----------------------------------------------------------------------------------------------
def simple_pooling(x: torch.Tensor, gap: int, store_dtype=None) -> torch.Tensor:
    """TR/cogvideo_blocksparseattn.py:83-88 — replicate-pad to a multiple of ``gap`` and mean
    groups of ``gap`` consecutive (reordered) tokens; fp32 accumulate, stored in x.dtype."""
    store_dtype = store_dtype or x.dtype
    xp = pad_replicate(x.float(), gap)
    B, H, L, D = xp.shape
    return xp.reshape(B, H, L // gap, gap, D).mean(-2).to(store_dtype)


def simple_pooling_bwd(dxp: torch.Tensor, L: int, gap: int) -> torch.Tensor:
    """Adjoint of simple_pooling: each pooled row's gradient / gap to its ``gap`` sources;
    replicate-padded rows fold onto the last token (F.pad replicate backward)."""
    B, H, Lp, D = dxp.shape
    g = (dxp.float() / gap).repeat_interleave(gap, dim=2)       # [B,H,Lp*gap,D]
    dx = g[:, :, :L].clone()
    if Lp * gap > L:
        dx[:, :, L - 1] += g[:, :, L:].sum(2)
    return dx


def combine_reference(out1: torch.Tensor, lse1: torch.Tensor, out2: torch.Tensor,
                      lse2: torch.Tensor, gap: int, dtype=torch.bfloat16):
    """TR/cogvideo_blocksparseattn.py:374-393 executed op-by-op in ``dtype`` (each eager op
    computes in fp32 and rounds to ``dtype``); lse1/lse2 are first cast to ``dtype`` (:324).
    Returns (out [B,H,L,D] in fp32 holding ``dtype`` values, alpha)."""
    R = lambda t: rnd(t, dtype)  # noqa: E731
    l1 = R(lse1.float())[..., None]
    l2 = R(lse2.float())[..., None]
    log_g = R(torch.log(R(torch.tensor(float(gap)))))
    w2 = R(l2 + log_g)
    mx = torch.maximum(l1, w2)
    e1 = R(torch.exp(R(l1 - mx)))
    e2 = R(torch.exp(R(w2 - mx)))
    alpha = R(e1 / R(e1 + e2))
    o = R(R(R(out1.float()) * alpha) + R(R(out2.float()) * R(1.0 - alpha)))
    return o, alpha


# ----------------------------------------------------------------------------------------------
# whole adaptive path (a1-a9)
# ----------------------------------------------------------------------------------------------
class AdaptiveConfig:
    """Reference module-level globals (TR/cogvideo_blocksparseattn.py:9-16; wanx :9-16)."""

    def __init__(self, variant="cog", width=45, height=30, depth=13, text_length=226,
                 sample_gap=15, min_retain_ratio=0.05, max_retain_ratio=0.1,
                 energy_threshold=0.95, block=128, num_keep=32, use_rearrange=True):
        self.variant = variant
        self.width, self.height, self.depth = width, height, depth
        self.text_length = text_length
        self.sample_gap = sample_gap
        self.min_retain_ratio, self.max_retain_ratio = min_retain_ratio, max_retain_ratio
        self.energy_threshold = energy_threshold
        self.block, self.num_keep = block, num_keep
        self.use_rearrange = use_rearrange

    @property
    def force_tail(self):
        return 2 if self.variant == "cog" else 0

    @staticmethod
    def cogvideox(**kw):
        return AdaptiveConfig(**{**dict(variant="cog"), **kw})

    @staticmethod
    def wan(**kw):
        base = dict(variant="wan", width=52, height=30, depth=21, text_length=0, sample_gap=30,
                    min_retain_ratio=0.05, max_retain_ratio=0.17)
        return AdaptiveConfig(**{**base, **kw})


def predict_mask(q_r, k_r, cfg: AdaptiveConfig, q_off, k_off, store_dtype=torch.bfloat16):
    """efficient_attn_with_pooling + transfer_attn_to_mask (TR/cogvideo_blocksparseattn.py:57-82,
    343-358) on already-reordered q, k. Returns (po, mask)."""
    D = q_r.shape[-1]
    qs = sample_tokens(pad_replicate(q_r, cfg.block), q_off, cfg.block)
    ks = sample_tokens(pad_replicate(k_r, cfg.block), k_off, cfg.block)
    po = pooled_scores(qs, ks, 1.0 / (D ** 0.5), cfg.num_keep, store_dtype)
    nb = po.shape[-1]
    lo, hi = retain_counts(nb, cfg.min_retain_ratio, cfg.max_retain_ratio, cfg.variant)
    mask = energy_mask(po, lo, hi, cfg.energy_threshold, cfg.force_tail, store_dtype)
    return po, mask


def adaptive_attention(q, k, v, cfg: AdaptiveConfig, q_off, k_off, mask=None,
                       store_dtype=torch.bfloat16):
    """AdaptiveBlockSparseAttnTrain.forward (TR/cogvideo_blocksparseattn.py:405-427) +
    adaptive_block_sparse_attn (:327-394), reference-faithful rounding (out1/out2 rounded to the
    storage dtype, bf16 combine). Returns dict with out (original order, fp32 values),
    mask, po, sparsity, and the intermediate branch results."""
    from gilbert_oracle import full_sequence_perm  # local import: oracle dir is on sys.path
    B, H, L, D = q.shape
    if cfg.use_rearrange:
        P = torch.from_numpy(full_sequence_perm(cfg.width, cfg.height, cfg.depth, cfg.text_length))
    else:
        P = torch.arange(L)
    assert P.numel() == L
    q_r, k_r, v_r = q[:, :, P], k[:, :, P], v[:, :, P]
    po = None
    if mask is None:
        po, mask = predict_mask(q_r, k_r, cfg, q_off, k_off, store_dtype)
    out1, lse1 = block_sparse_attention(q_r, k_r, v_r, mask, block=cfg.block)
    kp = simple_pooling(k_r, cfg.sample_gap, store_dtype)
    vp = simple_pooling(v_r, cfg.sample_gap, store_dtype)
    out2, lse2 = block_sparse_attention(q_r, kp, vp, None, block=cfg.block)
    out_r, alpha = combine_reference(rnd(out1, store_dtype), lse1, rnd(out2, store_dtype), lse2,
                                     cfg.sample_gap, store_dtype)
    inv = torch.empty_like(P)
    inv[P] = torch.arange(L)
    sparsity = 1.0 - mask.float().mean().item() - 1.0 / cfg.sample_gap
    return dict(out=out_r[:, :, inv], out_r=out_r, mask=mask, po=po, perm=P, out1=out1, lse1=lse1,
                out2=out2, lse2=lse2, kp=kp, vp=vp, alpha=alpha, sparsity=sparsity)


def adaptive_attention_joint(q, k, v, cfg: AdaptiveConfig, mask):
    """The single-softmax identity of a9 (no intermediate rounding): softmax over the kept
    full-resolution keys united with the pooled keys carrying a +ln(gap) bias. Equal to
    ``adaptive_attention`` up to the reference's bf16 rounding of out1/out2/lse/alpha."""
    from gilbert_oracle import full_sequence_perm
    B, H, L, D = q.shape
    P = (torch.from_numpy(full_sequence_perm(cfg.width, cfg.height, cfg.depth, cfg.text_length))
         if cfg.use_rearrange else torch.arange(L))
    q_r, k_r, v_r = q[:, :, P], k[:, :, P], v[:, :, P]
    out1, lse1 = block_sparse_attention(q_r, k_r, v_r, mask, block=cfg.block)
    kp = simple_pooling(k_r, cfg.sample_gap)
    vp = simple_pooling(v_r, cfg.sample_gap)
    out2, lse2 = block_sparse_attention(q_r, kp, vp, None, block=cfg.block,
                                        key_bias=math.log(cfg.sample_gap))
    lse = torch.logaddexp(lse1, lse2)
    a = torch.exp(lse1 - lse)[..., None]
    out_r = out1 * a + out2 * (1 - a)
    inv = torch.empty_like(P)
    inv[P] = torch.arange(L)
    return out_r[:, :, inv], lse


def joint_from_branches(fwd: dict, log_gap: float) -> torch.Tensor:
    """Exact (fp64) single-softmax combine of ``adaptive_attention``'s unrounded branch results
    (out1/lse1, out2/lse2): the a9 identity with no bf16 rounding of lse, alpha or the branch
    outputs, the pooled keys carrying the bias ``log_gap`` (the reference's combine uses the bf16
    value of ln g, :375-376). Returns the output in the original token order (fp64)."""
    l1 = fwd["lse1"].double()
    l2 = fwd["lse2"].double() + log_gap
    lse = torch.logaddexp(l1, l2)
    a = torch.exp(l1 - lse)[..., None]
    out_r = fwd["out1"].double() * a + fwd["out2"].double() * (1 - a)
    P = fwd["perm"]
    inv = torch.empty_like(P)
    inv[P] = torch.arange(P.numel())
    return out_r[:, :, inv]


def bf16_ulp_distance(got: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Checker utility: |bf16(got) - bf16(ref)| in bf16 units in the last place at the reference's
    magnitude, with magnitudes below the tensor's RMS binade measured in that binade's ULP (an
    output near zero from cancellation is judged at the scale of the tensor, not in ULPs of its
    own tiny value). bf16 keeps 8 significant bits: ULP(x) = 2^(floor(log2|x|) - 7). int64."""
    g = got.float().to(torch.bfloat16).double()
    r = ref.float().to(torch.bfloat16).double()
    rms = float(r.pow(2).mean().sqrt())
    floor = 2.0 ** math.floor(math.log2(rms)) if rms > 0 else 2.0 ** -126
    mag = torch.clamp(r.abs(), min=floor)
    ulp = torch.exp2(torch.floor(torch.log2(mag)) - 7)
    return torch.round((g - r).abs() / ulp).to(torch.int64)


ULP_BUCKETS = ((0, 0), (1, 1), (2, 2), (3, 4), (5, 8), (9, 16), (17, None))


def bf16_ulp_histogram(got: torch.Tensor, ref: torch.Tensor) -> dict:
    """Fractions of elements per bf16-ULP distance bucket (0, 1, 2, 3-4, 5-8, 9-16, >16; see
    bf16_ulp_distance), plus the maximum distance (SURVEY §8d Quality)."""
    d = bf16_ulp_distance(got, ref).flatten()
    n = d.numel()
    hist = {}
    for lo, hi in ULP_BUCKETS:
        sel = (d >= lo) if hi is None else ((d >= lo) & (d <= hi))
        key = f">{lo - 1}" if hi is None else (str(lo) if lo == hi else f"{lo}-{hi}")
        hist[key] = round(int(sel.sum()) / n, 6)
    return {"ulp_hist": hist, "max_ulp": int(d.max()), "n": n,
            "ulp_unit": "bf16 ULP at |ref|, floored at the RMS binade of ref"}


def adaptive_attention_bwd(q, k, v, dout, cfg: AdaptiveConfig, fwd: dict):
    """Gradient of adaptive_attention w.r.t. q, k, v under the reference's autograd semantics
    (a10): mask under no_grad; LSEs carry no gradient (FA2 convention) so alpha is a constant;
    dO1 = alpha dO, dO2 = (1-alpha) dO; each branch's backward uses its own output and LSE;
    pooled-branch K/V grads flow back through the mean pool; the Gilbert gather transposes.
    fp32/fp64 arithmetic (no bf16 emulation of the backward)."""
    P = fwd["perm"]
    L = q.shape[2]
    q_r, k_r, v_r = q[:, :, P], k[:, :, P], v[:, :, P]
    do_r = dout.float()[:, :, P]
    a = fwd["alpha"]
    do1, do2 = do_r * a, do_r * (1 - a)
    dq1, dk1, dv1 = block_sparse_attention_bwd(q_r, k_r, v_r, fwd["out1"], fwd["lse1"], do1,
                                               fwd["mask"], block=cfg.block)
    dq2, dkp, dvp = block_sparse_attention_bwd(q_r, fwd["kp"], fwd["vp"], fwd["out2"], fwd["lse2"],
                                               do2, None, block=cfg.block)
    dq_r = dq1 + dq2
    dk_r = dk1 + simple_pooling_bwd(dkp, L, cfg.sample_gap)
    dv_r = dv1 + simple_pooling_bwd(dvp, L, cfg.sample_gap)
    inv = torch.empty_like(P)
    inv[P] = torch.arange(L)
    return dq_r[:, :, inv], dk_r[:, :, inv], dv_r[:, :, inv]


def block_mask_from_density(B, H, nbq, nbk, density, seed=3):
    """BASELINE.md §3 synthetic mask: (rand < density) | eye, at least one block per row."""
    g = torch.Generator().manual_seed(seed)
    m = torch.rand(B, H, nbq, nbk, generator=g) < density
    eye = torch.zeros(nbq, nbk, dtype=torch.bool)
    d = min(nbq, nbk)
    eye[torch.arange(d), torch.arange(d)] = True
    return m | eye
