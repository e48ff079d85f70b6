#!/usr/bin/env python3
"""CPU model of the attention kernel's L2 traffic under different q-block dispatch orders
(VERDICT r04 item 4). Predicts the masks of the locality-faithful inputs with the oracle, then
replays each XCD's workgroup stream through an LRU model of its 4 MiB L2: `conc` workgroups run at
once (the D=128 kernel holds two per CU, 32 CUs per XCD), each walks its kept key blocks then the
pooled keys one 64-key tile at a time, round-robin with the others; a new workgroup starts when one
ends. Reports key/value bytes fetched past the L2 per order (a model: no Infinity Cache, no
prefetch, no timing), against the algorithmic bytes.

usage: python tools/diag/qorder_sim.py [wan|cog] [heads]"""
import os
import sys
from collections import OrderedDict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
import bench  # noqa: E402
from oracle import bsa_oracle as O  # noqa: E402
from vblade.attention import GilbertRearranger  # noqa: E402


def masks(variant, H):
    cfg = O.AdaptiveConfig.wan() if variant == "wan" else O.AdaptiveConfig.cogvideox()
    D = 128 if variant == "wan" else 64
    gr = GilbertRearranger(cfg.width, cfg.height, cfg.depth, cfg.text_length)
    q, k, _ = bench.local_qkv(variant, H, D, 0, "cpu")
    r = gr.rows.long()
    q_r, k_r = q[..., r, :].float(), k[..., r, :].float()
    g = torch.Generator().manual_seed(0)
    qo = O.draw_sample_offsets(1, H, generator=g)
    ko = O.draw_sample_offsets(1, H, generator=g)
    po, mask = O.predict_mask(q_r.bfloat16(), k_r.bfloat16(), cfg, qo, ko)
    return po[0].float().numpy(), mask[0].numpy().astype(bool), D, q.shape[2], cfg


def simulate(order, mask, D, L, gap, conc=64, l2_bytes=4 << 20):
    """order: list of (head, qblk) in dispatch order for ONE XCD. Returns fetched bytes."""
    blk_bytes = 2 * 128 * D * 2            # K and V of one 128-key block
    Lkp = (L + gap - 1) // gap
    ptiles = (Lkp + 63) // 64
    cap = l2_bytes // (blk_bytes // 2)      # cache lines of 64-key half blocks
    lru = OrderedDict()
    fetched = 0

    def touch(key):
        nonlocal fetched
        if key in lru:
            lru.move_to_end(key)
            return
        fetched += blk_bytes // 2
        lru[key] = 1
        if len(lru) > cap:
            lru.popitem(last=False)

    def tiles(h, i):
        for j in np.nonzero(mask[h, i])[0]:
            yield ("k", h, int(j), 0)
            yield ("k", h, int(j), 1)
        for t in range(ptiles):
            yield ("p", h, t, 0)

    pending = list(order)
    active = []
    while pending or active:
        while pending and len(active) < conc:
            h, i = pending.pop(0)
            active.append(tiles(h, i))
        nxt = []
        for it in active:
            key = next(it, None)
            if key is not None:
                touch(key)
                nxt.append(it)
        active = nxt
    return fetched


def xcd_ranges(H, nb):
    """the kernel's phase-2 mapping: each XCD a contiguous head-major range of (head, q-block)"""
    n = H * nb
    q8, r8 = n // 8, n % 8
    out, s = [], 0
    for x in range(8):
        c = q8 + (1 if x < r8 else 0)
        out.append((s, s + c))
        s += c
    return out


def main():
    variant = sys.argv[1] if len(sys.argv) > 1 else "wan"
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    po, mask, D, L, cfg = masks(variant, H)
    nb = mask.shape[-1]
    algo = sum(mask[h].sum() for h in range(H)) * 2 * 128 * D * 2
    comp = H * L * D * 2 * 2
    print(f"{variant}: H={H} nb={nb} density={mask.mean():.3f} K/V bytes read by the workgroups {algo / 1e6:.1f} MB,"
          f" compulsory {comp / 1e6:.1f} MB")
    orders = {}
    # default: head-major, q-blocks descending within a head (attn_fwd_kernel phase 2)
    orders["default"] = [(h, nb - 1 - i) for h in range(H) for i in range(nb)]
    # anchor: q-blocks of a head sorted by the key block of their largest pooled score
    anc = po.copy()
    for h in range(H):
        np.fill_diagonal(anc[h], -1)   # the own block is always near the top: not informative
    key = anc.argmax(-1)
    orders["anchor"] = [(h, int(i)) for h in range(H) for i in np.lexsort((np.arange(nb), key[h]))]
    # centroid of the kept set
    cen = np.array([[np.nonzero(mask[h, i])[0].mean() for i in range(nb)] for h in range(H)])
    orders["centroid"] = [(h, int(i)) for h in range(H) for i in np.argsort(cen[h], kind="stable")]
    # greedy chain: next = the unvisited q-block sharing the most kept blocks with the last `win`
    # chosen ones (an upper bound on what a clustering can buy; O(nb^2) per head)
    for win in (1, 8):
        og = []
        for h in range(H):
            m = mask[h].astype(np.int32)
            left = set(range(nb))
            cur = [nb - 1]
            left.discard(nb - 1)
            while left:
                ref = m[cur[-win:]].sum(0)
                cand = np.array(sorted(left))
                best = cand[np.argmax(m[cand] @ ref)]
                cur.append(int(best))
                left.discard(int(best))
            og += [(h, i) for i in cur]
        orders[f"greedy{win}"] = og
    # round 6: the order the kernel runs since ABI 3 (attn_order_kernel: longest first inside each
    # XCD range), the same with ties broken by head and first kept off-diagonal block, and the
    # greedy chain restricted to what a per-XCD queue can realise (inside each XCD's range, from its
    # longest q-block, heads mixed as the range mixes them)
    cnt = mask.sum(-1)
    def first_kept(h, i):
        js = [j for j in np.nonzero(mask[h, i])[0] if j != i]
        return js[0] if js else i
    lf, lfk, gx = [], [], []
    m = mask.astype(np.int32)
    for a, b in xcd_ranges(H, nb):
        r = orders["default"][a:b]
        lf += sorted(r, key=lambda x: -cnt[x])
        lfk += sorted(r, key=lambda x: (-cnt[x], x[0], first_kept(*x)))
        V = np.zeros((len(r), H * nb), np.int32)
        for k, (h, i) in enumerate(r):
            V[k, h * nb:(h + 1) * nb] = m[h, i]
        left = set(range(len(r)))
        cur = [max(left, key=lambda k: cnt[r[k]])]
        left.discard(cur[0])
        while left:
            ref = V[cur[-8:]].sum(0)
            cand = np.array(sorted(left))
            best = int(cand[np.argmax(V[cand] @ ref)])
            cur.append(best)
            left.discard(best)
        gx += [r[k] for k in cur]
    orders["longest1st"] = lf
    orders["lf+head+fk"] = lfk
    orders["greedy8/xcd"] = gx
    for name, o in orders.items():
        tot = 0
        for a, b in xcd_ranges(H, nb):
            tot += simulate(o[a:b], mask, D, L, cfg.sample_gap)
        print(f"  {name:11s} fetched {tot / 1e6:8.1f} MB = {tot / comp:5.2f}x compulsory K/V")


if __name__ == "__main__":
    main()
