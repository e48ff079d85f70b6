#!/usr/bin/env python3
"""Replay captured activations (vblade.dump.QKDumpAttention / the reference's blocksparseattn.py
dump layout: <root>/timestep_{t}_layer_{l}/{q,k[,v]}.pt) through the HIP mask predictor and the
oracle, on the GPU box:

  * mask parity — the HIP energy mask equals the oracle's energy rule applied to the HIP pooled
    scores, and the HIP pooled scores match the oracle's (fraction of bit-exact entries);
  * quality — PSNR of the sparse attention output against dense attention when v was captured
    (else v = q, which still exercises the real q/k statistics).

    python tools/replay_dumps.py <root> [--variant cog|wan] [--limit N]
Prints one JSON line per dump and a summary line. The oracle here is the checker only.
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    peak = ref.double().abs().max().item()
    return 99.0 if mse == 0 else 10 * math.log10(peak * peak / mse)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--variant", default="cog", choices=["cog", "wan"])
    ap.add_argument("--limit", type=int, default=0)
    args = ap.parse_args()
    import bsa_oracle as O
    import vblade
    from vblade import dump
    from vblade.attention import retain_counts
    dumps = dump.load_dumps(args.root)
    if args.limit:
        dumps = dumps[:args.limit]
    dev = torch.device("cuda")
    mod = vblade.AdaptiveBlockSparseAttn(args.variant, log_every=0)
    summary = {"dumps": 0, "mask_equal": 0, "po_exact_frac": [], "psnr": []}
    for t, layer, d in dumps:
        q = d["q"].to(dev).bfloat16()
        k = d["k"].to(dev).bfloat16()
        v = d.get("v", d["q"]).to(dev).bfloat16()
        B, H, L, D = q.shape
        g = torch.Generator().manual_seed(1000 * t + layer)
        qo = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0].int()
        ko = torch.topk(torch.rand(B, H, 1, 128, generator=g), 32, dim=3).indices[:, :, 0].int()
        po, mask = mod.predict_mask(q, k, qo.to(dev), ko.to(dev))
        nb = po.shape[-1]
        lo, hi = retain_counts(nb, mod.min_retain_ratio, mod.max_retain_ratio, mod.variant)
        ref_mask = O.energy_mask(po.float().cpu(), lo, hi, mod.energy_threshold, mod.force_tail)
        rows = mod._rows(dev).long().cpu() if mod.use_rearrange else torch.arange(L)
        qs = O.sample_tokens(O.pad_replicate(q.cpu()[:, :, rows], 128), qo.long())
        ks = O.sample_tokens(O.pad_replicate(k.cpu()[:, :, rows], 128), ko.long())
        ref_po = O.pooled_scores(qs, ks, 1.0 / D ** 0.5, 32, torch.bfloat16)
        exact = (po.float().cpu() == ref_po).float().mean().item()
        with torch.no_grad():
            out = mod(q, k, v, q_off=qo.to(dev), k_off=ko.to(dev))
            dense = torch.nn.functional.scaled_dot_product_attention(q, k, v)
        p = psnr(out.float(), dense.float())
        eq = bool(torch.equal(mask.bool().cpu(), ref_mask))
        summary["dumps"] += 1
        summary["mask_equal"] += int(eq)
        summary["po_exact_frac"].append(exact)
        summary["psnr"].append(p)
        print(json.dumps({"timestep": t, "layer": layer, "shape": [B, H, L, D], "mask_equal_oracle_rule": eq,
                          "po_exact_frac": round(exact, 5), "density": round(mask.float().mean().item(), 4),
                          "psnr_vs_dense_db": round(p, 2)}), flush=True)
    if summary["dumps"]:
        n = summary["dumps"]
        print(json.dumps({"summary": True, "dumps": n, "mask_equal": summary["mask_equal"],
                          "po_exact_frac_min": round(min(summary["po_exact_frac"]), 5),
                          "psnr_vs_dense_db_mean": round(sum(summary["psnr"]) / n, 2)}))
    else:
        print(json.dumps({"summary": True, "dumps": 0, "note": f"no dumps under {args.root}"}))


if __name__ == "__main__":
    main()
