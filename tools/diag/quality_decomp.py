#!/usr/bin/env python3
"""Where the fused inference path's error against the oracle comes from.

At full length (CogVideoX [1,2,17776,64], Wan [1,1,32760,128]; realistic block-structured inputs)
and for the energy rule plus fixed densities 0.3 / 0.5 / 0.7, compares on the GPU's own mask:

  fused    the module's inference path (one softmax over kept ∪ pooled keys; Q pre-scaled by
           scale*log2e and rounded to bf16 inside the kernel)
  refmode  the module's combine="reference" path (two attention launches + the bf16 combine)
  ref      oracle.adaptive_attention: the reference's rounding (out1/out2 bf16, lse cast to bf16,
           alpha and the combine op by op in bf16; cogvideo_blocksparseattn.py:324, 374-393)
  exact    oracle.joint_from_branches: the same two branches combined exactly in fp64
  exact_qs exact, with q replaced by bf16(q*c)/c (c = fp32(D^-1/2)*fp32(log2 e)): the fused
           kernel's pre-scaled Q and nothing else

and prints one JSON line per case: max|.|, PSNR and bf16 ULP histograms of every pair.
usage: python tools/diag/quality_decomp.py [--variant cog|wan|both] [--out FILE]
"""
import argparse
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bsa_oracle as O  # noqa: E402


def realistic_qkv(B, H, L, D, seed, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    cent = torch.randn(B, H, L // 128 + 1, D, generator=g).repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(B, H, L, D, generator=g) + 2 * cent).to(dtype)
    k = (torch.randn(B, H, L, D, generator=g) + 2 * cent).to(dtype)
    v = torch.randn(B, H, L, D, generator=g).to(dtype)
    return q, k, v


def psnr(x, ref):
    mse = torch.mean((x.double() - ref.double()) ** 2).item()
    peak = ref.double().abs().max().item()
    return 99.0 if mse == 0 else round(10 * math.log10(peak * peak / mse), 2)


def pair(a, b):
    return {"max_abs": round((a.double() - b.double()).abs().max().item(), 6), "psnr_db": psnr(a, b),
            **O.bf16_ulp_histogram(a, b)}


def prescaled_q(q, D):
    c = np.float32(np.float32(1.0 / math.sqrt(D)) * np.float32(1.4426950408889634))
    return ((q.float() * float(c)).to(torch.bfloat16).double() / float(c))


def run_case(variant, density, H, seed=5):
    import vblade
    over = {} if density is None else dict(min_retain_ratio=density, max_retain_ratio=density)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **over)
    L = m.gilbert_rearranger.seq_len
    D = 64 if variant == "cog" else 128
    q, k, v = realistic_qkv(1, H, L, D, seed)
    dev = torch.device("cuda")
    torch.manual_seed(3)
    with torch.no_grad():
        fused = m(q.to(dev), k.to(dev), v.to(dev)).float().cpu()
        mask_d = m.last_mask
        m2 = vblade.AdaptiveBlockSparseAttn(variant, combine="reference", log_every=0, **over)
        refmode = m2(q.to(dev), k.to(dev), v.to(dev), block_mask=mask_d).float().cpu()
    mask = mask_d.bool().cpu()
    cfg = O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan()
    log_gap = m._log_gap(torch.bfloat16)
    fwd = O.adaptive_attention(q, k, v, cfg, None, None, mask=mask, store_dtype=torch.bfloat16)
    ref = fwd["out"]
    exact = O.joint_from_branches(fwd, log_gap)
    fwd_qs = O.adaptive_attention(prescaled_q(q, D), k, v, cfg, None, None, mask=mask,
                                  store_dtype=torch.bfloat16)
    exact_qs = O.joint_from_branches(fwd_qs, log_gap)
    return {
        "variant": variant, "heads": H, "L": L, "D": D,
        "mask": "energy rule" if density is None else f"density {density}",
        "kept_frac": round(mask.float().mean().item(), 4),
        "max_abs_exact": round(exact.abs().max().item(), 4),
        "fused_vs_ref": pair(fused, ref),
        "fused_vs_exact": pair(fused, exact),
        "ref_vs_exact": pair(ref, exact),
        "fused_vs_exact_qs": pair(fused, exact_qs),
        "exact_qs_vs_exact": pair(exact_qs, exact),
        "refmode_vs_ref": pair(refmode, ref),
        "refmode_vs_exact": pair(refmode, exact),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="both")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cases = []
    if a.variant in ("cog", "both"):
        cases += [("cog", d, 2) for d in (None, 0.3, 0.5, 0.7)]
    if a.variant in ("wan", "both"):
        cases += [("wan", d, 1) for d in (None, 0.5)]
    res = []
    for variant, d, H in cases:
        r = run_case(variant, d, H)
        res.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
