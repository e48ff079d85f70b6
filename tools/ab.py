#!/usr/bin/env python3
"""A/B timing of library variants (video-blade_amd/vblade/variants/lib_<tag>.so) in ONE process on
ONE GPU: the same inputs, launches interleaved A,B,A,B,... so clock/device drift cancels.
usage: python tools/ab.py TAG_A TAG_B [--variant cog|wan|both] [--what attn|pred|call]
TAG "cur" is the in-tree libvblade_hip.so; a "@torchrand" suffix runs that tag with the sampling
draws made by torch.rand instead of inside the sampling launch (ops.PHILOX_DRAWS off), "@lvsep"
with the multi-level mask as its own vb_level_mask launch (--what mlcall: the multi-level module),
"@noorder" with the attention launches in the kernel's own q-block order (no longest-first sort),
"@win:N" with only the last N q-blocks of each XCD range re-ordered,
"@env:VAR=VAL+VAR=VAL" with those environment variables set around its launches, "@persist" with the
persistent (work-queue) attention launch (ops.attention_fwd persistent=True; off otherwise),
"@sel:N" with the backward's kernel_select bits N (--what bwd / mlbwd), "@serialfwd" with the
training forward's two branches on one stream (--what trainfwd; autograd.FORK_POOLED_BRANCH off).
Compile-time switches are A/B'd as build variants (VB_EXTRA_FLAGS=-D... tools/build_variant.sh TAG)."""
import argparse
import ctypes
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import vblade  # noqa: E402
from vblade import _lib, multilevel, ops  # noqa: E402
from vblade import autograd as vautograd  # noqa: E402
from bench import attn_flops, ml_attn_flops, realistic_qkv  # noqa: E402


def load(tag):
    tag = tag.split("@")[0]
    path = os.path.join(ROOT, "video-blade_amd", "vblade", "variants", f"lib_{tag}.so")
    if tag == "cur":
        path = os.path.join(ROOT, "video-blade_amd", "vblade", "libvblade_hip.so")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _lib.SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:   # an older ABI: entry points it predates become no-op stubs
            setattr(lib, name, lambda *a: 0)
            continue
        fn.restype, fn.argtypes = res, args
    return lib


ORDER = [True, 0, False, 0]   # longest-first order, order window, persistent attention launch,
                             # backward kernel_select


def select(tag, libs):
    """make `tag` the active variant: its library, its module switches and its environment"""
    _lib._lib = libs[tag]
    ORDER[0] = "@noorder" not in tag
    ORDER[1] = 0
    ORDER[2] = "@persist" in tag
    ORDER[3] = 0
    for part in tag.split("@")[1:]:
        if part.startswith("win:"):
            ORDER[1] = int(part[4:])
        if part.startswith("sel:"):
            ORDER[3] = int(part[4:])
    ops.PHILOX_DRAWS = "@torchrand" not in tag
    vautograd.FORK_POOLED_BRANCH = "@serialfwd" not in tag
    multilevel.FUSED_LEVEL_MASK = "@lvsep" not in tag
    for kv in ENV_SET:
        os.environ.pop(kv, None)
    ENV_SET.clear()
    for part in tag.split("@")[1:]:
        if part.startswith("env:"):
            for kv in part[4:].split("+"):
                k, v = kv.split("=", 1)
                os.environ[k] = v
                ENV_SET.append(k)


ENV_SET = []


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--variant", default="both")
    ap.add_argument("--what", default="attn")
    ap.add_argument("--rounds", type=int, default=15)
    a = ap.parse_args()
    libs = {t: load(t) for t in set(a.tags)}
    keys = [f"{t}#{i}" for i, t in enumerate(a.tags)]
    dev = torch.device("cuda")
    for variant in (["cog", "wan"] if a.variant == "both" else [a.variant]):
        H, D = (48, 64) if variant == "cog" else (12, 128)
        m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **({"gather_kv": os.environ["AB_GATHER"] == "1"} if "AB_GATHER" in os.environ else {}))
        L = m.gilbert_rearranger.seq_len
        q, k, v = realistic_qkv(H, L, D, 0, dev)
        rows = m._rows(dev)
        qo = vblade.draw_sample_offsets(1, H, dev)
        ko = vblade.draw_sample_offsets(1, H, dev)
        _lib._lib = libs[a.tags[0]]
        _, mask = m.predict_mask(q, k, qo, ko)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
        fl = attn_flops(mask, L, D, kp.shape[2])
        qlen = (mask != 0).sum(-1).to(torch.int32).contiguous()
        if a.what == "attn":
            fn = lambda: ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp,  # noqa
                                           vp=vp, kp_log_bias=m._log_gap(q.dtype),
                                           heavy_rows=m.force_tail, order=ORDER[0], q_lengths=qlen,
                                           order_window=ORDER[1], persistent=ORDER[2])
        elif a.what == "fwdlse":   # the training forward's main branch (LSE out: the non-lazy kernel)
            fn = lambda: ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True,  # noqa
                                           heavy_rows=m.force_tail, persistent=ORDER[2])[0]
            fl = attn_flops(mask, L, D, 0)
        elif a.what == "trainfwd":   # the training forward (two LSE branches + combine), no grad taken
            fn = lambda: vautograd.adaptive_split_attention(q, k, v, mask, rows, m.sample_gap,  # noqa
                                                            heavy_rows=m.force_tail)
            fl = attn_flops(mask, L, D, kp.shape[2])
        elif a.what == "pred":
            fn = lambda: m.predict_mask(q, k, qo, ko)  # noqa
        elif a.what == "bwd":   # the training-path backward (vb_attn_bwd) on the two-branch forward
            do = torch.randn_like(q)
            gap = m.sample_gap
            out1, lse1 = ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, need_lse=True,
                                           heavy_rows=m.force_tail)
            out2, lse2 = ops.attention_fwd(q, None, None, use_main=False, q_rows=rows, kp=kp, vp=vp,
                                           need_lse=True)
            _, alpha = ops.lse_combine(out1, lse1, out2, lse2, gap)
            fn = lambda: ops.attention_bwd(do, q, k_r, v_r, out1, lse1, block_mask=mask, q_rows=rows,  # noqa
                                           kv_rows=rows, kp=kp, vp=vp, out2=out2, lse2=lse2,
                                           alpha=alpha, gap=gap, heavy_rows=m.force_tail,
                                           kernel_select=ORDER[3])
            fl = 2.5 * fl
        elif a.what == "mlbwd":   # the multi-level path's backward (vb_ml_attn_bwd), dk compared
            do = torch.randn_like(q)
            _, lmask = multilevel.predict_level_mask(q, k, rows=rows)
            kpy, vpy = ops.kv_pyramid(k, v, rows)
            mo, mlse = ops.ml_attention_fwd(q, kpy, vpy, lmask, q_rows=rows, want_lse=True, heavy_rows=2)
            fn = lambda: ops.ml_attention_bwd(do, q, kpy, vpy, lmask, mo, mlse, rows=rows,  # noqa
                                              kernel_select=ORDER[3])[1]
            fl = 2.5 * ml_attn_flops(lmask, L, D)
        elif a.what == "mlattn":   # the multi-level attention launch alone
            _, lmask = multilevel.predict_level_mask(q, k, rows=rows)
            kpy, vpy = ops.kv_pyramid(k, v, rows)
            fn = lambda: ops.ml_attention_fwd(q, kpy, vpy, lmask, q_rows=rows, heavy_rows=2,  # noqa
                                              persistent=ORDER[2])
            fl = ml_attn_flops(lmask, L, D)
        elif a.what == "mlcall":   # the multi-level (VBench) module, whole call
            mlm = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0)

            def fn():
                mlm.persistent = ORDER[2]
                return mlm(q, k, v)
        else:
            def fn():
                m.order, m.order_window, m.persistent = ORDER[0], ORDER[1], ORDER[2]
                return m(q, k, v)
        ref = None
        times = {kk: [] for kk in keys}
        with torch.no_grad():
            for t in a.tags:   # warm + cross-check outputs (a repeated tag checks determinism)
                select(t, libs)
                if a.what in ("call", "mlcall"):
                    torch.cuda.manual_seed(1234)   # the module draws its sampling offsets per call
                out = fn()
                torch.cuda.synchronize()
                if a.what == "pred":   # the same scores and energy rule: masks must be identical
                    if ref is None:
                        ref = out[1].clone()
                    else:
                        print(f"  {t}: mask identical to {a.tags[0]}: {torch.equal(out[1], ref)}")
                if a.what in ("attn", "fwdlse", "bwd", "mlbwd", "mlattn", "trainfwd", "call", "mlcall"):
                    outs = tuple(out) if isinstance(out, tuple) else (out,)   # bwd: dq, dk, dv
                    if ref is None:
                        ref = tuple(o.clone() for o in outs)
                    else:
                        same = all(torch.equal(o, r) for o, r in zip(outs, ref))
                        err = max((o.float() - r.float()).abs().max().item() for o, r in zip(outs, ref))
                        rel = ", ".join(f"{(o.float() - r.float()).abs().max().item() / max(r.float().abs().max().item(), 1e-30):.2e}"
                                        for o, r in zip(outs, ref))
                        print(f"  {t}: bit-identical to {a.tags[0]} over {len(outs)} output(s): {same}; "
                              f"max|diff| = {err:.3e}; per output max|diff|/max|ref| = {rel}")
            for _ in range(a.rounds):
                for kk, t in zip(keys, a.tags):
                    select(t, libs)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(5):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    times[kk].append(e0.elapsed_time(e1) / 5)
        base = statistics.median(times[keys[0]])
        for kk, t in zip(keys, a.tags):
            md = statistics.median(times[kk])
            extra = f" {fl / md / 1e9:.0f} TF/s" if a.what in ("attn", "fwdlse", "bwd", "mlbwd", "mlattn") else ""
            print(f"{variant} {a.what} {kk}: median {md:.4f} ms (min {min(times[kk]):.4f}){extra}  "
                  f"x{base / md:.3f} vs {a.tags[0]}", flush=True)


if __name__ == "__main__":
    main()
