#!/usr/bin/env python3
"""Per-segment cycle stamps of the one-wave-per-SIMD forward (vb_attn_fwd1.hip) from a diagnostic
build (VB_EXTRA_FLAGS=-DVB_DIAG=1 tools/build_variant.sh TAG): wait+barrier, region A, region B, end
of iteration per tile, prologue and epilogue per workgroup (cycles per wave, s_memtime).
usage: python tools/diag/fwd1_stamps.py TAG [cog|wan]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import vblade  # noqa: E402
from vblade import _lib, ops  # noqa: E402
from ab import load  # noqa: E402
from bench import realistic_qkv  # noqa: E402

tag = sys.argv[1]
variant = sys.argv[2] if len(sys.argv) > 2 else "cog"
lib = load(tag)
lib.vb_fwd1_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib._lib = lib
dev = torch.device("cuda")
H, D = (48, 64) if variant == "cog" else (12, 128)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, gather_kv=False)
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(H, L, D, 0, dev)
rows = m._rows(dev)
qo, ko = vblade.draw_sample_offsets(1, H, dev), vblade.draw_sample_offsets(1, H, dev)
_, mask = m.predict_mask(q, k, qo, ko)
kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
fn = lambda: ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp, vp=vp,  # noqa
                               kp_log_bias=m._log_gap(q.dtype), heavy_rows=m.force_tail)
for _ in range(20):
    fn()
buf = (ctypes.c_ulonglong * 16)()
lib.vb_fwd1_stamps(buf, 1)
n = 20
for _ in range(n):
    fn()
lib.vb_fwd1_stamps(buf, 1)
tiles, wgs = buf[8] / n, buf[9] / n
names = ["wait+barrier", "region A", "region B", "end of iteration"]
print(f"{variant}: {tiles / wgs:.1f} tiles per workgroup, {wgs:.0f} workgroups per launch")
tot = sum(buf[i] for i in range(4))
for i, nm in enumerate(names):
    print(f"  {nm:18s} {buf[i] / n / (4 * tiles):8.1f} cycles per wave-tile  ({100 * buf[i] / tot:.1f} %)")
print(f"  {'loop total':18s} {tot / n / (4 * tiles):8.1f}")
print(f"  prologue {buf[4] / n / (4 * wgs):.0f}, epilogue {buf[5] / n / (4 * wgs):.0f} cycles per wave and workgroup")
