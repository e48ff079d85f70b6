#!/usr/bin/env python3
"""Per-workgroup timeline of the predictor's launch (diagnostic build: VB_PRED_FLAGS=-DVB_PRED_TRACE=1
tools/build_variant.sh ptrace) or of the attention kernel's (what = attn; VB_EXTRA_FLAGS=-DVB_ATTN_TRACE=1
tools/build_variant.sh atrace): start and per-wave end times (s_memrealtime, 10 ns), CU and XCD of
every workgroup, and the shader clock over it. Prints how long the workgroups live, when they start,
and how many are resident per CU over the launch (slot utilisation, the tail).
usage: python tools/diag/pred_trace.py [cog|wan] [pred|call|attn] [TAG]
(attn: TRACE_PERSIST=0 traces the one-workgroup-per-q-block launch; with the persistent launch every
work item is one record, and the gaps between a workgroup's items count as idle slot time)"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)
import ab  # noqa: E402
import vblade  # noqa: E402
from vblade import _lib  # noqa: E402
from bench import realistic_qkv  # noqa: E402

variant = sys.argv[1] if len(sys.argv) > 1 else "cog"
what = sys.argv[2] if len(sys.argv) > 2 else "pred"
tag = sys.argv[3] if len(sys.argv) > 3 else ("atrace" if what == "attn" else "ptrace")
lib = ab.load(tag)
getter = getattr(lib, "vb_debug_attn_trace" if what == "attn" else "vb_debug_pred_trace")
getter.restype = ctypes.c_int
getter.argtypes = [ctypes.c_void_p, ctypes.c_int]
_lib._lib = lib
dev = torch.device("cuda")
H, D = (48, 64) if variant == "cog" else (12, 128)
m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
m.persistent = os.environ.get("TRACE_PERSIST", "1") != "0"   # the attention launch's dispatch form
L = m.gilbert_rearranger.seq_len
q, k, v = realistic_qkv(H, L, D, 0, dev)
qo = vblade.draw_sample_offsets(1, H, dev)
ko = vblade.draw_sample_offsets(1, H, dev)
N = 8192
F = 10
buf = (ctypes.c_ulonglong * (F * N))()
with torch.no_grad():
    for _ in range(5):
        m.predict_mask(q, k, qo, ko) if what == "pred" else m(q, k, v)
    torch.cuda.synchronize()
    getter(buf, N)   # clear
    m.predict_mask(q, k, qo, ko) if what == "pred" else m(q, k, v)
    torch.cuda.synchronize()
    assert getter(buf, N) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(N, F).astype(np.int64)
a = a[a[:, 0] > 0]
out = os.environ.get("TRACE_OUT")
if out:   # the raw rows, for offline analysis
    np.save(out, a)
t0 = a[:, 0].min()
start = (a[:, 0] - t0) / 100.0          # us
ends = a[:, 1:5].astype(np.float64)
ends[ends == 0] = np.nan
end = (np.nanmax(ends, 1) - t0) / 100.0
wave_end = (ends - t0) / 100.0
kind = a[:, 7]
hw, xcc = a[:, 5], a[:, 6]
cu = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 15)
print(f"{variant} {what}: {len(a)} workgroups traced ({(kind == 1).sum()} pooling), launch span {np.nanmax(end):.1f} us")
for kd, name in ((0, "score"), (1, "pool")):
    s = kind == kd
    if not s.any():
        continue
    dur = end[s] - start[s]
    print(f"  {name:5s}: start p0/p50/p100 {np.percentile(start[s], 0):6.1f} {np.percentile(start[s], 50):6.1f} "
          f"{start[s].max():6.1f} us; duration p10/p50/p90/max {np.percentile(dur, 10):6.1f} {np.median(dur):6.1f} "
          f"{np.percentile(dur, 90):6.1f} {dur.max():6.1f} us; last end {end[s].max():6.1f}")
    clk = (a[s, 9] - a[s, 8]) / ((a[s, 1] - a[s, 0]) / 100.0) / 1e3   # shader cycles per us -> GHz
    print(f"         clock over the workgroup (wave 0) p10/p50/p90 {np.percentile(clk, 10):.2f} {np.median(clk):.2f} "
          f"{np.percentile(clk, 90):.2f} GHz")
    ws = np.nanmax(wave_end[s], 1) - np.nanmin(wave_end[s], 1)
    print(f"         wave end spread within a workgroup p50/p90 {np.median(ws):5.1f} {np.percentile(ws, 90):5.1f} us")
ncu = len(np.unique(cu))
end = np.where(np.isnan(end), start, end)
T = np.arange(0, end.max(), 1.0)
res = np.array([((start <= t) & (end > t)).sum() for t in T]) / ncu
print(f"  {ncu} CUs; resident workgroups per CU over time (1 us bins, every 10th):")
print("   " + " ".join(f"{x:.1f}" for x in res[::max(1, len(res) // 40)]))
print(f"  mean residency {res.mean():.2f} per CU; score-only residency "
      f"{np.mean([((start <= t) & (end > t) & (kind == 0)).sum() for t in T]) / ncu:.2f}")
per_cu = np.bincount(np.unique(cu, return_inverse=True)[1])
print(f"  workgroups per CU min/median/max {per_cu.min()} {int(np.median(per_cu))} {per_cu.max()}")
# duration against the residency of the workgroup's CU while it ran (is a workgroup faster alone?)
cu_id = np.unique(cu, return_inverse=True)[1]
occ = np.zeros(len(a))
for i in range(len(a)):
    same = (cu_id == cu_id[i]) & (start < end[i]) & (end > start[i])
    occ[i] = same.sum()
dur = end - start
for lo, hi in ((1, 1.5), (1.5, 2.5), (2.5, 3.5), (3.5, 9)):
    s_ = (occ >= lo) & (occ < hi) & (kind == 0)
    if s_.any():
        print(f"  co-resident workgroups on its CU {lo:.1f}-{hi:.1f}: {s_.sum():5d} workgroups, duration p50 {np.median(dur[s_]):6.1f} us")
