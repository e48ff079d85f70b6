"""CPU: the C ABI library loads, exports every symbol include/vblade.h declares, its ctypes
struct layouts match the C header (compiled with gcc), host-side entry points behave, and the
argument validation returns the documented error codes without touching a GPU."""
import ctypes
import os
import re
import subprocess
import tempfile

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

HEADER = os.path.join(ROOT, "include", "vblade.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vb_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from vblade import _lib
    return _lib.load()


def test_every_declared_symbol_is_exported_and_bound(lib):
    from vblade import _lib
    names = _declared_functions()
    assert names, "no functions parsed from vblade.h"
    for n in names:
        assert hasattr(lib, n), f"{n} missing from libvblade_hip.so"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    assert set(_lib.SIGNATURES) == set(names)


def test_abi_version(lib):
    from vblade import _lib
    assert lib.vb_abi_version() == _lib.ABI_VERSION == 4


def test_struct_layouts_match_header():
    """sizeof/offsetof of vb_attn_args and vb_predict_args from gcc == the ctypes mirrors."""
    from vblade._lib import AttnArgs, BwdArgs, MlAttnArgs, MlBwdArgs, PredictArgs
    structs = (("vb_attn_args", AttnArgs), ("vb_predict_args", PredictArgs),
               ("vb_attn_bwd_args", BwdArgs), ("vb_ml_attn_args", MlAttnArgs),
               ("vb_ml_attn_bwd_args", MlBwdArgs))
    fields = {st: [f[0] for f in cls._fields_] for st, cls in structs}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for st, fl in fields.items():
        lines.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fl:
            lines.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "l.c")
        open(c, "w").write("\n".join(lines))
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-std=c99", c, "-o", exe])
        out = subprocess.check_output([exe]).decode().split("\n")
    got = dict(line.split() for line in out if line)
    for st, cls in structs:
        assert int(got[st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(got[f"{st}.{f}"]) == getattr(cls, f).offset, f"{st}.{f}"


def test_gilbert_perm_host_entry_matches_reference_fixture(lib):
    from vblade import ops
    z = np.load(os.path.join(GOLDEN, "gilbert_perms.npz"))
    for key in z.files:
        w, h, d = map(int, key.split("_")[1].split("x"))
        assert np.array_equal(ops.gilbert_perm(w, h, d), z[key]), key


def test_invalid_arguments_return_codes_without_gpu(lib):
    from vblade import _lib
    buf = np.zeros(8, dtype=np.int32)
    assert lib.vb_gilbert3d_perm(0, 2, 2, buf.ctypes.data) == _lib.VB_ERR_INVALID
    assert b"positive" in lib.vb_last_error()
    # dropout is rejected before any device work
    rc = lib.vb_block_sparse_attn_fwd(1, 1, 1, 1, 1, None, None, None, 1, 1, 64, 128, 128,
                                      0.1, 1, 0.0, 0, 0, 0, 1, 1, 0, None)
    assert rc == _lib.VB_ERR_UNSUPPORTED and b"dropout" in lib.vb_last_error()
    rc = lib.vb_block_sparse_attn_fwd(1, 1, 1, 1, 1, None, None, None, 1, 1, 64, 128, 128,
                                      0.0, 1, 0.0, 1, 0, 0, 1, 1, 0, None)
    assert rc == _lib.VB_ERR_UNSUPPORTED
    # SURVEY Appendix B's mask_head_mode: per_head (0) and shared_head0 (1) only
    rc = lib.vb_block_sparse_attn_fwd(1, 1, 1, 1, 1, None, None, None, 1, 1, 64, 128, 128,
                                      0.0, 1, 0.0, 0, 0, 0, 1, 1, 2, None)
    assert rc == _lib.VB_ERR_INVALID and b"mask_head_mode" in lib.vb_last_error()
    a = _lib.AttnArgs()
    assert lib.vb_attn_fwd(ctypes.byref(a), None) == _lib.VB_ERR_INVALID
    p = _lib.PredictArgs()
    assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
    assert lib.vb_energy_mask(None, 1, 1, 1, 1, 0.95, 1, 1, 0, 0, None, None, None) == _lib.VB_ERR_INVALID
    assert lib.vb_pool_kv(None, None, None, None, None, 1, 1, 1, 64, 15, 0, None, None, None, None, None) == _lib.VB_ERR_INVALID
    assert lib.vb_lse_combine(None, None, None, None, 1, 1, 1, 64, 15.0, 0, None, None, None) == _lib.VB_ERR_INVALID
    b = _lib.BwdArgs()
    assert lib.vb_attn_bwd(ctypes.byref(b), None) == _lib.VB_ERR_INVALID
    b.B = b.H = 1
    b.Lq = b.Lk = 128
    b.D = 96
    assert lib.vb_attn_bwd(ctypes.byref(b), None) == _lib.VB_ERR_UNSUPPORTED
    assert b"head_dim" in lib.vb_last_error()
    # kernel_select: unknown bits refused before any launch (ABI 4)
    b.D = 64
    b.q = b.k = b.v = b.out = b.lse = b.dout = b.dq = b.dk = b.dv = 1 << 20
    b.kernel_select = 8
    assert lib.vb_attn_bwd(ctypes.byref(b), None) == _lib.VB_ERR_INVALID
    assert b"kernel_select" in lib.vb_last_error()
    b.kernel_select = 0
    # workspace sizing is pure host arithmetic
    assert lib.vb_attn_bwd_workspace_size(ctypes.byref(b)) >= 2 * 64 * 4 * 4
    assert lib.vb_block_sparse_attn_bwd_workspace_size(1, 1, 128) > 0
    rc = lib.vb_block_sparse_attn_bwd(*([None] * 11), 1, 1, 64, 128, 128, 0.1, 0.0, 0, 0, 1, 0,
                                      None, None, None, None, 0, 0, None)
    assert rc == _lib.VB_ERR_UNSUPPORTED and b"dropout" in lib.vb_last_error()
    rc = lib.vb_block_sparse_attn_bwd(*([None] * 11), 1, 1, 64, 128, 128, 0.0, 0.0, 0, 0, 1, 0,
                                      None, None, None, None, 0, 5, None)
    assert rc == _lib.VB_ERR_INVALID and b"mask_head_mode" in lib.vb_last_error()
    # multi-level entry points
    assert lib.vb_kv_pyramid_rows(17776) == 15 * 17792 // 8
    assert lib.vb_kv_pyramid_rows(128) == 240
    m = _lib.MlAttnArgs()
    assert lib.vb_ml_attn_fwd(ctypes.byref(m), None) == _lib.VB_ERR_INVALID
    m.B = m.H = 1
    m.L = 300
    m.D = 80
    m.q = m.kpyr = m.vpyr = m.level_mask = m.out = 16
    assert lib.vb_ml_attn_fwd(ctypes.byref(m), None) == _lib.VB_ERR_UNSUPPORTED
    mb = _lib.MlBwdArgs()
    assert lib.vb_ml_attn_bwd(ctypes.byref(mb), None) == _lib.VB_ERR_INVALID
    mb.B = mb.H = 1
    mb.L, mb.D = 300, 64
    assert lib.vb_ml_attn_bwd_workspace_size(ctypes.byref(mb)) > 7 * 384 // 8 * 64 * 4 * 2
    mb.q = mb.kpyr = mb.vpyr = mb.level_mask = mb.out = mb.lse = mb.dout = mb.dq = mb.dk = mb.dv = 1 << 20
    mb.kernel_select = _lib.VB_BWD_SEL_DQ_RING4     # the multi-level dQ has one ring
    assert lib.vb_ml_attn_bwd(ctypes.byref(mb), None) == _lib.VB_ERR_INVALID
    assert b"kernel_select" in lib.vb_last_error()
    assert lib.vb_kv_pyramid(None, None, None, None, None, 1, 1, 1, 64, 0, None, None, None) == _lib.VB_ERR_INVALID
    vals = np.array([3], dtype=np.int32)
    se = np.array([0.0, 1.0], dtype=np.float64)
    rc = lib.vb_level_mask(16, 1, 1, 4, 4, 1, vals.ctypes.data, se[:1].ctypes.data, se[1:].ctypes.data,
                           0, 16, None)
    assert rc == _lib.VB_ERR_INVALID and b"band values" in lib.vb_last_error()


def test_mask_predict_option_checks_without_gpu(lib):
    """vb_mask_predict's host-side checks of the round-3 options run before any launch: Philox
    draws exclusive with rand_q/rand_k and limited to one torch.rand grid-stride pass, level bands
    validated and needing a mask output."""
    from vblade import _lib
    def args(B=1, H=2, L=1000):
        p = _lib.PredictArgs()
        p.q = p.k = p.q_off = p.k_off = p.po = p.mask = 1 << 20
        p.B, p.H, p.L, p.D, p.block, p.num_keep = B, H, L, 64, 128, 32
        p.q_stride = p.k_stride = (H * L * 64, L * 64, 64)
        p.min_keep = p.max_keep = 1
        p.workspace = 1 << 24
        p.workspace_bytes = lib.vb_mask_predict_workspace_size(ctypes.byref(p))
        return p
    p = args()
    p.philox, p.rand_q, p.rand_k = 1, 1 << 20, 1 << 20
    assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
    assert b"exclusive" in lib.vb_last_error()
    p = args(B=2, H=2049)                         # 2*2049*128 > 524288 (CUs x threads per CU)
    p.philox = 1
    rc = lib.vb_mask_predict(ctypes.byref(p), None)
    import torch
    if torch.cuda.is_available():   # the bound is the device's own CUs x max threads per CU
        pr = torch.cuda.get_device_properties(0)
        assert rc == _lib.VB_ERR_UNSUPPORTED
        assert str(pr.multi_processor_count * pr.max_threads_per_multi_processor).encode() in lib.vb_last_error()
    else:                           # no device to query: refused before any launch
        assert rc == _lib.VB_ERR_LAUNCH and b"CU count" in lib.vb_last_error()
    vals = np.array([3], dtype=np.int32)
    se = np.array([0.0, 1.0], dtype=np.float64)
    p = args()
    p.mask_level, p.level_bands = 1, 1
    p.level_band_value, p.level_band_start, p.level_band_end = vals.ctypes.data, se[:1].ctypes.data, se[1:].ctypes.data
    assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
    assert b"band values" in lib.vb_last_error()
    p = args()
    p.mask_level, p.level_bands, p.level_band_value = 1, 9, vals.ctypes.data
    assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
    p = args()
    p.mask, p.mask_level = None, 1
    assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
    assert b"mask output" in lib.vb_last_error()
    # the kept counts come from the energy rule only: refused with the level mask or scores only
    for level, mask in ((1, 1 << 20), (0, None)):
        p = args()
        p.mask_rows_kept = 1 << 20
        p.mask = mask
        if level:
            p.mask_level, p.level_bands = 1, 1
            p.level_band_value, p.level_band_start, p.level_band_end = (
                np.array([1], dtype=np.int32).ctypes.data, se[:1].ctypes.data, se[1:].ctypes.data)
        assert lib.vb_mask_predict(ctypes.byref(p), None) == _lib.VB_ERR_INVALID
        assert b"mask_rows_kept" in lib.vb_last_error()


def test_level_bands_follow_mask_ratio_dict_order():
    from vblade import ops
    vals, st, en = ops._level_bands({8: (0.25, 0.5), 1: (0.0, 0.05)})
    assert vals.tolist() == [8, 1] and st.tolist() == [0.25, 0.0] and en.tolist() == [0.5, 0.05]
    vals, _, _ = ops._level_bands(None)
    assert vals.tolist() == [int(v) for v in ops.ML_MASK_RATIOS]
    assert ops.claim_rand_draws("cuda", ops.RAND_ONE_PASS_NUMEL + 1) is None   # past one pass: torch.rand


def test_ops_refuse_cpu_tensors():
    """The product path has no CPU fallback: CPU tensors raise."""
    import torch
    from vblade import ops
    q = torch.zeros(1, 1, 128, 64, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="HIP"):
        ops.attention_fwd(q, q, q)
    lse = torch.zeros(1, 1, 128)
    with pytest.raises(RuntimeError, match="HIP"):
        ops.attention_bwd(q, q, q, q, q, lse)


def test_module_config_and_retain_counts():
    import vblade
    from vblade.attention import retain_counts
    m = vblade.AdaptiveBlockSparseAttn("cog")
    assert m.gilbert_rearranger.seq_len == 17776 and m.force_tail == 2 and m.sample_gap == 15
    w = vblade.AdaptiveBlockSparseAttn("wan")
    assert w.gilbert_rearranger.seq_len == 32760 and w.force_tail == 0 and w.sample_gap == 30
    assert retain_counts(139, 0.05, 0.1, "cog") == (6, 13)
    assert retain_counts(256, 0.05, 0.17, "wan") == (12, 43)
    rows = m.gilbert_rearranger.rows.long()
    assert sorted(rows.tolist()) == list(range(17776))
    assert rows[-226:].tolist() == list(range(226))  # text tail, in order


def test_gilbert_rearranger_round_trip_cpu():
    import torch
    import vblade
    g = vblade.GilbertRearranger(8, 6, 4, text_length=10)
    x = torch.randn(2, 3, 8 * 6 * 4 + 10, 16)
    q, k, v = g.rearrange(x, x, x)
    assert torch.equal(q[..., -10:, :], x[..., :10, :])
    assert torch.equal(g.reversed_rearrange(q), x)
