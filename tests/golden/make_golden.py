"""Generate the golden fixtures in tests/golden/ by running the REFERENCE's own Python/Triton code
in this container (CPU, Triton interpreter). Run from the repo root:

    TRITON_INTERPRET=1 python tests/golden/make_golden.py

It reads /root/reference (present only in the build container, never on the GPU box). The
fixtures it writes are data (inputs + expected outputs), committed so the tests need no access
to the reference.

Harness shims (test infrastructure only, none of them part of the product):
  * ``attn_pooling_kernel.is_hip`` -> False: with no GPU driver Triton cannot answer it.
  * the third-party CUDA package ``block_sparse_attn`` (mit-han-lab/Block-Sparse-Attention,
    un-vendored) is absent; a stand-in module whose ``block_sparse_attn_func`` is the ORACLE's
    masked-softmax restatement (oracle/bsa_oracle.py) is registered so the reference glue can be
    imported. Fixtures produced through it therefore pin the reference GLUE (reorder, padding,
    sampling, Triton pooled scores, energy mask, pooling, combine, un-reorder), not that op.
  * the multi-level kernel wrapper's ``torch.cuda.device(...)`` context is a no-op (CPU tensors).
  * the CogVideoX GilbertRearranger hard-codes device='cuda' (cogvideo_blocksparseattn.py:127-128);
    it is built here through its own ``_gilbert3d_with_index`` with CPU index tensors.
"""
import os
import sys
import types

os.environ.setdefault("TRITON_INTERPRET", "1")

import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import bsa_oracle as O  # noqa: E402

REF = "/root/reference"
COG_TRAIN = os.path.join(REF, "cogvideox/train")
WAN_TRAIN = os.path.join(REF, "wanx/train")


def _install_block_sparse_stub():
    """Stand-in for the absent external package (see module docstring)."""
    pkg = types.ModuleType("block_sparse_attn")
    bp = types.ModuleType("block_sparse_attn.bert_padding")

    def unpad_input(hidden, mask):
        b, s = mask.shape
        idx = torch.nonzero(mask.flatten()).flatten()
        lens = mask.sum(-1, dtype=torch.int32)
        cu = torch.nn.functional.pad(torch.cumsum(lens, 0, dtype=torch.int32), (1, 0))
        return hidden.reshape(b * s, *hidden.shape[2:])[idx], idx, cu, int(lens.max())

    def pad_input(hidden, idx, b, s):
        out = torch.zeros(b * s, *hidden.shape[1:], dtype=hidden.dtype)
        out[idx] = hidden
        return out.reshape(b, s, *hidden.shape[1:])

    def block_sparse_attn_func(q, k, v, cu_q, cu_k, head_mask_type, streaming_info, base_blockmask,
                               max_q, max_k, p_dropout=0.0, deterministic=False, softmax_scale=None,
                               is_causal=False, exact_streaming=False, return_attn_probs=False):
        B = cu_q.numel() - 1
        H, D = q.shape[1], q.shape[2]
        qb = q.reshape(B, max_q, H, D).transpose(1, 2)
        kb = k.reshape(B, max_k, H, D).transpose(1, 2)
        vb = v.reshape(B, max_k, H, D).transpose(1, 2)
        # head_mask_type == 1 for every head -> renumbered 1..H (one base mask per head)
        out, lse = O.block_sparse_attention(qb, kb, vb, base_blockmask, softmax_scale)
        out = out.to(q.dtype).transpose(1, 2).reshape(B * max_q, H, D)
        return out, lse, None

    pkg.block_sparse_attn_func = block_sparse_attn_func
    bp.pad_input, bp.unpad_input = pad_input, unpad_input
    pkg.bert_padding = bp
    sys.modules["block_sparse_attn"] = pkg
    sys.modules["block_sparse_attn.bert_padding"] = bp


def _import_ref(train_dir, modname):
    sys.path.insert(0, train_dir)
    for k in [k for k in sys.modules if k.startswith("special_attentions_local")]:
        del sys.modules[k]
    import importlib
    mod = importlib.import_module(f"special_attentions_local.TrainRelated.{modname}")
    apk = importlib.import_module("special_attentions_local.TrainRelated.attn_pooling_kernel")
    apk.is_hip = lambda: False
    sys.path.remove(train_dir)
    return mod, apk


def gen_gilbert(out):
    sys.path.insert(0, os.path.join(COG_TRAIN, "special_attentions_local/utils"))
    from gilbert3d import gilbert3d
    res = {}
    for dims in [(8, 6, 4), (2, 2, 2), (3, 5, 7), (4, 4, 4), (5, 1, 3), (45, 30, 13), (52, 30, 21)]:
        w, h, d = dims
        pts = np.array(list(gilbert3d(w, h, d)), dtype=np.int64)
        res["perm_%dx%dx%d" % dims] = (pts[:, 0] + w * (pts[:, 1] + h * pts[:, 2])).astype(np.int32)
    np.savez_compressed(os.path.join(out, "gilbert_perms.npz"), **res)


def gen_pooled_scores(out, apk):
    res = {}
    cases = [("f32_d64", torch.float32, 1, 2, 11, 64), ("f16_d64", torch.float16, 1, 2, 11, 64),
             ("f32_d128", torch.float32, 2, 1, 9, 128), ("f16_d128", torch.float16, 1, 1, 9, 128),
             ("f32_nb40", torch.float32, 1, 1, 40, 64)]
    for name, dt, B, H, nb, D in cases:
        g = torch.Generator().manual_seed(sum(map(ord, name)))
        # block-structured scores so the rows are not all ties
        qs = torch.randn(B, H, nb * 32, D, generator=g)
        ks = torch.randn(B, H, nb * 32, D, generator=g)
        cent = torch.randn(B, H, nb, D, generator=g) * 1.5
        qs = (qs + cent.repeat_interleave(32, 2)).to(dt)
        ks = (ks + cent.repeat_interleave(32, 2)).to(dt)
        v = torch.zeros_like(qs)
        _, po = apk.attn_with_pooling(qs, ks, v, False, 1.0 / (D ** 0.5), 32)
        res[name + "_q"] = qs.float().numpy()
        res[name + "_k"] = ks.float().numpy()
        res[name + "_po"] = po.float().numpy()
        res[name + "_dtype"] = np.array(str(dt))
    np.savez_compressed(os.path.join(out, "pooled_scores.npz"), **res)


def gen_energy_masks(out, cog, wan, apk):
    res = {}
    g = torch.Generator().manual_seed(11)
    for name, mod, B, H, nb in [("cog", cog, 2, 3, 139), ("wan", wan, 1, 2, 256), ("cog_small", cog, 1, 2, 20)]:
        # mixture: smooth random rows and tie-heavy rows (many equal maxima as the predictor gives)
        po = torch.rand(B, H, nb, nb, generator=g) ** 4
        ties = (torch.rand(B, H, nb, nb, generator=g) < 0.15).float()
        po = torch.where(torch.rand(B, H, nb, 1, generator=g) < 0.5, po, torch.maximum(po, ties))
        po = po.bfloat16()
        po = (po.float() / po.float().sum(-1, keepdim=True).bfloat16().float()).bfloat16()
        if mod is cog:
            mx = torch.ones(B, H) * cog.max_retain_ratio
            mn = torch.ones(B, H) * cog.min_retain_ratio
        else:
            mx, mn = wan.max_retain_ratio, wan.min_retain_ratio
        m = mod.transfer_attn_to_mask(po, mode="energy", max_retain_ratio=mx, min_retain_ratio=mn,
                                      energy_threshold=0.95)
        res[name + "_po"] = po.float().numpy()
        res[name + "_mask"] = m.numpy()
    np.savez_compressed(os.path.join(out, "energy_masks.npz"), **res)


def gen_sampling(out, cog):
    res = {}
    for name, B, H, L, D, seed in [("a", 1, 2, 300, 64, 5), ("b", 2, 3, 256, 32, 9)]:
        g = torch.Generator().manual_seed(seed + 100)
        x = torch.randn(B, H, L, D, generator=g)
        xp = cog.pad_to_multiple(x, 128)
        torch.manual_seed(seed)
        s = cog.random_sample_tokens(xp, 128, 32)
        torch.manual_seed(seed)
        off = O.draw_sample_offsets(B, H)
        res[name + "_x"] = x.numpy()
        res[name + "_sampled"] = s.numpy()
        res[name + "_offsets"] = off.numpy().astype(np.int32)
        assert torch.equal(O.sample_tokens(O.pad_replicate(x, 128), off), s)
    np.savez_compressed(os.path.join(out, "sampling.npz"), **res)


def _cog_module(cog, w, h, d, text):
    cog.width, cog.height, cog.depth, cog.text_length = w, h, d, text
    gr = cog.GilbertRearranger.__new__(cog.GilbertRearranger)
    gr.width, gr.height, gr.depth, gr.text_length = w, h, d, text
    gr.total_elements = w * h * d
    c2i = gr._gilbert3d_with_index(w, h, d)
    o2g = [0] * gr.total_elements
    g2o = [0] * gr.total_elements
    for ci, oi in c2i.items():
        o2g[oi] = ci
        g2o[ci] = oi
    gr.original_order2gilbert_order = torch.tensor(o2g, dtype=torch.long)
    gr.gilbert_order2original_order = torch.tensor(g2o, dtype=torch.long)
    m = cog.AdaptiveBlockSparseAttnTrain.__new__(cog.AdaptiveBlockSparseAttnTrain)
    torch.nn.Module.__init__(m)
    m.gilbert_rearranger = gr
    m.sparsity_acc, m.sparsity_counter, m.use_rearrange = 0.0, 0, True
    return m


def gen_e2e(out, cog, wan):
    res = {}
    # (name, variant, dtype, B, H, (w,h,d), text, D, (min_ratio, max_ratio), sample_gap)
    cases = [
        ("cog_f32", "cog", torch.float32, 1, 1, (14, 10, 6), 26, 64, (0.15, 0.45), 15),
        ("cog_f16", "cog", torch.float16, 1, 2, (14, 10, 6), 26, 64, (0.15, 0.45), 15),
        ("cog_b2", "cog", torch.float32, 2, 1, (10, 6, 5), 26, 32, (0.05, 0.1), 15),
        ("wan_f32", "wan", torch.float32, 1, 1, (8, 8, 7), 0, 128, (0.05, 0.17), 30),
        ("wan_f16", "wan", torch.float16, 1, 2, (12, 8, 7), 0, 64, (0.2, 0.5), 30),
    ]
    for name, variant, dt, B, H, (w, h, d), text, D, (rmin, rmax), gap in cases:
        L = w * h * d + text
        g = torch.Generator().manual_seed(len(name) * 7 + B)
        cent = torch.randn(B, H, L // 16 + 1, D, generator=g).repeat_interleave(16, 2)[:, :, :L]
        q = (torch.randn(B, H, L, D, generator=g) + 1.5 * cent).to(dt)
        k = (torch.randn(B, H, L, D, generator=g) + 1.5 * cent).to(dt)
        v = torch.randn(B, H, L, D, generator=g).to(dt)
        if variant == "cog":
            cog.sample_gap, cog.min_retain_ratio, cog.max_retain_ratio = gap, rmin, rmax
            mod = _cog_module(cog, w, h, d, text)
            ref = cog
        else:
            wan.width, wan.height, wan.depth = w, h, d
            wan.sample_gap, wan.min_retain_ratio, wan.max_retain_ratio = gap, rmin, rmax
            mod = wan.AdaptiveBlockSparseAttnTrain()
            ref = wan
        torch.manual_seed(1234)
        with torch.no_grad():
            o = mod(q, k, v)
        torch.manual_seed(1234)
        qo = O.draw_sample_offsets(B, H)
        ko = O.draw_sample_offsets(B, H)
        # the predicted mask, recomputed by the reference's own functions on reordered inputs
        q_r, k_r, v_r = mod.gilbert_rearranger.rearrange(q, k, v)
        torch.manual_seed(1234)
        with torch.no_grad():
            po = ref.efficient_attn_with_pooling(q_r, k_r, v_r, block_size=128)
        if variant == "cog":
            mx = torch.ones(B, H) * ref.max_retain_ratio
            mn = torch.ones(B, H) * ref.min_retain_ratio
        else:
            mx, mn = ref.max_retain_ratio, ref.min_retain_ratio
        mask = ref.transfer_attn_to_mask(po, mode="energy", max_retain_ratio=mx, min_retain_ratio=mn,
                                         energy_threshold=0.95)
        store = np.float16 if dt == torch.float16 else np.float32
        res.update({name + "_q": q.numpy().astype(store), name + "_k": k.numpy().astype(store),
                    name + "_v": v.numpy().astype(store), name + "_out": o.numpy().astype(store),
                    name + "_ratios": np.array([rmin, rmax, gap], dtype=np.float64),
                    name + "_qoff": qo.numpy().astype(np.int32),
                    name + "_koff": ko.numpy().astype(np.int32),
                    name + "_po": po.float().numpy(), name + "_mask": mask.numpy(),
                    name + "_meta": np.array([B, H, w, h, d, text, D], dtype=np.int64),
                    name + "_dtype": np.array(str(dt)), name + "_variant": np.array(variant),
                    name + "_sparsity": np.array(mod.sparsity_acc)})
    np.savez_compressed(os.path.join(out, "adaptive_e2e.npz"), **res)


TRI = os.path.join(REF, "cogvideox/sample_evaluate")


class _Ctx:
    """Minimal autograd ctx for calling the reference kernel's _forward/_backward directly."""

    def save_for_backward(self, *t):
        self.saved_tensors = t


def _import_multilevel():
    """TRI/Triton/cogvideo_newattn.py and its kernel module (Triton interpreter on CPU)."""
    sys.path.insert(0, TRI)
    import importlib
    kml = importlib.import_module("Triton.kernels.block_sparse_attn_kernel_with_backward_9_10")
    kml.is_hip = lambda: False
    # the kernel wrapper enters torch.cuda.device(q.device.index); with no GPU driver that raises
    import contextlib
    torch.cuda.device = lambda idx: contextlib.nullcontext()
    apk = importlib.import_module("Triton.kernels.attn_pooling_kernel")
    apk.is_hip = lambda: False
    newattn = importlib.import_module("Triton.cogvideo_newattn")
    sys.path.remove(TRI)
    return newattn, kml


def gen_multilevel(out):
    """Multi-level path: level masks, KV pyramid, the Triton multi-level
    kernel's forward (out, l, m) and backward (dq, dk, dv), and the whole
    adaptive_block_sparse_attn of the VBench sampler module."""
    import ml_oracle as ML
    newattn, kml = _import_multilevel()
    res = {}
    g = torch.Generator().manual_seed(29)
    # level masks on tie-heavy bf16 rows
    for name, B, H, nb in [("m139", 1, 3, 139), ("m256", 1, 1, 256), ("m21", 2, 2, 21), ("m5", 1, 1, 5)]:
        po = torch.rand(B, H, nb, nb, generator=g) ** 4
        ties = (torch.rand(B, H, nb, nb, generator=g) < 0.15).float()
        po = torch.where(torch.rand(B, H, nb, 1, generator=g) < 0.5, po, torch.maximum(po, ties))
        po = (po / po.sum(-1, keepdim=True)).bfloat16()
        res["lm_" + name + "_po"] = po.float().numpy()
        res["lm_" + name + "_mask"] = newattn.transfer_attn_to_mask(po, newattn.mask_ratios).numpy()
    # KV pyramid (pad_to_multiple + pooling, fp16 storage)
    x = (torch.randn(1, 2, 300, 64, generator=g) * 2).half()
    xp = kml.pad_to_multiple(x, 128)
    x2 = kml.pooling(xp, 2)
    x4 = kml.pooling(x2, 2)
    x8 = kml.pooling(x4, 2)
    res["pyr_x"] = x.float().numpy()
    for nm, t in [("pad", xp), ("p2", x2), ("p4", x4), ("p8", x8)]:
        res["pyr_" + nm] = t.float().numpy()
    # the kernel itself: forward + backward on random level masks
    cases = [("f32_d64", torch.float32, 1, 2, 300, 64), ("f16_d64", torch.float16, 1, 2, 300, 64),
             ("f32_d128", torch.float32, 1, 1, 256, 128), ("f16_d128_b2", torch.float16, 2, 1, 200, 128)]
    for name, dt, B, H, L, D in cases:
        nb = (L + 127) // 128
        q = torch.randn(B, H, L, D, generator=g).to(dt)
        k = torch.randn(B, H, L, D, generator=g).to(dt)
        v = torch.randn(B, H, L, D, generator=g).to(dt)
        lv = torch.tensor([0, 1, 2, 4, 8], dtype=torch.int32)
        mask = lv[torch.randint(0, 5, (B, H, nb, nb), generator=g)]
        mask[..., -1] = 1          # every row attends somewhere
        do = torch.randn(B, H, L, D, generator=g).to(dt)
        ctx = _Ctx()
        o = kml._forward(ctx, q.clone().requires_grad_(), k, v, mask, D ** -0.5, 128, 128, 128)
        saved = ctx.saved_tensors
        lsum, mmax = saved[12], saved[13]
        dq, dk, dv, _, _ = kml._backward(ctx, do)
        res.update({"k_" + name + "_q": q.float().numpy(), "k_" + name + "_k": k.float().numpy(),
                    "k_" + name + "_v": v.float().numpy(), "k_" + name + "_mask": mask.numpy(),
                    "k_" + name + "_do": do.float().numpy(), "k_" + name + "_out": o.detach().float().numpy(),
                    "k_" + name + "_l": lsum.reshape(B, H, L).numpy(),
                    "k_" + name + "_m": mmax.reshape(B, H, L).numpy(),
                    "k_" + name + "_dq": dq.float().numpy(), "k_" + name + "_dk": dk.float().numpy(),
                    "k_" + name + "_dv": dv.float().numpy(), "k_" + name + "_dtype": np.array(str(dt))})
    # the whole adaptive_block_sparse_attn (sampler + Triton pooled scores + level mask + kernel)
    for name, dt, H, L, D in [("e2e_f32", torch.float32, 1, 2600, 64), ("e2e_f16", torch.float16, 1, 2600, 64)]:
        store = np.float16 if dt == torch.float16 else np.float32
        cent = torch.randn(1, H, L // 16 + 1, D, generator=g).repeat_interleave(16, 2)[:, :, :L]
        q = (torch.randn(1, H, L, D, generator=g) + 1.5 * cent).to(dt)
        k = (torch.randn(1, H, L, D, generator=g) + 1.5 * cent).to(dt)
        v = torch.randn(1, H, L, D, generator=g).to(dt)
        torch.manual_seed(4321)
        with torch.no_grad():
            o, sp = newattn.adaptive_block_sparse_attn(q, k, v)
        torch.manual_seed(4321)
        qo = O.draw_sample_offsets(1, H)
        ko = O.draw_sample_offsets(1, H)
        torch.manual_seed(4321)
        with torch.no_grad():
            po = newattn.efficient_attn_with_pooling(q, k, v, block_size=128)
        mask = newattn.transfer_attn_to_mask(po, newattn.mask_ratios)
        res.update({name + "_q": q.float().numpy().astype(store), name + "_k": k.float().numpy().astype(store),
                    name + "_v": v.float().numpy().astype(store), name + "_out": o.float().numpy().astype(store),
                    name + "_qoff": qo.numpy().astype(np.int32), name + "_koff": ko.numpy().astype(np.int32),
                    name + "_po": po.float().numpy(), name + "_mask": mask.numpy(),
                    name + "_sparsity": np.array(sp), name + "_dtype": np.array(str(dt))})
    assert abs(ML.density() - (1 - res["e2e_f32_sparsity"])) < 1e-12
    np.savez_compressed(os.path.join(out, "multilevel.npz"), **res)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "multilevel":   # regenerate only multilevel.npz
        gen_multilevel(HERE)
        return
    _install_block_sparse_stub()
    cog, apk = _import_ref(COG_TRAIN, "cogvideo_blocksparseattn")
    wan, _ = _import_ref(WAN_TRAIN, "wanx_blocksparseattn")
    gen_gilbert(HERE)
    gen_pooled_scores(HERE, apk)
    gen_energy_masks(HERE, cog, wan, apk)
    gen_sampling(HERE, cog)
    gen_e2e(HERE, cog, wan)
    gen_multilevel(HERE)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
