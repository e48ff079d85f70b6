import math, os, sys, torch
ROOT = "/root/repo"
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd")); sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import vblade
from vblade import ops
from bench import realistic_qkv
dev = torch.device("cuda")
for variant in ("wan", "cog"):
    H, D = (48, 64) if variant == "cog" else (12, 128)
    m = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = m.gilbert_rearranger.seq_len
    q, k, v = realistic_qkv(H, L, D, 0, dev)
    rows = m._rows(dev)
    with torch.no_grad():
        _, mask = m.predict_mask(q, k)
        kp, vp, k_r, v_r = ops.pool_kv(k, v, m.sample_gap, rows, reordered=True)
        outs = []
        for i in range(4):
            outs.append(ops.attention_fwd(q, k_r, v_r, block_mask=mask, q_rows=rows, kp=kp, vp=vp,
                                          kp_log_bias=math.log(m.sample_gap), heavy_rows=m.force_tail).float())
        torch.cuda.synchronize()
    for i in range(1, 4):
        d = (outs[i] - outs[0]).abs()
        nz = (d > 0).nonzero()
        print(variant, "call", i, "vs 0: max", d.max().item(), "n_diff", nz.shape[0])
        if nz.shape[0]:
            print("  first diffs (b,h,row,d):", nz[:8].tolist())
            hs = nz[:, 1].unique().tolist(); rs = nz[:, 2].unique()
            print("  heads", hs[:10], "rows", rs[:10].tolist(), "n rows", rs.numel())
    d = (outs[2] - outs[1]).abs().max().item()
    print(variant, "call2 vs call1 max", d)
