"""GPU: the training steps (vblade.train) through the HIP sparse attention — LoRA gradients of a
stand-in block match the same block whose attention is the oracle (forward and the explicit
reference-semantics backward of oracle/bsa_oracle.py, run on the CPU as the checker), at a small
length and for one head at the full CogVideoX length; the two-model TDM step (student + fake with
sparse attention, dense CFG teacher) gives the oracle-attention step's losses and gradients; and a
few optimizer steps lower the loss with deterministic results."""
import pytest
import torch
import torch.nn as nn

import bsa_oracle as O
from vblade import train as T

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import vblade
    vblade.load_library()


W, Hh, Dp, TEXT = 10, 6, 5, 26     # L = 326 (3 blocks, text tail)


class FixedMaskAttention(nn.Module):
    """The module under test with its mask pinned (the predictor is tested elsewhere)."""

    def __init__(self, mask):
        super().__init__()
        import vblade
        self.m = vblade.AdaptiveBlockSparseAttn("cog", width=W, height=Hh, depth=Dp, text_length=TEXT,
                                                log_every=0)
        self.mask = mask

    def forward(self, q, k, v):
        return self.m(q, k, v, block_mask=self.mask)


class _OracleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, mask, cfg):
        qc, kc, vc = (t.detach().cpu() for t in (q, k, v))
        fwd = O.adaptive_attention(qc, kc, vc, cfg, None, None, mask=mask.cpu().bool())
        ctx.saved = (qc, kc, vc, cfg, fwd)
        return fwd["out"].to(q.dtype).to(q.device)

    @staticmethod
    def backward(ctx, dout):
        qc, kc, vc, cfg, fwd = ctx.saved
        dq, dk, dv = O.adaptive_attention_bwd(qc, kc, vc, dout.cpu(), cfg, fwd)
        dev, dt = dout.device, dout.dtype
        return dq.to(dt).to(dev), dk.to(dt).to(dev), dv.to(dt).to(dev), None, None


class OracleAttention(nn.Module):
    def __init__(self, mask):
        super().__init__()
        self.mask = mask
        self.cfg = O.AdaptiveConfig.cogvideox(width=W, height=Hh, depth=Dp, text_length=TEXT)

    def forward(self, q, k, v):
        return _OracleFn.apply(q, k, v, self.mask, self.cfg)


def _mask(H, nb, seed=5):
    g = torch.Generator().manual_seed(seed)
    m = torch.rand(1, H, nb, nb, generator=g) < 0.5
    m[..., -2:] = True
    m[..., -2:, :] = True
    return m.to(torch.uint8)


def _build(attn, heads=2, hidden=128, rank=8):
    m = T.StandInTransformer(1, hidden, heads, rank, float(rank), attn, dtype=torch.bfloat16, device=DEV, seed=0)
    g = torch.Generator().manual_seed(4)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("lora_B"):
                p.copy_((torch.randn(p.shape, generator=g) * 0.05).to(DEV))
    return m


def test_lora_grads_through_hip_attention_match_oracle():
    L = W * Hh * Dp + TEXT
    heads, hidden = 2, 128
    nb = (L + 127) // 128
    mask = _mask(heads, nb).to(DEV)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV)
    y = torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV)
    grads = []
    for attn in (FixedMaskAttention(mask), OracleAttention(mask)):
        m = _build(attn.to(DEV) if isinstance(attn, FixedMaskAttention) else attn)
        T.pseudo_huber(m(x), y, 1e-3).backward()
        grads.append([p.grad.float().cpu() for p in m.lora_parameters()])
    for a, b in zip(*grads):
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert rel <= 3e-2, rel


def test_train_steps_lower_the_loss_deterministically():
    L = W * Hh * Dp + TEXT
    nb = (L + 127) // 128
    mask = _mask(2, nb).to(DEV)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(2, L, 128, generator=g).bfloat16().to(DEV)
    y = torch.randn(2, L, 128, generator=g).bfloat16().to(DEV)
    runs = []
    for _ in range(2):
        m = _build(FixedMaskAttention(mask).to(DEV))
        step = T.TrainStep(m, lr=5e-3, accum=2)
        losses = [float(step([(x[:1], y[:1]), (x[1:], y[1:])])) for _ in range(4)]
        runs.append((losses, [p.detach().clone() for p in m.lora_parameters()]))
    assert runs[0][0][-1] < runs[0][0][0]
    assert runs[0][0] == runs[1][0]
    for a, b in zip(runs[0][1], runs[1][1]):
        assert torch.equal(a, b)


class _RecordingTDM(T.TDMTrainStep):
    """Records both models' LoRA gradients (after the reducers, before clipping) at each step."""

    def _step(self, params, opt, red):
        if red is not None:
            red.finish()
        self.recorded = getattr(self, "recorded", []) + [[p.grad.float().cpu().clone() for p in params]]
        return super()._step(params, opt, None)


def test_tdm_step_through_hip_attention_matches_oracle_attention():
    """TDMTrainStep (fake-score update then generator update, train_cogvideo_tdm.py:1640-1737) with
    the student's and fake model's sparse attention on the HIP path vs the same step with the
    oracle as attention (the dense CFG teacher is the same SDPA in both): equal losses and LoRA
    gradients of both models within the bf16 tolerance of the LoRA-gradient test."""
    L = W * Hh * Dp + TEXT
    heads, hidden = 2, 128
    nb = (L + 127) // 128
    mask = _mask(heads, nb).to(DEV)
    g = torch.Generator().manual_seed(8)
    mbs = [(torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV),
            torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV),
            (torch.rand(1, 1, 1, generator=g) + 0.5).to(DEV),
            (torch.randn(1, 1, hidden, generator=g) * 0.5).bfloat16().to(DEV)) for _ in range(2)]
    runs = []
    for attn in (FixedMaskAttention(mask).to(DEV), OracleAttention(mask)):
        step = _RecordingTDM(_build(attn), lr=1e-3, lr_fake=1e-3, accum=2, cfg=3.5)
        assert isinstance(step.teacher.transformer_blocks[0].inner_attention, T.DenseAttention)
        lf, lg = step(mbs)
        runs.append((float(lf), float(lg), step.recorded))
    (lf_h, lg_h, rec_h), (lf_o, lg_o, rec_o) = runs
    assert abs(lf_h - lf_o) <= 2e-2 * abs(lf_o) + 1e-6
    assert abs(lg_h - lg_o) <= 2e-2 * abs(lg_o) + 1e-6
    assert len(rec_h) == len(rec_o) == 2          # fake model, then student
    for gh, go in zip(rec_h, rec_o):
        for a, b in zip(gh, go):
            rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
            assert rel <= 3e-2, rel


def test_lora_grads_full_length_one_head_match_oracle():
    """The LoRA-gradient check at the real CogVideoX length (L = 17776, one 64-dim head, the
    reference's forced tail rows/columns and a 12 % random block mask)."""
    L = 45 * 30 * 13 + 226
    nb = (L + 127) // 128
    g = torch.Generator().manual_seed(9)
    m = torch.rand(1, 1, nb, nb, generator=g) < 0.12
    m[..., -2:] = True
    m[..., -2:, :] = True
    mask = m.to(torch.uint8).to(DEV)

    class _Full(nn.Module):
        def __init__(self):
            super().__init__()
            import vblade
            self.m = vblade.AdaptiveBlockSparseAttn("cog", log_every=0)

        def forward(self, q, k, v):
            return self.m(q, k, v, block_mask=mask)

    class _FullOracle(nn.Module):
        cfg = O.AdaptiveConfig.cogvideox()

        def forward(self, q, k, v):
            return _OracleFn.apply(q, k, v, mask, self.cfg)

    hidden = 64
    x = torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV)
    y = torch.randn(1, L, hidden, generator=g).bfloat16().to(DEV)
    grads = []
    for attn in (_Full().to(DEV), _FullOracle()):
        mdl = _build(attn, heads=1, hidden=hidden, rank=8)
        T.pseudo_huber(mdl(x), y, 1e-3).backward()
        grads.append([p.grad.float().cpu() for p in mdl.lora_parameters()])
    for a, b in zip(*grads):
        rel = ((a - b).norm() / b.norm().clamp_min(1e-12)).item()
        assert rel <= 3e-2, rel
