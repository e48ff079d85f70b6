"""CPU: the TDM training-step integration (vblade.train) — LoRA layers, gradient checkpointing,
the bucketed data-parallel gradient all-reduce (gloo, world size 2) and the diffusers LoRA
checkpoint format. The attention inside is a CPU stand-in here (plain softmax attention); the
GPU tests (test_gpu_train.py) run TrainStep and TDMTrainStep through the HIP sparse attention."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from vblade import train as T


class CpuAttention(nn.Module):
    def forward(self, q, k, v):
        return F.scaled_dot_product_attention(q.float(), k.float(), v.float()).to(q.dtype)


def _model(layers=2, hidden=64, heads=4, rank=4, ckpt=True, seed=0):
    return T.StandInTransformer(layers, hidden, heads, rank, float(rank), CpuAttention(),
                                gradient_checkpointing=ckpt, dtype=torch.float32, seed=seed)


def _batch(n, L=32, hidden=64, seed=1):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, L, hidden, generator=g), torch.randn(n, L, hidden, generator=g)


def _perturb_b(model, seed=3):
    # LoRA B starts at zero (so A gets no gradient on the first step); give it values
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if n.endswith("lora_B"):
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)


def test_lora_linear_starts_as_the_base_layer():
    lin = T.LoRALinear(8, 6, 2, 2.0, dtype=torch.float32, generator=torch.Generator().manual_seed(0))
    x = torch.randn(3, 8)
    assert torch.equal(lin(x), F.linear(x, lin.weight, lin.bias))
    assert [n for n, p in lin.named_parameters() if p.requires_grad] == ["lora_A", "lora_B"]


def test_gradient_checkpointing_gives_identical_grads():
    grads = []
    for ckpt in (False, True):
        m = _model(ckpt=ckpt)
        _perturb_b(m)
        x, y = _batch(2)
        T.pseudo_huber(m(x), y, 1e-3).backward()
        grads.append([p.grad.clone() for p in m.lora_parameters()])
    for a, b in zip(*grads):
        assert torch.allclose(a, b, atol=1e-7, rtol=1e-6)


def test_train_step_accumulation_equals_full_batch():
    m1, m2 = _model(), _model()
    _perturb_b(m1)
    _perturb_b(m2)
    x, y = _batch(4)
    s1 = T.TrainStep(m1, lr=1e-2, accum=1)
    s2 = T.TrainStep(m2, lr=1e-2, accum=2)
    s1([(x, y)])
    s2([(x[:2], y[:2]), (x[2:], y[2:])])
    for a, b in zip(m1.lora_parameters(), m2.lora_parameters()):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5)


def test_lora_checkpoint_round_trip_and_key_format(tmp_path):
    m = _model()
    _perturb_b(m)
    path = T.save_lora_weights(str(tmp_path), m)
    assert os.path.basename(path) == "pytorch_lora_weights.safetensors"
    keys = set(T.lora_state_dict(m))
    assert "transformer.transformer_blocks.0.attn1.to_q.lora_A.weight" in keys
    assert "transformer.transformer_blocks.1.attn1.to_out.0.lora_B.weight" in keys
    assert len(keys) == 2 * 4 * 2
    m2 = _model(seed=9)
    T.load_lora_weights(m2, str(tmp_path))
    for a, b in zip(m.lora_parameters(), m2.lora_parameters()):
        assert torch.equal(a, b)
    bad = T.StandInTransformer(3, 64, 4, 4, 4.0, CpuAttention(), dtype=torch.float32)
    with pytest.raises(KeyError):
        T.load_lora_weights(bad, path)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    m = _model()
    _perturb_b(m)
    red = T.BucketedGradReducer(m.lora_parameters(), bucket_bytes=4096)   # several buckets
    step = T.TrainStep(m, lr=1e-2, accum=2, reducer=red)
    x, y = _batch(8)
    xs, ys = x[4 * rank:4 * rank + 4], y[4 * rank:4 * rank + 4]   # this rank's shard
    step([(xs[:2], ys[:2]), (xs[2:], ys[2:])])
    q.put((rank, [p.detach().numpy().copy() for p in m.lora_parameters()], len(red.buckets)))
    red.close()
    dist.destroy_process_group()


def test_two_rank_bucketed_all_reduce_equals_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (ps, nb)) for r, ps, nb in (q.get(timeout=180) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] > 1
    # single process, whole batch, accumulation 4 x 2 samples = the same global mean
    m = _model()
    _perturb_b(m)
    step = T.TrainStep(m, lr=1e-2, accum=2)
    x, y = _batch(8)
    step([(x[:4], y[:4]), (x[4:], y[4:])])
    for a, b, c in zip(res[0][0], res[1][0], m.lora_parameters()):
        a, b = torch.from_numpy(a), torch.from_numpy(b)
        assert torch.equal(a, b)                       # ranks agree exactly
        assert torch.allclose(a, c.detach(), atol=2e-6, rtol=1e-5)


def test_qk_dump_counter_and_layout_match_the_reference(tmp_path):
    """blocksparseattn.py:375-386: timestep = counter % (8*42) // 42, layer = counter % 42;
    q.pt / k.pt saved at the chosen timesteps under timestep_{t}_layer_{l}/."""
    from vblade import dump
    m = dump.QKDumpAttention(str(tmp_path), CpuAttention(), layers=3, steps=4, timesteps=(1, 3))
    qs = []
    for c in range(3 * 4 + 2):        # wraps into a second "video"
        q = torch.full((1, 2, 8, 4), float(c))
        m(q, q + 0.5, q)
        qs.append(q)
    got = dump.load_dumps(str(tmp_path))
    assert [(t, l) for t, l, _ in got] == [(1, 0), (1, 1), (1, 2), (3, 0), (3, 1), (3, 2)]
    for t, l, d in got:
        c = t * 3 + l
        assert torch.equal(d["q"], qs[c]) and torch.equal(d["k"], qs[c] + 0.5)
    assert m.counter == 14


def _tdm_batches(n_micro, per, L=32, hidden=64, seed=5):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n_micro):
        out.append((torch.randn(per, L, hidden, generator=g), torch.randn(per, L, hidden, generator=g),
                    torch.rand(per, 1, 1, generator=g) + 0.5))
    return out


def _tdm_models(seed=0):
    student = _model(seed=seed)
    _perturb_b(student)
    teacher = _model(seed=seed)            # the base model: LoRA B = 0
    return student, teacher


def test_tdm_step_updates_both_models_and_fake_starts_as_student():
    student, teacher = _tdm_models()
    step = T.TDMTrainStep(student, teacher, lr=1e-2, lr_fake=1e-2, accum=2)
    assert all(torch.equal(a, b) for a, b in zip(step.fake.lora_parameters(), student.lora_parameters()))
    assert step.fake.transformer_blocks[0].inner_attention is not student.transformer_blocks[0].inner_attention
    g0 = [p.detach().clone() for p in student.lora_parameters()]
    f0 = [p.detach().clone() for p in step.fake.lora_parameters()]
    t0 = [p.detach().clone() for p in teacher.parameters()]
    lf, lg = step(_tdm_batches(2, 2))
    assert torch.isfinite(lf) and torch.isfinite(lg)
    assert any(not torch.equal(a, b) for a, b in zip(g0, student.lora_parameters()))
    assert any(not torch.equal(a, b) for a, b in zip(f0, step.fake.lora_parameters()))
    assert all(torch.equal(a, b) for a, b in zip(t0, teacher.parameters()))      # frozen
    assert step.opt_g.defaults["betas"] == (0.0, 0.95) and step.opt_d.defaults["betas"] == (0.0, 0.95)


def test_tdm_default_teacher_is_dense_unpatched_base_with_cfg():
    """The reference's teacher is loaded separately and never patched (train_cogvideo_tdm.py:
    1014-1022; the sparse patch at :997-1000 is the student's) and runs classifier-free guidance
    (:1712, :1487-1498); the fake model is a deep copy of the (patched) student (:1301)."""
    student, base = _tdm_models()
    step = T.TDMTrainStep(student, lr=1e-2, lr_fake=1e-2, accum=1, cfg=3.5)
    blk = step.teacher.transformer_blocks[0]
    assert isinstance(blk.inner_attention, T.DenseAttention)
    assert not isinstance(student.transformer_blocks[0].inner_attention, T.DenseAttention)
    assert type(step.fake.transformer_blocks[0].inner_attention) is type(student.transformer_blocks[0].inner_attention)
    assert all(not p.requires_grad for p in step.teacher.parameters())
    for (n, a), b in zip(step.teacher.named_parameters(), base.parameters()):
        assert torch.equal(a, b), n          # base weights, LoRA B zero: no adapter
    x = torch.randn(2, 32, 64)
    cond = torch.randn(2, 1, 64)
    with torch.no_grad():
        got = step.teacher_predict(x, cond)
        c = step.teacher(x, cond)
        u = step.teacher(x, step.uncond)
    assert torch.allclose(got, u + 3.5 * (c - u))
    assert abs(step.huber_c - 1e-3 / ((64 * 64 * 4) ** 0.5 * (60 * 90 * 16 * 13) ** 0.5)) < 1e-20
    lf, lg = step([_tdm_batches(1, 2)[0] + (cond,)])
    assert torch.isfinite(lf) and torch.isfinite(lg)


def _tdm_dp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    student, teacher = _tdm_models()
    step = T.TDMTrainStep(student, teacher, lr=1e-2, lr_fake=1e-2, accum=2, bucket_bytes=4096)
    full = _tdm_batches(2, 4)
    mine = [tuple(t[2 * rank:2 * rank + 2] for t in mb) for mb in full]   # this rank's half
    step(mine)
    q.put((rank, [p.detach().numpy().copy() for p in student.lora_parameters()],
           [p.detach().numpy().copy() for p in step.fake.lora_parameters()]))
    step.close()
    dist.destroy_process_group()


def test_tdm_two_rank_all_reduce_of_both_models_equals_single_process():
    """Two ranks on half micro-batches end with the student AND the fake model equal to one
    process on the whole micro-batches (each model's own bucketed all-reduce)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tdm_dp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (g, f) for r, g, f in (q.get(timeout=180) for _ in procs)}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    student, teacher = _tdm_models()
    step = T.TDMTrainStep(student, teacher, lr=1e-2, lr_fake=1e-2, accum=2, distributed=False)
    step(_tdm_batches(2, 4))
    for which, mine in ((0, student.lora_parameters()), (1, step.fake.lora_parameters())):
        for a, b, c in zip(res[0][which], res[1][which], mine):
            a, b = torch.from_numpy(a), torch.from_numpy(b)
            assert torch.equal(a, b)
            assert torch.allclose(a, c.detach(), atol=5e-6, rtol=1e-4)
