"""TDM training-step integration of the sparse attention.

The reference trains LoRA adapters of CogVideoX-5B with TDM (cogvideox/train/train_cogvideo_tdm.py):
  * LoRA on ``to_q``, ``to_k``, ``to_v``, ``to_out.0`` of every attention (:1085-1119), rank 64,
    alpha 64 in train_tdm_1.sh, ``init_lora_weights=True`` (A random, B zero);
  * the attention's ``inner_attention`` is the adaptive block-sparse module with autograd
    (modify_cogvideo.py:79-91, used with grad in the student/fake forward passes :1666, :1713);
  * gradient checkpointing per transformer block (:1077-1079), bf16 mixed precision;
  * AdamW with betas (0.0, 0.95), grad-norm clip 1.0, gradient accumulation 4 (train_tdm_1.sh);
  * data parallel over 4 GPUs with DeepSpeed ZeRO-2 (config.yaml): one gradient all-reduce per
    optimizer step; LoRA weights saved with ``CogVideoXPipeline.save_lora_weights`` (:1130-1151).

The diffusers transformer and its weights are not available here, so this module carries the
attention geometry of CogVideoX-5B (hidden 3072 = 48 heads x 64) in stand-in blocks
(LayerNorm -> LoRA q/k/v -> inner_attention -> LoRA out + residual). What it integrates is the
part of the step the hot path owns: the sparse attention forward/backward under autograd and
gradient checkpointing, and the data-parallel exchange around it:
  * ``BucketedGradReducer`` — the one collective of the step: LoRA gradients packed into
    ~64 MiB flat buckets and all-reduced asynchronously (RCCL over xGMI) as soon as backward has
    produced every gradient of a bucket, overlapping the rest of backward; averaged at the end;
  * ``lora_state_dict`` / ``save_lora_weights`` / ``load_lora_weights`` — the diffusers LoRA
    checkpoint format (``pytorch_lora_weights.safetensors``, keys
    ``transformer.transformer_blocks.{i}.attn1.{to_q|to_k|to_v|to_out.0}.lora_{A|B}.weight``).
"""
from __future__ import annotations

import math
import os
from typing import Callable, Dict, Iterable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

LORA_TARGETS = ("to_q", "to_k", "to_v", "to_out.0")


class LoRALinear(nn.Module):
    """A frozen linear layer plus a trainable low-rank update scaled by alpha / rank
    (peft LoraConfig(r, lora_alpha, init_lora_weights=True): A kaiming-uniform, B zero)."""

    def __init__(self, in_features: int, out_features: int, rank: int, alpha: float, *,
                 bias: bool = True, dtype=torch.bfloat16, device=None, generator=None):
        super().__init__()
        w = torch.empty(out_features, in_features, dtype=torch.float32)
        nn.init.kaiming_uniform_(w, a=math.sqrt(5), generator=generator)
        self.weight = nn.Parameter(w.to(dtype).to(device), requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(out_features, dtype=dtype, device=device), requires_grad=False)
                     if bias else None)
        a = torch.empty(rank, in_features, dtype=torch.float32)
        nn.init.kaiming_uniform_(a, a=math.sqrt(5), generator=generator)
        self.lora_A = nn.Parameter(a.to(device))
        self.lora_B = nn.Parameter(torch.zeros(out_features, rank, dtype=torch.float32, device=device))
        self.scaling = alpha / rank

    def forward(self, x):
        y = F.linear(x, self.weight, self.bias)
        return y + F.linear(F.linear(x, self.lora_A.to(x.dtype)), self.lora_B.to(x.dtype)) * self.scaling


class StandInAttentionBlock(nn.Module):
    """One transformer block's attention with CogVideoX-5B's geometry: the LoRA targets of the
    reference (to_q, to_k, to_v, to_out.0) around ``inner_attention(q, k, v)`` on [B,H,L,D]."""

    def __init__(self, hidden: int, heads: int, rank: int, alpha: float, inner_attention: nn.Module, *,
                 dtype=torch.bfloat16, device=None, generator=None):
        super().__init__()
        self.heads = heads
        self.norm = nn.LayerNorm(hidden, elementwise_affine=False)
        kw = dict(dtype=dtype, device=device, generator=generator)
        self.to_q = LoRALinear(hidden, hidden, rank, alpha, **kw)
        self.to_k = LoRALinear(hidden, hidden, rank, alpha, **kw)
        self.to_v = LoRALinear(hidden, hidden, rank, alpha, **kw)
        self.to_out = nn.ModuleList([LoRALinear(hidden, hidden, rank, alpha, **kw)])
        self.inner_attention = inner_attention

    def forward(self, x):
        B, L, C = x.shape
        h = self.norm(x)
        D = C // self.heads

        def heads(t):
            return t.view(B, L, self.heads, D).transpose(1, 2)

        q, k, v = heads(self.to_q(h)), heads(self.to_k(h)), heads(self.to_v(h))
        o = self.inner_attention(q, k, v.contiguous())
        o = o.transpose(1, 2).reshape(B, L, C)
        return x + self.to_out[0](o)


class StandInTransformer(nn.Module):
    """``num_layers`` stand-in blocks sharing one ``inner_attention`` module (as
    set_block_sparse_attn_cogvideox installs one instance on every block), with optional
    per-block gradient checkpointing (the reference's enable_gradient_checkpointing)."""

    def __init__(self, num_layers: int, hidden: int, heads: int, rank: int, alpha: float,
                 inner_attention: nn.Module, *, gradient_checkpointing: bool = True,
                 dtype=torch.bfloat16, device=None, seed: int = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed)
        self.transformer_blocks = nn.ModuleList(
            [StandInAttentionBlock(hidden, heads, rank, alpha, inner_attention, dtype=dtype, device=device,
                                   generator=g) for _ in range(num_layers)])
        self.gradient_checkpointing = gradient_checkpointing

    def forward(self, x, cond: Optional[torch.Tensor] = None):
        """``cond``: the stand-in for the prompt embedding (encoder_hidden_states), added to the
        input; the classifier-free-guidance pair runs the model once per embedding."""
        if cond is not None:
            x = x + cond.to(x.dtype)
        for blk in self.transformer_blocks:
            if self.gradient_checkpointing and torch.is_grad_enabled():
                x = checkpoint(blk, x, use_reentrant=False)
            else:
                x = blk(x)
        return x

    def lora_parameters(self) -> List[nn.Parameter]:
        return [p for p in self.parameters() if p.requires_grad]


class DenseAttention(nn.Module):
    """The unpatched attention of a diffusers CogVideoX block: dense
    F.scaled_dot_product_attention over [B,H,L,D] (what the TDM teacher runs: the reference loads
    ``transformer_real`` separately and never patches it, train_cogvideo_tdm.py:1014-1022 vs the
    student-only patch at :997-1000)."""

    def forward(self, q, k, v):
        return F.scaled_dot_product_attention(q, k, v)


def dense_copy(model: StandInTransformer) -> StandInTransformer:
    """A frozen copy of ``model``'s base weights (LoRA B zeroed, i.e. no adapter) with dense
    attention: the TDM teacher (transformer_real, from_pretrained without LoRA, requires_grad
    False)."""
    import copy
    t = copy.deepcopy(model)
    dense = DenseAttention()
    for blk in t.transformer_blocks:
        blk.inner_attention = dense
    with torch.no_grad():
        for n, p in t.named_parameters():
            if n.endswith("lora_B"):
                p.zero_()
            p.requires_grad_(False)
    return t


# the generator loss's pseudo-Huber constant, as the reference overwrites it before the loss
# (train_cogvideo_tdm.py:1723): 1e-3 / (sqrt(64*64*4) * sqrt(60*90*16*13)) ~= 7.4e-9
HUBER_C_REF = 1e-3 / (((64 * 64 * 4) ** 0.5) * (60 * 90 * 16 * 13) ** 0.5)


# ------------------------------------------------------------------------------------------------
# data-parallel gradient exchange
# ------------------------------------------------------------------------------------------------
class BucketedGradReducer:
    """All-reduce (average) of the trainable gradients over a process group in flat buckets.

    Buckets are filled in reverse parameter order (the order backward produces gradients). A
    bucket's all-reduce is launched asynchronously from the post-accumulate-grad hook of its last
    outstanding parameter, so communication overlaps the rest of backward. ``finish()`` waits and
    scatters the averaged buckets back into ``.grad``. With gradient accumulation call
    ``enable(False)`` for the micro-batches that must not communicate."""

    def __init__(self, params: Iterable[nn.Parameter], group=None, bucket_bytes: int = 64 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.enabled = True
        self.buckets: List[List[nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            nbytes = p.numel() * 4
            if cur and size + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self._bucket_of[id(p)] = bi
        self._pending = [0] * len(self.buckets)
        self._flat: List[Optional[torch.Tensor]] = [None] * len(self.buckets)
        self._work: List = [None] * len(self.buckets)
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]
        self._reset()

    def enable(self, flag: bool):
        self.enabled = flag

    def _reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._work = [None] * len(self.buckets)

    def _on_grad(self, p):
        if not self.enabled or self.world == 1:
            return
        bi = self._bucket_of[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch(bi)

    def _launch(self, bi):
        b = self.buckets[bi]
        flat = torch.cat([p.grad.reshape(-1).float() for p in b])
        self._flat[bi] = flat
        self._work[bi] = dist.all_reduce(flat, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket and write the averaged gradients back."""
        if self.world == 1 or not self.enabled:
            self._reset()
            return
        for bi, b in enumerate(self.buckets):
            if self._work[bi] is None:      # a parameter without a gradient this step: zeros
                for p in b:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                self._launch(bi)
            self._work[bi].wait()
            flat = self._flat[bi].div_(self.world)
            off = 0
            for p in b:
                n = p.numel()
                p.grad.copy_(flat[off:off + n].view_as(p.grad))
                off += n
            self._flat[bi] = None
        self._reset()

    def close(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


# ------------------------------------------------------------------------------------------------
# the training step
# ------------------------------------------------------------------------------------------------
def pseudo_huber(pred: torch.Tensor, target: torch.Tensor, c: float, weight=None) -> torch.Tensor:
    """The generator loss of the TDM step (train_cogvideo_tdm.py:1724-1727):
    mean((sqrt((pred - target)^2 + c^2) - c) / weight), in fp32."""
    d = pred.float() - target.float()
    loss = torch.sqrt(d * d + c * c) - c
    if weight is not None:
        loss = loss / weight
    return loss.mean()


class TrainStep:
    """One optimizer step: ``accum`` micro-batches of forward + backward through the stand-in
    transformer (the sparse attention under autograd), the bucketed DP all-reduce on the last
    micro-batch, grad-norm clipping and AdamW (the reference's betas (0, 0.95), clip 1.0)."""

    def __init__(self, model: StandInTransformer, *, lr: float = 1e-4, betas=(0.0, 0.95),
                 weight_decay: float = 1e-4, eps: float = 1e-8, max_grad_norm: float = 1.0,
                 accum: int = 1, reducer: Optional[BucketedGradReducer] = None, huber_c: float = 1e-3):
        self.model = model
        self.params = model.lora_parameters()
        foreach_ok = all(p.is_cuda for p in self.params)
        self.opt = torch.optim.AdamW(self.params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                     foreach=foreach_ok)
        self.max_grad_norm = max_grad_norm
        self.accum = accum
        self.reducer = reducer
        self.huber_c = huber_c

    def __call__(self, micro_batches: List[tuple]) -> float:
        assert len(micro_batches) == self.accum
        total = 0.0
        losses = []
        for i, (x, target) in enumerate(micro_batches):
            if self.reducer is not None:
                self.reducer.enable(i == self.accum - 1)
            loss = pseudo_huber(self.model(x), target, self.huber_c) / self.accum
            loss.backward()
            losses.append(loss.detach())
        if self.reducer is not None:
            self.reducer.finish()
        gnorm = torch.nn.utils.clip_grad_norm_(self.params, self.max_grad_norm)
        self.opt.step()
        self.opt.zero_grad(set_to_none=True)
        total = torch.stack(losses).sum()
        self.last_grad_norm = gnorm
        return total


class TDMTrainStep:
    """The TDM joint step with its two trained models (train_cogvideo_tdm.py:1301-1325, loop
    :1640-1737): a student (the K-step generator) and a fake-score model initialised as a deep copy
    of it (:1301, so it carries the student's sparse attention and LoRA), each with its own AdamW
    (betas (0, 0.95): ``args.adam_beta1 = 0`` at :1310), learning rate, gradient clipping and
    data-parallel gradient exchange (two accelerators, :1318-1325), plus a frozen teacher ("real"
    model) with DENSE attention and no LoRA (loaded separately and never patched, :1014-1022;
    ``dense_copy`` of the student by default). Every micro-batch runs, in the reference's order:

    1. fake-score update (:1640-1688): the student's prediction without grad, the fake model's
       prediction WITH grad (sparse attention under autograd), the weighted regression loss
       ``mean(w * (fake - student)^2)``, backward into the fake model;
    2. generator update (:1690-1737): the student's prediction WITH grad; the teacher with
       classifier-free guidance (predictor.predict(..., cfg=args.cfg) :1712, :1487-1498: one pass
       on the prompt embedding, one on the unconditional embedding, uncond + cfg * (cond -
       uncond); cfg 3.5 in train_tdm_1.sh) and the fake model without grad; the revised target
       ``student + real - fake`` (detached), the pseudo-Huber loss over ``weighting_factor`` with
       the reference's c (:1719-1727), backward into the student.

    On the last micro-batch of an accumulation window each model's reducer exchanges its LoRA
    gradients (one bucketed all-reduce per model), then clip + AdamW per model. The diffusion
    specifics (noise schedules, timesteps, K-step ODE states) are outside the hot path: a
    micro-batch gives the student's input ``x_gen`` (the noisy ODE state), the re-noised input the
    fake and teacher models see ``x_noisy`` (noisy_model_latents), the regression weight ``w``
    (1 / (1 - alphas_cumprod[t])) and optionally the prompt embedding ``cond`` (the stand-in adds
    it to the input; zeros if absent). The unconditional embedding is ``uncond`` (fixed)."""

    def __init__(self, student: StandInTransformer, teacher: Optional[StandInTransformer] = None, *,
                 lr: float = 1e-4, lr_fake: float = 1e-4, betas=(0.0, 0.95), weight_decay: float = 1e-4,
                 eps: float = 1e-8, max_grad_norm: float = 1.0, accum: int = 1, group=None,
                 bucket_bytes: int = 64 << 20, huber_c: float = HUBER_C_REF, cfg: Optional[float] = 3.5,
                 uncond: Optional[torch.Tensor] = None, distributed: Optional[bool] = None):
        import copy
        self.student = student
        self.teacher = teacher if teacher is not None else dense_copy(student)
        self.fake = copy.deepcopy(student)
        for q in self.teacher.parameters():
            q.requires_grad_(False)
        self.cfg = cfg
        self.uncond = uncond
        self.accum = accum
        self.max_grad_norm = max_grad_norm
        self.huber_c = huber_c
        self.g_params = student.lora_parameters()
        self.f_params = self.fake.lora_parameters()

        def adamw(params, lr_):
            return torch.optim.AdamW(params, lr=lr_, betas=betas, eps=eps, weight_decay=weight_decay,
                                     foreach=all(q.is_cuda for q in params))

        self.opt_g = adamw(self.g_params, lr)
        self.opt_d = adamw(self.f_params, lr_fake)
        if distributed is None:
            distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.red_g = BucketedGradReducer(self.g_params, group, bucket_bytes) if distributed else None
        self.red_d = BucketedGradReducer(self.f_params, group, bucket_bytes) if distributed else None

    def _step(self, params, opt, red):
        if red is not None:
            red.finish()
        gnorm = torch.nn.utils.clip_grad_norm_(params, self.max_grad_norm)
        opt.step()
        opt.zero_grad(set_to_none=True)
        return gnorm

    def _uncond_like(self, x):
        if self.uncond is None:
            g = torch.Generator().manual_seed(1234)
            self.uncond = torch.randn(1, 1, x.shape[-1], generator=g) * 0.5
        if self.uncond.device != x.device or self.uncond.dtype != x.dtype:
            # moved once: a pageable host copy per teacher call would sync the timed step
            self.uncond = self.uncond.to(device=x.device, dtype=x.dtype)
        return self.uncond

    def teacher_predict(self, x_noisy, cond):
        """predictor.predict(transformer_real, ..., cfg=args.cfg) (:1712, :1475-1498): with cfg,
        uncond + cfg * (cond - uncond) of the conditional and unconditional passes."""
        real = self.teacher(x_noisy, cond)
        if self.cfg is None:
            return real
        real_u = self.teacher(x_noisy, self._uncond_like(x_noisy))
        return real_u + self.cfg * (real - real_u)

    def __call__(self, micro_batches: List[tuple]):
        """micro_batches: ``accum`` tuples (x_gen, x_noisy, w[, cond]). Returns (loss_fake, loss_gen)."""
        assert len(micro_batches) == self.accum
        lf, lg = [], []
        for i, mb in enumerate(micro_batches):
            x_gen, x_noisy, w = mb[:3]
            cond = mb[3] if len(mb) > 3 else None
            last = i == self.accum - 1
            # 1. fake-score update
            if self.red_d is not None:
                self.red_d.enable(last)
            with torch.no_grad():
                target = self.student(x_gen, cond)
            fake = self.fake(x_noisy, cond)
            loss_f = (w * (fake.float() - target.float()) ** 2).mean() / self.accum
            loss_f.backward()
            lf.append(loss_f.detach())
            if last:
                self.last_grad_norm_fake = self._step(self.f_params, self.opt_d, self.red_d)
            # 2. generator update
            if self.red_g is not None:
                self.red_g.enable(last)
            pred = self.student(x_gen, cond)
            with torch.no_grad():
                real = self.teacher_predict(x_noisy, cond)
                fake_g = self.fake(x_noisy, cond)
                revised = (pred.detach() + real - fake_g).float()
                weighting = (pred.detach().float() - real.float()).abs().mean(
                    dim=tuple(range(1, pred.dim())), keepdim=True).clamp(max=5.0)
            loss_g = pseudo_huber(pred, revised, self.huber_c, weighting) / self.accum
            loss_g.backward()
            lg.append(loss_g.detach())
            if last:
                self.last_grad_norm = self._step(self.g_params, self.opt_g, self.red_g)
        return torch.stack(lf).sum(), torch.stack(lg).sum()

    def close(self):
        for r in (self.red_g, self.red_d):
            if r is not None:
                r.close()


# ------------------------------------------------------------------------------------------------
# LoRA checkpoint (diffusers save_lora_weights format)
# ------------------------------------------------------------------------------------------------
WEIGHT_NAME = "pytorch_lora_weights.safetensors"


def lora_state_dict(model: StandInTransformer) -> Dict[str, torch.Tensor]:
    """get_peft_model_state_dict + the ``transformer.`` prefix save_lora_weights adds:
    ``transformer.transformer_blocks.{i}.attn1.{target}.lora_{A|B}.weight``."""
    out = {}
    for i, blk in enumerate(model.transformer_blocks):
        for name in LORA_TARGETS:
            mod = blk.to_out[0] if name == "to_out.0" else getattr(blk, name)
            pre = f"transformer.transformer_blocks.{i}.attn1.{name}"
            out[f"{pre}.lora_A.weight"] = mod.lora_A.detach()
            out[f"{pre}.lora_B.weight"] = mod.lora_B.detach()
    return out


def save_lora_weights(output_dir: str, model: StandInTransformer, dtype=None):
    from safetensors.torch import save_file
    os.makedirs(output_dir, exist_ok=True)
    sd = {k: (v.to(dtype) if dtype is not None else v).contiguous().cpu() for k, v in lora_state_dict(model).items()}
    path = os.path.join(output_dir, WEIGHT_NAME)
    save_file(sd, path, metadata={"format": "pt"})
    return path


def load_lora_weights(model: StandInTransformer, path: str):
    """Load a LoRA checkpoint written by save_lora_weights (keys must match exactly)."""
    from safetensors.torch import load_file
    if os.path.isdir(path):
        path = os.path.join(path, WEIGHT_NAME)
    sd = load_file(path)
    expect = lora_state_dict(model)
    missing = set(expect) - set(sd)
    unexpected = set(sd) - set(expect)
    if missing or unexpected:
        raise KeyError(f"LoRA checkpoint mismatch: missing {sorted(missing)[:4]}, unexpected {sorted(unexpected)[:4]}")
    with torch.no_grad():
        for k, v in expect.items():
            v.copy_(sd[k].to(v.dtype))
    return model
