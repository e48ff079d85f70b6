#!/usr/bin/env python3
"""Training-step benchmark: one TDM-style optimizer step of LoRA stand-in
blocks with CogVideoX-5B's attention geometry (hidden 3072 = 48 x 64, L = 17776) around the
sparse attention under autograd + gradient checkpointing, with the bucketed RCCL gradient
all-reduce across ranks (torchrun: one process per GPU).

    python tools/train_bench.py [--layers 4] [--batch 1] [--accum 1] [--steps 3] [--warmup 1]
    python tools/train_bench.py --gpus N ...   (starts N worker processes itself, one per GPU)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/train_bench.py ...

Prints one JSON line: samples/s over all ranks, ms per optimizer step, and the share of the
step spent in the attention op (HIP events around every forward/backward of inner_attention on
rank 0). Synthetic inputs and random-init frozen weights (no checkpoints offline)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))
sys.path.insert(0, ROOT)


class TimedAttention(torch.nn.Module):
    """inner_attention wrapper recording HIP events around the forward and (through a no-op
    autograd node on each side) around the backward of every call."""

    def __init__(self, inner):
        super().__init__()
        self.inner = inner
        self.events = None

    def forward(self, q, k, v):
        if self.events is None:
            return self.inner(q, k, v)
        ev = self.events
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = self.inner(_Mark.apply(q, ev, "bwd_end"), k, v)
        e1.record()
        ev.append(("fwd", e0, e1))
        return _Mark.apply(out, ev, "bwd_start")


class _Mark(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ev, tag):
        ctx.ev, ctx.tag = ev, tag
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        ctx.ev.append((ctx.tag, e, None))
        return g, None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rank-lora", type=int, default=64)
    ap.add_argument("--variant", default="cog", choices=["cog", "wan"])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tdm", action="store_true",
                    help="the two-model TDM step (student + fake-score model with sparse attention, frozen "
                         "dense teacher with CFG, two AdamW, two reducers; train_cogvideo_tdm.py:1301-1325, "
                         "1640-1737)")
    ap.add_argument("--stub-cpu", action="store_true", help=argparse.SUPPRESS)  # launcher tests
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    import bench
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one fresh process per GPU, as bench.py --gpus N (reference: simple_multiprocess_sampler.py:304-309)
        sys.exit(bench.launch_workers(args.gpus, argv, script=os.path.abspath(__file__)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub_cpu:
        return run_stub(args, world, rank)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)
    import vblade
    from vblade import train as T
    heads, D = (48, 64) if args.variant == "cog" else (12, 128)
    hidden = heads * D
    attn = vblade.AdaptiveBlockSparseAttn(args.variant, log_every=0)
    timed = TimedAttention(attn)
    L = attn.gilbert_rearranger.seq_len
    model = T.StandInTransformer(args.layers, hidden, heads, args.rank_lora, float(args.rank_lora), timed,
                                 gradient_checkpointing=True, device=dev, seed=0)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    if args.tdm:
        # teacher: a dense (unpatched) copy with classifier-free guidance, cfg 3.5 (train_tdm_1.sh)
        step = T.TDMTrainStep(model, lr=1e-4, lr_fake=1e-4, accum=args.accum, distributed=world > 1,
                              cfg=3.5)
        micro = [(torch.randn(args.batch, L, hidden, generator=g, device=dev).bfloat16(),
                  torch.randn(args.batch, L, hidden, generator=g, device=dev).bfloat16(),
                  torch.rand(args.batch, 1, 1, generator=g, device=dev) + 0.5,
                  (torch.randn(args.batch, 1, hidden, generator=g, device=dev) * 0.5).bfloat16())
                 for _ in range(args.accum)]
    else:
        reducer = T.BucketedGradReducer(model.lora_parameters()) if world > 1 else None
        step = T.TrainStep(model, lr=1e-4, accum=args.accum, reducer=reducer)
        micro = [(torch.randn(args.batch, L, hidden, generator=g, device=dev).bfloat16(),
                  torch.randn(args.batch, L, hidden, generator=g, device=dev).bfloat16()) for _ in range(args.accum)]
    torch.manual_seed(1234 + rank)
    for _ in range(args.warmup):
        step(micro)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    if rank == 0:
        timed.events = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step(micro)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = bench.max_over_ranks(elapsed, dev)
    if rank == 0:
        ev = timed.events
        timed.events = None
        fwd_ms = sum(a.elapsed_time(b) for tag, a, b in ev if tag == "fwd")
        # backward of one call: from the gradient reaching its output to leaving its input
        starts = [a for tag, a, _ in ev if tag == "bwd_start"]
        ends = [a for tag, a, _ in ev if tag == "bwd_end"]
        bwd_ms = sum(s.elapsed_time(e) for s, e in zip(starts, ends))
        ms_step = 1000.0 * elapsed / args.steps
        samples = world * args.batch * args.accum * args.steps
        print(json.dumps({
            "metric": ("TDM two-model step (student + fake-score, sparse; dense CFG teacher)" if args.tdm else
                       "TDM-style LoRA training step") + ", stand-in blocks with " +
                      ("CogVideoX-5B" if args.variant == "cog" else "Wan2.1-1.3B") + " attention geometry",
            "value": round(samples / elapsed, 4), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_step, 2),
            "higher_is_better": True, "scaling": "weak", "dtype": "bf16", "data": "synthetic",
            "config": {"layers": args.layers, "micro_batch": args.batch, "accum": args.accum, "seq_len": L,
                       "heads": heads, "head_dim": D, "lora_rank": args.rank_lora,
                       "gradient_checkpointing": True,
                       "parallelism": f"dp{world} (bucketed RCCL all-reduce of LoRA grads)"},
            "attention_fwd_ms_per_step": round(fwd_ms / args.steps, 2),
            "attention_bwd_ms_per_step": round(bwd_ms / args.steps, 2),
            "attention_share": round((fwd_ms + bwd_ms) / args.steps / ms_step, 3),
            "attention_timed": "student model's calls only (fake/teacher copies untimed)" if args.tdm else "all calls",
            "last_loss": [float(x) for x in loss] if isinstance(loss, tuple) else float(loss)}), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def run_stub(args, world, rank):
    """Launcher test path (no GPU): gloo ranks, each step a CPU sleep of 20 ms x (rank + 1) in
    place of the training step; the same barrier + max-over-ranks timing and JSON line."""
    import bench
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    dev = torch.device("cpu")
    ranks = bench._ranks_seen(world, rank, dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.02 * (rank + 1))
    if world > 1:
        dist.barrier()
    elapsed = bench.max_over_ranks(time.perf_counter() - t0, dev)
    if rank == 0:
        samples = world * args.batch * args.accum * args.steps
        print(json.dumps({"metric": "stub", "value": samples / elapsed, "n_gpus": world, "ranks": ranks,
                          "ms_per_step": 1000.0 * elapsed / args.steps}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
