#!/usr/bin/env python3
"""Benchmark of the Video-BLADE hot path on MI355X: adaptive block-sparse attention.

Metric (BASELINE.json): frames/sec/GPU for CogVideoX-5B 8-step 49x720x480 bf16 (+ attention
TFLOPS vs dense). One bench STEP = the attention work of one 8-step video = 8 denoising steps x
42 transformer blocks = 336 calls of ``inner_attention(q, k, v)`` on q,k,v [1,48,17776,64] bf16
(Wan2.1-1.3B with --variant wan: 8 x 30 calls on [1,12,32760,128], 81 frames). Each call runs the
whole hot path: Gilbert-order mask prediction, pooled K/V, fused block-sparse + pooled attention,
scatter back to token order. Inputs are synthetic (no weights/datasets offline): N_SETS distinct
random q/k/v sets with the block-structured "realistic" distribution, resident in
HBM before the timed region, cycled across calls.

Attention-only frames/s = frames / (time of 8 x layers calls). The transformer's GEMMs, VAE and
scheduler are not in the hot path and are not timed.

N GPUs: one process per GPU, each rank renders its own videos (prompt-batch replicas, no
data-path collective). ``--gpus N`` without a launcher's WORLD_SIZE spawns the N
worker processes itself (one per GPU, as the reference's simple_multiprocess_sampler.py:304-309
does); under torchrun the launcher's ranks are used. An RCCL barrier + synchronize brackets the
timed region, the job time is the max over ranks, and ``value`` = frames rendered by ALL ranks /
that time (whole-job aggregate, "scaling": "weak"); ``per_gpu_frames_per_s`` = value / N.

Rank 0 at N=1 adds (``--no-extras`` skips the sweep and the backward):
  roofline        attn_fwd_kernel: algorithmic FLOPs / HIP-event launch time (every 8th launch of
                  the timed region, --event-every; its FLOPs replayed for exactly those launches),
                  PMC traffic
  quality         PSNR, max|err| and bf16 ULP histograms of head 0 of the timed config vs the
                  oracle (same mask): vs the reference's rounding and vs the exact fp64 combine
  points          Wan at the energy rule, the multi-level sampler op (cog-ml), CogVideoX at fixed
                  densities 0.05/0.3/0.5/0.7, each vs dense SDPA; Wan and 0.05 with PMC traffic
                  (counter HBM-side GB/s vs 8 TB/s)
  backward        the training path's vb_attn_bwd at the reference operating point
  cpu_baseline    the reference's CPU SDPA path on BASELINE config 1 (oracle/ref_cpu_path.py)
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import math
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "video-blade_amd"))

VARIANTS = {
    "cog": dict(H=48, D=64, layers=42, frames=49, name="CogVideoX-5B 8-step 49x720x480 bf16",
                video="13x30x45 latent tokens + 226 text"),
    "wan": dict(H=12, D=128, layers=30, frames=81, name="Wan2.1-1.3B 8-step 81x832x480 bf16",
                video="21x30x52 latent tokens"),
    # the VBench sampler's op (cogvideox/sample_evaluate/modify_cogvideo.py:9): multi-level mask
    "cog-ml": dict(H=48, D=64, layers=42, frames=49,
                   name="CogVideoX-5B 8-step 49x720x480 bf16, multi-level sampler path",
                   video="13x30x45 latent tokens + 226 text"),
}
DENOISE_STEPS = 8
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--variant", choices=list(VARIANTS), default="cog")
    ap.add_argument("--density", type=float, default=None,
                    help="fixed block density (min=max retain) instead of the energy rule")
    ap.add_argument("--sets", type=int, default=3, help="distinct resident q/k/v sets")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-dense", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the density/Wan points, the backward and the quality check")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 FETCH_SIZE/WRITE_SIZE passes (roofline.traffic = null)")
    ap.add_argument("--event-every", type=int, default=8,
                    help="time every N-th attention launch of the timed region with HIP events")
    ap.add_argument("--stub-cpu", action="store_true", help=argparse.SUPPRESS)  # launcher tests
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_workers(n: int, argv: list[str], script: str | None = None) -> int:
    """Start ``n`` fresh worker processes of ``script`` (default: this file), one per GPU, before
    anything touches a GPU (the parent never does). Each gets RANK/LOCAL_RANK/WORLD_SIZE and a
    127.0.0.1 rendezvous. Rank 0 prints the JSON line. If a worker fails, the others are stopped
    so none waits at a barrier. Returns the first non-zero exit code (0 if all succeeded)."""
    port = _free_port()
    procs = []
    script = os.path.abspath(script or __file__)
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + argv, env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for other in live:
                    other.terminate()
        time.sleep(0.05)
    return rc if rc >= 0 else 1


# ---------------------------------------------------------------------------------- workload
def realistic_qkv(H, L, D, seed, device):
    g = torch.Generator(device=device).manual_seed(seed)
    cent = torch.randn(1, H, L // 128 + 1, D, generator=g, device=device)
    cent = cent.repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(1, H, L, D, generator=g, device=device) + 2 * cent).bfloat16()
    k = (torch.randn(1, H, L, D, generator=g, device=device) + 2 * cent).bfloat16()
    v = torch.randn(1, H, L, D, generator=g, device=device).bfloat16()
    return q, k, v


# latent token grids (width, height, frames) and text tokens of the two workloads (caller order:
# text first, then the video tokens frame-major, row-major: cogvideo_blocksparseattn.py:141-154)
LATENT_GRID = {"cog": (45, 30, 13, 226), "cog-ml": (45, 30, 13, 226), "wan": (52, 30, 21, 0)}


def local_qkv(variant, H, D, seed, device, waves=8, amp=2.0):
    """Locality-faithful synthetic inputs: q, k = N(0,1) + amp * c(x, y, t) with
    the centre c a smooth function of the token's latent coordinate — a sum of `waves` random
    low-frequency plane waves (0-2 periods across each axis) with random D-vectors per head — so
    tokens near each other in the video, and therefore the Gilbert-ordered 128-token blocks, share
    centres as real video attention does. Text tokens get independent random centres."""
    W, Hh, T, text = LATENT_GRID[variant]
    g = torch.Generator(device=device).manual_seed(seed)
    t, y, x = torch.meshgrid(torch.arange(T, device=device), torch.arange(Hh, device=device),
                             torch.arange(W, device=device), indexing="ij")
    pos = torch.stack([x.flatten() / W, y.flatten() / Hh, t.flatten() / T], 1).float()   # [Lv, 3]
    freq = torch.randint(0, 3, (waves, 3), generator=g, device=device).float()
    phase = torch.rand(waves, generator=g, device=device) * 2 * math.pi
    basis = torch.cos(2 * math.pi * pos @ freq.T + phase)                               # [Lv, waves]
    a = torch.randn(1, H, waves, D, generator=g, device=device) / math.sqrt(waves / 2)
    cent = basis @ a                                                                    # [1, H, Lv, D]
    if text:
        cent = torch.cat([torch.randn(1, H, text, D, generator=g, device=device), cent], 2)
    L = cent.shape[2]
    q = (torch.randn(1, H, L, D, generator=g, device=device) + amp * cent).bfloat16()
    k = (torch.randn(1, H, L, D, generator=g, device=device) + amp * cent).bfloat16()
    v = torch.randn(1, H, L, D, generator=g, device=device).bfloat16()
    return q, k, v


def ml_attn_flops(mask: torch.Tensor, L: int, D: int) -> float:
    """Algorithmic FLOPs of one multi-level launch: sum over (i,j) with level p in {1,2,4,8} of
    4*m_i*(128/p)*D (m_i the true query-block size; key blocks are full pyramid blocks, as the
    reference computes them)."""
    nb = mask.shape[-1]
    rows = torch.full((nb,), 128.0, device=mask.device)
    rows[-1] = L - 128 * (nb - 1)
    m = mask.to(torch.int32)
    keys = torch.zeros_like(m, dtype=torch.float32)
    for p in (1, 2, 4, 8):
        keys += (m == p).float() * (128.0 / p)
    return 4.0 * D * (rows[:, None] * keys).sum().item()


def attn_flops(mask: torch.Tensor, L: int, D: int, Lkp: int) -> float:
    """Algorithmic FLOPs of one fused attention launch: sum over kept (i,j) blocks of
    4*m_i*n_j*D (true block sizes, tail included) + pooled branch 4*L*Lkp*D, per head."""
    nb = mask.shape[-1]
    sizes = torch.full((nb,), 128.0, device=mask.device)
    sizes[-1] = L - 128 * (nb - 1)
    m = mask.float()
    pairs = (sizes[:, None] * sizes[None, :] * m).sum().item()
    heads = mask.shape[0] * mask.shape[1]
    return 4.0 * D * pairs + 4.0 * heads * L * Lkp * D


def attn_alg_bytes(H, L, D, Lkp) -> int:
    """Compulsory bytes of one fused launch: Q read + O written once, every K/V row
    read at least once (the kept blocks cover every key block), pooled K/V, the mask."""
    return H * (4 * L * D * 2) + H * 2 * Lkp * D * 2 + H * ((L + 127) // 128) ** 2


def max_over_ranks(elapsed: float, dev) -> float:
    """The job's time = the slowest rank's (weak scaling: every rank renders its own videos).
    Works on any initialised process group (RCCL on the GPU box, gloo in the CPU tests)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed
    if dist.get_backend() != "nccl":
        dev = torch.device("cpu")
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def whole_job_frames_per_s(world: int, frames: int, steps: int, elapsed: float) -> float:
    """value = frames rendered by ALL ranks / the job's time."""
    return world * frames * steps / elapsed


def _ranks_seen(world: int, rank: int, dev) -> list[int]:
    """Every rank reports its RANK through the process group (the launcher check)."""
    import torch.distributed as dist
    if world == 1:
        return [rank]
    t = torch.zeros(world, dtype=torch.int64, device=dev)
    t[rank] = rank + 1
    dist.all_reduce(t)
    return [int(x) - 1 for x in t.tolist()]


# ---------------------------------------------------------------------------------- main
def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, argv))
    run(args)


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and "WORLD_SIZE" in os.environ and rank == 0:
        print(f"bench: --gpus {args.gpus} but the launcher started {world} ranks; using {world}",
              file=sys.stderr)
    if args.stub_cpu:
        return run_stub(args, world, rank)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    import vblade

    V = VARIANTS[args.variant]
    H, D, layers, frames = V["H"], V["D"], V["layers"], V["frames"]
    over = {}
    if args.density is not None:
        over = dict(min_retain_ratio=args.density, max_retain_ratio=args.density)
    ml = args.variant == "cog-ml"
    if ml:
        from vblade import multilevel
        mod = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0)
    else:
        mod = vblade.AdaptiveBlockSparseAttn(args.variant, log_every=0, **over)
    L = mod.gilbert_rearranger.seq_len
    calls = DENOISE_STEPS * layers
    sets = [realistic_qkv(H, L, D, 1000 * rank + s, dev) for s in range(args.sets)]
    torch.manual_seed(1234 + rank)

    def one_video():
        for c in range(calls):
            q, k, v = sets[c % len(sets)]
            mod(q, k, v)

    with torch.no_grad():
        for _ in range(args.warmup):
            one_video()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        # the dominant kernel is timed live: HIP events around every `--event-every`-th attention
        # launch, recorded on the launch stream inside the timed region (rank 0). Each event pair
        # costs the stream ~12 us (two marker packets), so timing every launch would slow the very
        # throughput being measured by ~1 %.
        rng_state = torch.cuda.get_rng_state(dev)
        if rank == 0:
            mod.attn_events = []
            mod.attn_event_every = args.event_every
            mod._attn_launches = 0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            one_video()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
        events, mod.attn_events = mod.attn_events, None
    elapsed = max_over_ranks(elapsed, dev)
    ranks = _ranks_seen(world, rank, dev)
    ms_per_step = 1000.0 * elapsed / args.steps
    ms_per_call = ms_per_step / calls
    value = whole_job_frames_per_s(world, frames, args.steps, elapsed)
    sparsity = mod.sparsity_acc / mod.sparsity_counter if ml else mod.sparsity

    result = {
        # `value` is the whole-job aggregate over all ranks (the driver's contract); BASELINE's
        # per-GPU figure is per_gpu_frames_per_s = value / n_gpus (equal at N=1)
        "metric": "frames/sec (aggregate over n_gpus; per GPU = value/n_gpus), " + V["name"]
                  + " (attention path); attn TFLOPS vs dense",
        "value": round(value, 4),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic block-structured q/k/v (SURVEY §8d realistic option), "
                f"{args.sets} resident sets",
        "config": {
            "workload": f"{V['name']}: {calls} inner_attention calls per video "
                        f"(8 steps x {layers} blocks), q/k/v [1,{H},{L},{D}] ({V['video']})",
            "global_batch": world,
            "seq_len": L,
            "heads": H,
            "head_dim": D,
            "calls_per_step": calls,
            "mask": ("rank-band level mask, levels 1/2/4/8 (reference mask_ratios)" if ml
                     else "energy rule (reference defaults)" if args.density is None
                     else f"fixed density {args.density}"),
            "parallelism": f"replicas x{world} (prompt-batch DP, no collective)",
        },
        "value_is": "whole-job aggregate: frames rendered by all ranks / max-over-ranks time",
        "per_gpu_frames_per_s": round(value / world, 4),
        "aggregate_frames_per_s": round(value, 4),
        "ranks": ranks,
        "ms_per_call": round(ms_per_call, 4),
        "mean_sparsity": round(sparsity, 4),
    }

    if rank == 0:
        with torch.no_grad():
            extra = measure_kernels(mod, sets, L, H, D, dev, args, events, rng_state, calls)
        result.update(extra["top"])
        dense_ms = extra.get("dense_ms")
        if dense_ms:
            result["dense_sdpa_ms_per_call"] = round(dense_ms, 4)
            result["speedup_vs_dense_sdpa"] = round(dense_ms / ms_per_call, 3)
            dense_flops = 4.0 * H * L * L * D
            result["attn_tflops_dense_equiv"] = round(dense_flops / (ms_per_call * 1e-3) / 1e12, 2)
        if not args.no_pmc and world == 1:
            traffic = pmc_traffic(args.variant)
            if traffic is not None:
                result["roofline"]["traffic"] = traffic["bytes"]
                result["roofline"]["traffic_detail"] = traffic
        result["roofline"]["algorithmic_bytes"] = extra["alg_bytes"]
        if world == 1 and not args.no_extras and not ml:
            result["quality"] = quality_vs_oracle(mod, sets[0], args.variant)
        if world == 1 and not args.no_extras and args.variant == "cog" and args.density is None:
            dense_cache = {"cog": dense_ms}
            result["points"] = [measure_point(v, d, dev, dense_cache)
                                for v, d in (("wan", None), ("cog-ml", None), ("cog", 0.05),
                                             ("cog", 0.3), ("cog", 0.5), ("cog", 0.7))]
            # the energy rule on locality-faithful inputs (neighbouring Gilbert blocks share
            # centres, as video does): mask density and counter traffic of both workloads
            result["points"] += [measure_point(v, None, dev, dense_cache, inputs="local")
                                 for v in ("cog", "wan")]
            if not args.no_pmc:
                # counter-measured HBM-side traffic of the attention kernel at the Wan point and at
                # the high-sparsity point (density 0.05), as GB/s against the 8 TB/s peak
                for pt in result["points"]:
                    local = pt["inputs"].startswith("locality")
                    if (pt["variant"], pt["mask"]) in (("wan", "energy rule"), ("cog", "density 0.05")) or local:
                        d = None if pt["mask"] == "energy rule" else 0.05
                        tr = pmc_traffic(pt["variant"], density=d, local=local)
                        if tr is not None:
                            gbs = tr["bytes"] / (pt["attn_fwd_ms"] * 1e-3) / 1e9
                            pt["traffic"] = tr["bytes"]
                            pt["traffic_over_algorithmic"] = round(tr["bytes"] / pt["algorithmic_bytes"], 3)
                            pt["hbm_gbs_counters"] = round(gbs, 1)
                            pt["hbm_frac_counters"] = round(gbs / PEAK_HBM_GBS, 4)
                            pt["traffic_detail"] = tr
            # the training path's backward of both TDM-trained variants (CogVideoX first: the
            # headline's model; Wan's sibling TDM script trains the D=128 geometry)
            result["backward"] = [measure_backward("cog", dev), measure_backward("wan", dev),
                                  measure_backward("cog-ml", dev)]
            result["end_to_end"] = measure_end_to_end(dev, ms_per_call, calls, frames)
        if world == 1 and not args.no_cpu_baseline:
            base = "cog" if args.variant == "cog-ml" else args.variant
            result["cpu_baseline"] = cpu_baseline_sdpa(base)
            result["cpu_oracle_port"] = (cpu_baseline_ml(calls, frames) if ml
                                         else cpu_baseline(args.variant, calls, frames))
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


def run_stub(args, world, rank):
    """The launcher and timing contract with the GPU work replaced by a rank-dependent CPU sleep
    (gloo): used by tests/test_multi_rank.py to check N workers, distinct ranks and the
    max-over-ranks time without a GPU."""
    import torch.distributed as dist
    dev = torch.device("cpu")
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.02 * (rank + 1))
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    ranks = _ranks_seen(world, rank, dev)
    value = whole_job_frames_per_s(world, 49, args.steps, elapsed)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": value, "n_gpus": world, "ranks": ranks,
                          "ms_per_step": 1000.0 * elapsed / args.steps,
                          "per_gpu_frames_per_s": value / world}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------- measurement
def dense_sdpa_ms(q, k, v, reps=5):
    """Dense bf16 SDPA (PyTorch-ROCm) on the same shapes: ms per call, HIP events."""
    stream = torch.cuda.current_stream(q.device)
    for _ in range(2):
        torch.nn.functional.scaled_dot_product_attention(q, k, v)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(reps):
        torch.nn.functional.scaled_dot_product_attention(q, k, v)
    b.record(stream)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def measure_kernels(mod, sets, L, H, D, dev, args, events, rng_state, calls):
    """Roofline of the dominant kernel (attn_fwd_kernel): its average launch duration from the
    HIP events recorded around every launch of the timed region, and its algorithmic FLOPs
    recomputed exactly per launch by replaying the timed region's mask predictions (same RNG
    state, same inputs -> the same sampled offsets and masks; no attention run). Plus dense
    SDPA on the same shapes for the speedup ratio."""
    ms = sum(a.elapsed_time(b) for a, b in events) / len(events)
    torch.cuda.set_rng_state(rng_state, dev)
    flops = 0.0
    ml = not hasattr(mod, "sample_gap")
    Lkp = 0 if ml else (L + mod.sample_gap - 1) // mod.sample_gap
    n = 0       # sampled (event-timed) launches: their FLOPs, replayed in order
    idx = 0
    for _ in range(args.steps):
        for c in range(calls):
            q, k, _ = sets[c % len(sets)]
            if ml:
                from vblade import multilevel
                _, mask = multilevel.predict_level_mask(q, k, rows=mod._rows(q.device),
                                                        mask_ratios=mod.mask_ratios)
                f = ml_attn_flops(mask, L, D)
            else:
                _, mask = mod.predict_mask(q, k)
                f = attn_flops(mask, L, D, Lkp)
            if idx % args.event_every == 0:
                flops += f
                n += 1
            idx += 1
    assert n == len(events)
    flops /= n
    achieved = flops / (ms * 1e-3) / 1e12
    top = {
        "roofline": {
            "bound": "mfma",
            "kernel": "attn_fwd_kernel",
            "achieved": round(achieved, 2),
            "peak": PEAK_BF16_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
            "traffic": None,
            "avg_launch_ms": round(ms, 4),
            "launches_timed": n,
            "launches_timed_every": args.event_every,
            "flops_per_launch": flops,
        }
    }
    alg_bytes = attn_alg_bytes(H, L, D, Lkp)
    if ml:   # Q read + O written once, both KV pyramids (15/8 of the padded rows) read once, mask
        R = 15 * ((L + 127) // 128 * 128) // 8
        alg_bytes = H * (2 * L * D * 2) + H * 2 * R * D * 2 + H * ((L + 127) // 128) ** 2
    out = {"top": top, "alg_bytes": alg_bytes}
    if not args.no_dense:
        q, k, v = sets[0]
        out["dense_ms"] = dense_sdpa_ms(q, k, v)
    return out


def measure_point(variant, density, dev, dense_cache, calls=None, seed=500, every=4, inputs="blocks"):
    """One more operating point, measured in-process on fresh resident inputs: one denoising
    step's calls (layers) of the whole module, timed with events, the attention launches timed
    individually, and their FLOPs replayed from the same RNG state (as the main line)."""
    import vblade
    V = VARIANTS[variant]
    H, D, layers, frames = V["H"], V["D"], V["layers"], V["frames"]
    calls = calls or layers
    ml = variant == "cog-ml"
    if ml:   # the VBench sampler's multi-level op (cogvideox/sample_evaluate/modify_cogvideo.py:9)
        from vblade import multilevel
        mod = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0)
    else:
        over = {} if density is None else dict(min_retain_ratio=density, max_retain_ratio=density)
        mod = vblade.AdaptiveBlockSparseAttn(variant, log_every=0, **over)
    L = mod.gilbert_rearranger.seq_len
    Lkp = 0 if ml else (L + mod.sample_gap - 1) // mod.sample_gap
    sets = [realistic_qkv(H, L, D, seed + s, dev) if inputs == "blocks" else local_qkv(variant, H, D, seed + s, dev)
            for s in range(2)]
    with torch.no_grad():
        for c in range(4):
            mod(*sets[c % 2])
        torch.cuda.synchronize()
        rng = torch.cuda.get_rng_state(dev)
        mod.attn_events = []
        mod.attn_event_every = every
        mod._attn_launches = 0
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for c in range(calls):
            mod(*sets[c % 2])
        b.record()
        torch.cuda.synchronize()
        ms_call = a.elapsed_time(b) / calls
        ev, mod.attn_events = mod.attn_events, None
        attn_ms = sum(x.elapsed_time(y) for x, y in ev) / len(ev)
        torch.cuda.set_rng_state(rng, dev)
        flops = 0.0
        for c in range(calls):
            q, k, _ = sets[c % 2]
            if ml:
                _, mask = multilevel.predict_level_mask(q, k, rows=mod._rows(q.device),
                                                        mask_ratios=mod.mask_ratios)
                f = ml_attn_flops(mask, L, D)
            else:
                _, mask = mod.predict_mask(q, k)
                f = attn_flops(mask, L, D, Lkp)
            if c % every == 0:   # the event-timed launches
                flops += f
        flops /= len(ev)
        dkey = "cog" if ml else variant
        if dkey not in dense_cache or dense_cache[dkey] is None:
            dense_cache[dkey] = dense_sdpa_ms(*sets[0])
        dense_ms = dense_cache[dkey]
    tfs = flops / (attn_ms * 1e-3) / 1e12
    if ml:   # Q read + O written once, both KV pyramids (15/8 of the padded rows) read once, mask
        R = 15 * ((L + 127) // 128 * 128) // 8
        alg = H * (2 * L * D * 2) + H * 2 * R * D * 2 + H * ((L + 127) // 128) ** 2
    else:
        alg = attn_alg_bytes(H, L, D, Lkp)
    sparsity = mod.sparsity_acc / mod.sparsity_counter if ml else mod.sparsity
    res = {
        "variant": variant,
        "inputs": ("block-structured (centres per caller-order 128-token run)" if inputs == "blocks"
                   else "locality-faithful (centres a smooth function of the latent x,y,t)"),
        "mask": ("rank-band level mask (reference mask_ratios)" if ml
                 else "energy rule" if density is None else f"density {density}"),
        "mask_density": round(float(mod.last_mask.float().mean().item()), 4) if not ml else None,
        "mean_sparsity": round(sparsity, 4),
        "frames_per_s": round(frames / (ms_call * 1e-3 * DENOISE_STEPS * layers), 3),
        "ms_per_call": round(ms_call, 4),
        "dense_sdpa_ms_per_call": round(dense_ms, 4),
        "speedup_vs_dense_sdpa": round(dense_ms / ms_call, 3),
        "attn_fwd_ms": round(attn_ms, 4),
        "attn_fwd_tflops": round(tfs, 2),
        "mfma_frac": round(tfs / PEAK_BF16_TFLOPS, 4),
        "algorithmic_bytes": alg,
        "hbm_gbs_algorithmic": round(alg / (attn_ms * 1e-3) / 1e9, 1),
        "hbm_frac": round(alg / (attn_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4),
    }
    del sets
    torch.cuda.empty_cache()
    return res


def measure_backward(variant, dev, reps=6):
    """The training path's backward (vb_attn_bwd: both branches, alpha detached, pooled grads
    through the mean pool) at the reference operating point, timed with HIP events around each
    launch; algorithmic FLOPs = 2.5 x the forward's (5 GEMMs per kept block pair against 2)."""
    import vblade
    from vblade import multilevel, ops
    V = VARIANTS[variant]
    H, D = V["H"], V["D"]
    ml = variant == "cog-ml"
    if ml:   # the VBench sampler's multi-level op (vb_ml_attn_bwd), cogvideo_newattn.py:210-234
        mod = multilevel.AdaptiveBlockSparseAttnTrain(log_every=0)
    else:
        mod = vblade.AdaptiveBlockSparseAttn(variant, log_every=0)
    L = mod.gilbert_rearranger.seq_len
    Lkp = 0 if ml else (L + mod.sample_gap - 1) // mod.sample_gap
    q, k, v = (t.requires_grad_() for t in realistic_qkv(H, L, D, 700, dev))
    dout = torch.randn(1, H, L, D, device=dev, dtype=torch.bfloat16)
    events = []
    name = "ml_attention_bwd" if ml else "attention_bwd"
    orig = getattr(ops, name)

    def timed(*a, **kw):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = orig(*a, **kw)
        e1.record()
        events.append((e0, e1))
        return r

    setattr(ops, name, timed)
    flops = 0.0
    try:
        for i in range(reps + 2):
            out = mod(q, k, v)
            if i >= 2:
                flops += ml_attn_flops(mod.last_mask, L, D) if ml else attn_flops(mod.last_mask, L, D, Lkp)
            out.backward(dout)
            q.grad = k.grad = v.grad = None
        torch.cuda.synchronize()
    finally:
        setattr(ops, name, orig)
    ms = sum(a.elapsed_time(b) for a, b in events[2:]) / reps
    bflops = 2.5 * flops / reps
    tfs = bflops / (ms * 1e-3) / 1e12
    return {"variant": variant,
            "kernel": ("vb_ml_attn_bwd (prep + pooled-level dK/dV + level-1 dK/dV + dQ)" if ml
                       else "vb_attn_bwd (bwd_prep + bwd_dkdv + bwd_dq)"),
            "mask": ("multi-level rank bands (reference mask_ratios)" if ml
                     else "energy rule (reference defaults)"), "avg_ms": round(ms, 4),
            "flops_per_call": bflops, "achieved": round(tfs, 2), "unit": "TFLOP/s",
            "peak": PEAK_BF16_TFLOPS, "frac": round(tfs / PEAK_BF16_TFLOPS, 4),
            "launches_timed": reps,
            # the deterministic design (no atomics) recomputes S and dP in the dQ kernel: 7 GEMMs
            # of the forward's size per kept block pair are executed against the 5 counted above
            "executed_gemm_frac": round(tfs * 7 / 5 / PEAK_BF16_TFLOPS, 4)}


class _StandInCogVideoXBlock(torch.nn.Module):
    """One CogVideoX-5B transformer block's compute at its real dimensions with random weights
    (diffusers' CogVideoXBlock: norm1 -> to_q/to_k/to_v -> per-head LayerNorm on q and k ->
    inner_attention -> to_out, gated residual; norm2 -> FFN 3072 -> 12288 -> 3072, GELU(tanh), gated
    residual). The adaLN modulation is a per-block constant here (its time-embedding MLP is
    O(hidden^2) per step, not per token) and RoPE is omitted (elementwise on q/k). Stand-in for
    timing only: no weights are available offline, so nothing about its outputs is claimed."""

    def __init__(self, hidden, heads, ffn, inner_attention, dev, gen):
        super().__init__()
        kw = dict(device=dev, dtype=torch.bfloat16)

        def w(o, i):
            return (torch.randn(o, i, device=dev, generator=gen) * (i ** -0.5)).to(torch.bfloat16)
        self.heads = heads
        self.qkv = w(3 * hidden, hidden)
        self.qkv_b = torch.zeros(3 * hidden, **kw)
        self.out = w(hidden, hidden)
        self.ff1, self.ff2 = w(ffn, hidden), w(hidden, ffn)
        self.mod = (torch.randn(6, hidden, device=dev, generator=gen) * 0.1).to(torch.bfloat16)
        self.inner_attention = inner_attention

    def forward(self, x):
        import torch.nn.functional as F
        B, L, C = x.shape
        sh1, sc1, g1, sh2, sc2, g2 = self.mod
        h = F.layer_norm(x, (C,)) * (1 + sc1) + sh1
        qkv = F.linear(h, self.qkv, self.qkv_b).view(B, L, 3, self.heads, C // self.heads)
        q, k, v = (F.layer_norm(qkv[:, :, i], (C // self.heads,)).transpose(1, 2) if i < 2
                   else qkv[:, :, i].transpose(1, 2) for i in range(3))
        o = self.inner_attention(q, k, v).transpose(1, 2).reshape(B, L, C)
        x = x + g1 * F.linear(o, self.out)
        h = F.layer_norm(x, (C,)) * (1 + sc2) + sh2
        return x + g2 * F.linear(F.gelu(F.linear(h, self.ff1), approximate="tanh"), self.ff2)


def measure_end_to_end(dev, attn_ms_per_call, calls, frames, steps=8):
    """SURVEY §8(d) end-to-end stand-in: one CogVideoX-5B 8-step video through 42 stand-in blocks at
    the model's dimensions (hidden 3072 = 48 heads x 64, FFN 4x, 226 text + 17550 video tokens,
    batch 1: guidance_scale 1 as at cogvideox/train/inference.py:85-90), bf16 GEMMs through
    PyTorch-ROCm (hipBLASLt), the HIP sparse attention inside every block. The scheduler step and
    the VAE are out of scope (parity unpinned: diffusers and the weights are absent)."""
    import vblade
    V = VARIANTS["cog"]
    H, layers = V["H"], V["layers"]
    hidden = H * V["D"]
    attn = vblade.AdaptiveBlockSparseAttn("cog", log_every=0)
    L = attn.gilbert_rearranger.seq_len
    gen = torch.Generator(device=dev).manual_seed(77)
    blocks = [_StandInCogVideoXBlock(hidden, H, 4 * hidden, attn, dev, gen) for _ in range(layers)]
    x0 = torch.randn(1, L, hidden, device=dev, dtype=torch.bfloat16, generator=gen)

    def video():
        x = x0
        for _ in range(steps):
            for blk in blocks:
                x = blk(x)
        return x

    def timed():
        video()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        video()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    with torch.no_grad():
        sec = timed()
        # the same video with the attention replaced by `v` (no attention at all): the difference
        # is the attention path's share inside the model (its inputs are the stand-in's q/k/v, so
        # its mask density is the energy rule's on them, not the synthetic inputs' of the headline)
        class _NoAttention(torch.nn.Module):
            def forward(self, q, k, v):
                return v

        for blk in blocks:
            blk.inner_attention = _NoAttention()
        sec_null = timed()
    gemm_flops = 2.0 * L * (3 * hidden * hidden + hidden * hidden + 2 * hidden * 4 * hidden) * layers * steps
    att_s = sec - sec_null
    sparsity = attn.sparsity
    del blocks, x0
    torch.cuda.empty_cache()
    return {"what": "CogVideoX-5B 8-step video, 42 stand-in blocks at the model's dimensions "
                    "(random weights, batch 1, no VAE/scheduler), HIP sparse attention inside",
            "frames_per_s": round(frames / sec, 3), "s_per_video": round(sec, 4),
            "attention_s_per_video": round(att_s, 4),
            "attention_fraction": round(att_s / sec, 4),
            "attention_sparsity": round(sparsity, 4),
            "headline_attention_s_per_video": round(attn_ms_per_call * 1e-3 * calls, 4),
            "gemm_tflop_per_video": round(gemm_flops / 1e12, 1),
            "non_attention_tflops": round(gemm_flops / sec_null / 1e12, 1)}


def quality_vs_oracle(mod, qkv, variant):
    """Head 0 of one call of the timed configuration against the oracle with the GPU's own mask
    (SURVEY §8d Quality): PSNR, max|err| and the bf16 ULP histogram against (a) the reference's
    rounding (two branches, lse cast to bf16, bf16 combine: adaptive_attention) and (b) the exact
    fp64 joint softmax of the same two branches (joint_from_branches), and the reference's own
    distance from (b)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bsa_oracle as O
    from vblade import ops
    q, k, v = qkv
    out = mod(q, k, v)
    mask = mod.last_mask[:, :1].bool().cpu()
    cfg = O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan()
    fwd = O.adaptive_attention(q[:, :1].cpu(), k[:, :1].cpu(), v[:, :1].cpu(), cfg, None, None,
                               mask=mask, store_dtype=torch.bfloat16)
    ref = fwd["out"]
    exact = O.joint_from_branches(fwd, mod._log_gap(torch.bfloat16))
    got = out[:, :1].float().cpu()

    def psnr(a, b):
        mse = torch.mean((a.double() - b.double()) ** 2).item()
        peak = b.double().abs().max().item()
        return round(10 * math.log10(peak * peak / max(mse, 1e-30)), 2)

    h_ref, h_ex, h_re = (O.bf16_ulp_histogram(a, b) for a, b in ((got, ref), (got, exact), (ref, exact)))
    return {"head": 0, "psnr_db": psnr(got, ref),
            # how head_mask_type = ones(H) reads the predicted masks
            "mask_head_mode": mod.mask_head_mode,
            "forward_kernel": "attn_fwd_kernel",
            "max_abs": round((got - ref).abs().max().item(), 5),
            "ulp_hist": h_ref["ulp_hist"], "max_ulp": h_ref["max_ulp"],
            "vs": "oracle/bsa_oracle.adaptive_attention (reference rounding), same mask",
            "vs_exact": {"psnr_db": psnr(got, exact),
                         "max_abs": round((got.double() - exact).abs().max().item(), 5),
                         "ulp_hist": h_ex["ulp_hist"], "max_ulp": h_ex["max_ulp"],
                         "vs": "oracle joint_from_branches: the same branches combined exactly (fp64)"},
            "reference_vs_exact": {"max_abs": round((ref.double() - exact).abs().max().item(), 5),
                                   "ulp_hist": h_re["ulp_hist"], "max_ulp": h_re["max_ulp"]}}


def pmc_traffic(variant, timeout=300, density=None, band=False, local=False):
    """HBM-side bytes per attn_fwd_kernel launch from rocprofv3 PMC counters, one counter per
    pass (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
    tallies wide coalesced reads at half their bytes, so traffic = 2*FETCH + WRITE. The target
    is tools/attn_only.py: the same kernel on the same shapes, in a child process."""
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None
    vals = {}
    env = dict(os.environ, TMPDIR="/tmp")
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="vb_pmc_", dir="/tmp")
        cmd = [exe, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.join(ROOT, "tools", "attn_only.py"), variant, "3", "attn",
               "none" if density is None else str(density)] + (["band"] if band else ["local"] if local else [])
        try:
            subprocess.run(cmd, cwd="/tmp", env=env, timeout=timeout, check=True,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except (subprocess.SubprocessError, OSError):
            shutil.rmtree(d, ignore_errors=True)
            return None
        xs = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                kn = r.get("Kernel_Name", "")
                if "attn_fwd_kernel" in kn and r.get("Counter_Name") == counter:
                    xs.append(float(r["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not xs:
            return None
        vals[counter] = sum(xs) / len(xs)
    read_b = 2.0 * vals["FETCH_SIZE"] * 1024.0
    write_b = vals["WRITE_SIZE"] * 1024.0
    return {"bytes": round(read_b + write_b), "read_bytes": round(read_b),
            "write_bytes": round(write_b), "FETCH_SIZE_KiB": vals["FETCH_SIZE"],
            "WRITE_SIZE_KiB": vals["WRITE_SIZE"],
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes on tools/attn_only.py; "
                      "traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction)"}


# ---------------------------------------------------------------------------------- CPU baselines
def cpu_baseline_sdpa(variant):
    """the reference's CPU attention path (F.scaled_dot_product_attention with the
    50 % block mask as a token mask; blocksparseattn.py:93-94) on config 1's inputs, 1 warm-up +
    median of 3, on a head slice scaled to all heads, threads = the host cores this process may
    use. Baseline only."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ref_cpu_path as R
    heads = 8 if variant == "cog" else 2
    r = R.time_cpu_sdpa(variant, heads=heads)
    c = R.CONFIGS[variant]
    return {"value": round(r["masked_frames_per_s"], 6), "unit": "frames/s",
            "cores": r["threads"], "kind": "reference",
            "cpu_model": r["cpu_model"], "os_cpu_count": r["os_cpu_count"],
            "masked_s_per_call": round(r["masked_s_per_call"], 3),
            "dense_s_per_call": round(r["dense_s_per_call"], 3),
            "dense_frames_per_s": round(r["dense_frames_per_s"], 6),
            "sample": f"reference CPU path F.scaled_dot_product_attention(q,k,v,attn_mask=token "
                      f"mask) on BASELINE config 1 inputs [1,{c['H']},{c['L']},{c['D']}] bf16, "
                      f"50% block mask (seeds 0-3): {heads} of {c['H']} heads timed (1 warm-up + "
                      f"median of 3), scaled x{c['H'] // heads} heads x {DENOISE_STEPS * c['layers']} "
                      f"calls per video; threads = cgroup CPU quota of the box "
                      f"({r['threads']} of os.cpu_count()={r['os_cpu_count']})"}


def cpu_baseline_ml(calls, frames):
    """The multi-level oracle (oracle/ml_oracle.py: sampler, pooled scores, level mask, pyramid,
    multi-level softmax) timed on this host's cores: 2 heads of one call, scaled to a video."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bsa_oracle as O
    import gilbert_oracle as G
    import ml_oracle as ML
    V = VARIANTS["cog-ml"]
    heads = 2
    rows = torch.from_numpy(G.full_sequence_perm(45, 30, 13, 226).astype("int64"))
    L = rows.numel()
    g = torch.Generator().manual_seed(0)
    cent = torch.randn(1, heads, L // 128 + 1, V["D"], generator=g).repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    k = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    v = torch.randn(1, heads, L, V["D"], generator=g).bfloat16()
    qo = O.draw_sample_offsets(1, heads, generator=g)
    ko = O.draw_sample_offsets(1, heads, generator=g)
    t0 = time.perf_counter()
    r = ML.adaptive_multilevel_attention(q[:, :, rows], k[:, :, rows], v[:, :, rows], qo, ko)
    out = torch.empty_like(r["out"])
    out[:, :, rows] = r["out"]
    dt = time.perf_counter() - t0
    t_call = dt * V["H"] / heads
    return {"value": round(frames / (calls * t_call), 6), "unit": "frames/s",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"multi-level oracle (fp32 torch CPU), {heads} of {V['H']} heads of one "
                      f"[1,{V['H']},{L},{V['D']}] call: {dt:.2f} s; scaled x{V['H'] // heads} heads "
                      f"x {calls} calls per video"}


def cpu_baseline(variant, calls, frames):
    """The oracle (CPU restatement of the whole adaptive path, oracle/bsa_oracle.py) timed on
    this host's cores on a bounded sample: a twelfth (cog) or a sixth (wan) of the heads of one
    attention call at the full sequence length, scaled to a whole video's calls. Reported beside
    cpu_baseline (the reference's own CPU path) as a second, labelled number."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import bsa_oracle as O
    cfg = O.AdaptiveConfig.cogvideox() if variant == "cog" else O.AdaptiveConfig.wan()
    V = VARIANTS[variant]
    heads = 4 if variant == "cog" else 2
    L = cfg.width * cfg.height * cfg.depth + cfg.text_length
    g = torch.Generator().manual_seed(0)
    cent = torch.randn(1, heads, L // 128 + 1, V["D"], generator=g).repeat_interleave(128, 2)[:, :, :L]
    q = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    k = (torch.randn(1, heads, L, V["D"], generator=g) + 2 * cent).bfloat16()
    v = torch.randn(1, heads, L, V["D"], generator=g).bfloat16()
    qo = O.draw_sample_offsets(1, heads, generator=g)
    ko = O.draw_sample_offsets(1, heads, generator=g)
    threads = torch.get_num_threads()
    orig = O.block_sparse_attention

    def fp32_attn(*a, **kw):
        kw.setdefault("acc_dtype", torch.float32)
        return orig(*a, **kw)

    O.block_sparse_attention = fp32_attn
    try:
        t0 = time.perf_counter()
        O.adaptive_attention(q, k, v, cfg, qo, ko, store_dtype=torch.bfloat16)
        dt = time.perf_counter() - t0
    finally:
        O.block_sparse_attention = orig
    t_call = dt * V["H"] / heads
    return {"value": round(frames / (calls * t_call), 6), "unit": "frames/s",
            "cores": threads, "kind": "port",
            "sample": f"oracle adaptive path (fp32 torch CPU), {heads} of {V['H']} heads of one "
                      f"[1,{V['H']},{L},{V['D']}] call: {dt:.2f} s; scaled x{V['H'] // heads} heads "
                      f"x {calls} calls per video"}


if __name__ == "__main__":
    main()
