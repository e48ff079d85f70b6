"""Real-activation capture for mask-parity goldens.

The reference's debug module (cogvideox/train/special_attentions_local/TrainRelated/
blocksparseattn.py:367-386) is an ``inner_attention`` that, for every call, derives
``timestep = counter % (8 * 42) // 42`` and ``layer = counter % 42`` and, at timestep 5, saves
``q.pt`` and ``k.pt`` (detached, on the CPU) under ``<root>/timestep_{t}_layer_{l}/``, then returns
dense attention. ``QKDumpAttention`` reproduces that capture (same counter arithmetic and file
layout, any set of timesteps) in front of any attention module — the sparse module itself by
default, so a sampler run both renders and records. ``load_dumps`` reads them back with
``torch.load(weights_only=True)``; tools/replay_dumps.py replays them through the HIP predictor and
the oracle to measure mask parity and output quality on real attention statistics.
"""
from __future__ import annotations

import os
from typing import Iterable, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


class DenseAttention(nn.Module):
    """The reference debug module's ``standard_attn`` (SDPA on [B,H,L,D])."""

    def forward(self, q, k, v):
        return F.scaled_dot_product_attention(q, k, v)


class QKDumpAttention(nn.Module):
    def __init__(self, root: str, inner: Optional[nn.Module] = None, *, layers: int = 42, steps: int = 8,
                 timesteps: Iterable[int] = (5,), save_v: bool = False):
        super().__init__()
        self.root = root
        self.inner = inner if inner is not None else DenseAttention()
        self.layers, self.steps = int(layers), int(steps)
        self.timesteps = set(int(t) for t in timesteps)
        self.save_v = save_v
        self.counter = 0

    def dump_dir(self, timestep: int, layer: int) -> str:
        return os.path.join(self.root, f"timestep_{timestep}_layer_{layer}")

    def forward(self, q, k, v):
        timestep = self.counter % (self.steps * self.layers) // self.layers
        layer = self.counter % self.layers
        if timestep in self.timesteps:
            d = self.dump_dir(timestep, layer)
            os.makedirs(d, exist_ok=True)
            torch.save(q.detach().cpu(), os.path.join(d, "q.pt"))
            torch.save(k.detach().cpu(), os.path.join(d, "k.pt"))
            if self.save_v:
                torch.save(v.detach().cpu(), os.path.join(d, "v.pt"))
        self.counter += 1
        return self.inner(q, k, v)


def load_dumps(root: str) -> List[Tuple[int, int, dict]]:
    """[(timestep, layer, {"q": tensor, "k": tensor[, "v": tensor]})] sorted by (timestep, layer)."""
    out = []
    if not os.path.isdir(root):
        return out
    for name in os.listdir(root):
        if not name.startswith("timestep_"):
            continue
        parts = name.split("_")
        try:
            t, layer = int(parts[1]), int(parts[3])
        except (IndexError, ValueError):
            continue
        d = os.path.join(root, name)
        tensors = {}
        for key in ("q", "k", "v"):
            f = os.path.join(d, f"{key}.pt")
            if os.path.exists(f):
                tensors[key] = torch.load(f, map_location="cpu", weights_only=True)
        if "q" in tensors and "k" in tensors:
            out.append((t, layer, tensors))
    out.sort(key=lambda x: (x[0], x[1]))
    return out
