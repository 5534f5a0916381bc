"""Synthetic inputs pinned by SURVEY.md §8(d): raw ~ N(0,1) mapped through LGM's activations
(core/models.py:40-44, 109-115)."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def synthetic_gaussians(B: int, N: int, seed: int = 0) -> torch.Tensor:
    """[B,N,14] fp32 CPU Gaussians: pos = clamp(0.35 raw), opacity = sigmoid, scale = 0.1 softplus(raw - 2.2522),
    rot = normalize, rgb = 0.5 tanh + 0.5."""
    g = torch.Generator("cpu").manual_seed(seed)
    raw = torch.randn(B, N, 14, generator=g, dtype=torch.float32)
    pos = (0.35 * raw[..., 0:3]).clamp(-1, 1)
    opacity = torch.sigmoid(raw[..., 3:4])
    scale = 0.1 * F.softplus(raw[..., 4:7] - 2.2522)
    rot = F.normalize(raw[..., 7:11], dim=-1)
    rgb = 0.5 * torch.tanh(raw[..., 11:14]) + 0.5
    return torch.cat([pos, opacity, scale, rot, rgb], dim=-1).contiguous()


def synthetic_upstream_grads(B: int, V: int, H: int, W: int, seed: int = 1):
    """dL/dimage, dL/dalpha ~ N(0,1) (seed), dL/ddepth = 0; plus a seeded bg = rand(3) as in
    core/models.py:135-136."""
    g = torch.Generator("cpu").manual_seed(seed)
    d_img = torch.randn(B, V, 3, H, W, generator=g)
    d_alpha = torch.randn(B, V, 1, H, W, generator=g)
    d_depth = torch.zeros(B, V, 1, H, W)
    bg = torch.rand(3, generator=g)
    return d_img, d_depth, d_alpha, bg
