"""TEST INFRASTRUCTURE ONLY -- fp32 torch restatement of LGM.forward_gaussians' epilogue (core/models.py:40-44,
96-117), the oracle of the fused Gaussian head (lgm_amd/head.py). The reference itself is not imported here: its
module pulls kiui / LPIPS (unavailable offline); these lines are the same torch ops in the same order."""
from __future__ import annotations

import torch
import torch.nn.functional as F


def forward_gaussians_epilogue(x, weight, bias, B: int, V: int):
    y = F.conv2d(x, weight, bias)  # self.conv, core/models.py:96
    _, C, h, w = y.shape
    y = y.reshape(B, V, C, h, w).permute(0, 1, 3, 4, 2).reshape(B, -1, C)  # :98, :107
    pos = y[..., 0:3].clamp(-1, 1)  # :40 pos_act
    opacity = torch.sigmoid(y[..., 3:4])  # :42
    scale = 0.1 * F.softplus(y[..., 4:7])  # :41
    rotation = F.normalize(y[..., 7:11])  # :43,112 -- F.normalize's default dim=1: over the N Gaussians
    rgbs = 0.5 * torch.tanh(y[..., 11:]) + 0.5  # :44
    return torch.cat([pos, opacity, scale, rotation, rgbs], dim=-1)  # :115
