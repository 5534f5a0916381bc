"""Fused Gaussian head: the epilogue of LGM.forward_gaussians (core/models.py:95-117) on one HIP kernel per
direction (include/lgm_head.h, lgm_amd/csrc/head.hip).

The reference does, after the UNet (x [B*V, 14, h, w]):
    x = self.conv(x)                                                     # nn.Conv2d(14, 14, 1), core/models.py:34
    x = x.reshape(B, V, 14, h, w).permute(0, 1, 3, 4, 2).reshape(B, -1, 14)
    gaussians = cat([clamp(-1, 1), sigmoid, 0.1 * softplus, F.normalize, 0.5 * tanh + 0.5] of the slices)
(F.normalize with its default dim=1 on the [B, N, 4] rotation slice, core/models.py:43,112: every quaternion
component is normalised over the object's N Gaussians -- reproduced as written.)
`gaussian_head(x, conv, B, V)` returns the same [B, V*h*w, 14] fp32 tensor (differentiable w.r.t. x and the conv's
weight and bias) from one read of x. Drop-in use inside LGM.forward_gaussians:
    gaussians = gaussian_head(self.unet(images), self.conv, B, V)
`GaussianHead` owns such a conv (parameter names `conv.weight` / `conv.bias`, as LGM's state_dict).
The reference hard-codes V = 4 (core/models.py:98); here V is a parameter (LGM 'big' at 6 input views).
x may be fp32 or bf16 (the UNet under bf16 autocast); arithmetic is fp32, dx is returned in x's dtype.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _native as nat

_DT = {torch.float32: 0, torch.bfloat16: 1}


class _Head(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, B, V):
        nat.require_device_tensor(x, "x")
        if x.dtype not in _DT:
            raise nat.NativeError(f"gaussian_head supports float32 / bfloat16 inputs, got {x.dtype}")
        BV, C, h, w = x.shape
        if C != 14 or BV != B * V:
            raise ValueError(f"x must be [B*V, 14, h, w] with B*V = {B * V}, got {tuple(x.shape)}")
        x = x.contiguous()
        W = weight.detach().reshape(14, 14).float().contiguous()
        b = None if bias is None else bias.detach().float().contiguous()
        out = torch.empty(B, V * h * w, 14, device=x.device, dtype=torch.float32)
        rot_norm = torch.empty(B, 4, device=x.device, dtype=torch.float32)
        L = nat.lib()
        ws_bytes = L.lgm_gaussian_head_workspace_size(B, V, h, w)
        ws = torch.empty(max(ws_bytes, 1), device=x.device, dtype=torch.uint8)
        nat.check(L.lgm_gaussian_head_forward(_DT[x.dtype], B, V, h, w, nat.ptr(x), nat.ptr(W), nat.ptr(b),
                                              nat.ptr(out), nat.ptr(rot_norm), nat.ptr(ws), ws_bytes,
                                              nat.stream_of(x.device), nat.diag()), "lgm_gaussian_head_forward")
        ctx.save_for_backward(x, W, b if b is not None else W.new_empty(0), rot_norm)
        ctx.dims = (B, V, h, w, bias is not None, weight.shape, weight.dtype, None if bias is None else bias.dtype)
        return out

    @staticmethod
    def backward(ctx, d_out):
        x, W, b, rot_norm = ctx.saved_tensors
        B, V, h, w, has_bias, wshape, wdtype, bdtype = ctx.dims
        L = nat.lib()
        d_out = d_out.float().contiguous()
        dx = torch.empty_like(x)
        dW = torch.empty(14, 14, device=x.device, dtype=torch.float32)
        db = torch.empty(14, device=x.device, dtype=torch.float32) if has_bias else None
        ws_bytes = L.lgm_gaussian_head_workspace_size(B, V, h, w)
        ws = torch.empty(max(ws_bytes, 1), device=x.device, dtype=torch.uint8)
        nat.check(L.lgm_gaussian_head_backward(_DT[x.dtype], B, V, h, w, nat.ptr(x), nat.ptr(W),
                                               nat.ptr(b) if has_bias else None, nat.ptr(rot_norm), nat.ptr(d_out),
                                               nat.ptr(dx),
                                               nat.ptr(dW), nat.ptr(db), nat.ptr(ws), ws_bytes,
                                               nat.stream_of(x.device), nat.diag()), "lgm_gaussian_head_backward")
        return dx, dW.reshape(wshape).to(wdtype), None if db is None else db.to(bdtype), None, None


def gaussian_head(x: torch.Tensor, conv: nn.Conv2d, B: int, V: int) -> torch.Tensor:
    """x [B*V, 14, h, w] (UNet output) -> Gaussians [B, V*h*w, 14] fp32 (core/models.py:96-117)."""
    if conv.kernel_size != (1, 1) or conv.in_channels != 14 or conv.out_channels != 14 or conv.groups != 1:
        raise ValueError("conv must be nn.Conv2d(14, 14, kernel_size=1)")
    if not x.is_cuda:  # BASELINE config 1 (CPU-only inference): torch ops, lgm_amd/cpu.py
        from .cpu import gaussian_head_cpu
        return gaussian_head_cpu(x, conv.weight, conv.bias, int(B), int(V))
    return _Head.apply(x, conv.weight, conv.bias, int(B), int(V))


class GaussianHead(nn.Module):
    """The 1x1 conv + permute + activations of LGM as a module (self.conv of core/models.py:34)."""

    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(14, 14, kernel_size=1)

    def forward(self, x: torch.Tensor, B: int, V: int) -> torch.Tensor:
        return gaussian_head(x, self.conv, B, V)
