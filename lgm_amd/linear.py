"""MVAttention's qkv / proj Linears (core/attention.py:46,48) under 16-bit autocast, with the weight gradient on the
HIP split-K MFMA kernel (lgm_amd/csrc/wgrad.hip, include/lgm_linear.h).

The forward and the input gradient are the library GEMMs torch's autocast runs for nn.Linear (F.linear on the
16-bit casts of input, weight and bias; grad_input = grad_out @ weight). The weight and bias gradients --
grad_out^T @ input and grad_out.sum(0), reductions over every token of the batch that hipBLASLt ran on a fifth of the
chip -- come from lgm_linear_wgrad, in fp32 straight into the fp32 parameters' gradients (torch rounds them to the
autocast dtype first and casts back). fp32 Linears (no autocast) stay on torch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _native as nat

_CODES = {torch.bfloat16: 1, torch.float16: 2}  # include/lgm_attn.h LGM_ATTN_BF16 / LGM_ATTN_F16


class _Linear16(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dt):
        with torch.autocast("cuda", enabled=False):
            x16 = x.to(dt)
            w16 = weight.to(dt)
            out = F.linear(x16, w16, None if bias is None else bias.to(dt))
        ctx.save_for_backward(x16, w16)
        ctx.meta = (x.dtype, weight.dtype, None if bias is None else bias.dtype, dt)
        return out

    @staticmethod
    def backward(ctx, g):
        x16, w16 = ctx.saved_tensors
        xdt, wdt, bdt, dt = ctx.meta
        M, N = w16.shape
        g2 = g.to(dt).reshape(-1, M).contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            gx = (g2 @ w16).reshape(*g.shape[:-1], N).to(xdt)
        dw = db = None
        want_w = ctx.needs_input_grad[1]
        want_b = bdt is not None and ctx.needs_input_grad[2]
        if want_w or want_b:
            x2 = x16.reshape(-1, N).contiguous()
            K = x2.shape[0]
            dw = torch.empty((M, N), device=g.device, dtype=torch.float32)
            db = torch.empty((M,), device=g.device, dtype=torch.float32) if want_b else None
            L = nat.lib()
            ws_bytes = L.lgm_linear_wgrad_workspace_size(K, M, N, int(want_b))
            ws = torch.empty(max(ws_bytes, 1), device=g.device, dtype=torch.uint8)
            nat.check(L.lgm_linear_wgrad(_CODES[dt], K, M, N, nat.ptr(g2), M, nat.ptr(x2), N, nat.ptr(dw), nat.ptr(db),
                                         nat.ptr(ws), ws_bytes, nat.stream_of(g.device), nat.diag()),
                      "lgm_linear_wgrad")
            dw = dw.to(wdt) if want_w else None
            db = None if db is None else db.to(bdt)
        return gx, dw, db, None


def _supported(x: torch.Tensor, weight: torch.Tensor, dt) -> bool:
    M, N = weight.shape
    return dt in _CODES and x.is_cuda and M % 8 == 0 and N % 8 == 0


def linear(x: torch.Tensor, lin: torch.nn.Linear) -> torch.Tensor:
    """lin(x), with the HIP weight gradient where the Linear runs in 16 bits on the GPU: under bf16 / fp16 autocast,
    or on a 16-bit module without autocast. Anything else (fp32, CPU tensors, widths not a multiple of 8) is lin(x),
    and so is a call that records no graph (inference: no weight gradient to compute, and the autograd Function's
    host cost per call -- with its own weight cast -- would only slow the launch stream of LGM's 16-block forward)."""
    if not (torch.is_grad_enabled() and (x.requires_grad or lin.weight.requires_grad)):
        return lin(x)
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
    elif x.dtype in _CODES and lin.weight.dtype == x.dtype:
        dt = x.dtype
    else:
        return lin(x)
    if not _supported(x, lin.weight, dt):
        return lin(x)
    return _Linear16.apply(x, lin.weight, lin.bias, dt)
