"""Multi-view self-attention of LGM's UNet on the HIP flash-attention kernels (lgm_amd/csrc/attention.hip).

Drop-in replacements, with the same constructors, submodules (so state_dicts load unchanged) and forward
signatures as the reference:
  * Attention / MemEffAttention -- core/attention.py:31-84. Both compute softmax(scale q k^T) v through the MFMA
    kernels; the reference's xformers call (core/attention.py:74-84) and its fp32 torch fallback (:51-64) are the
    same function;
  * MVAttention -- core/unet.py:11-49 (GroupNorm, the [B*F, C, h, w] <-> [B, F*h*w, C] token reshape across the
    F views, attention, residual * skip_scale).
q, k and v are read in place from the packed qkv Linear output and dq/dk/dv are written back packed, so the
reshape/unbind/permute of the reference costs no copies. fp32, bf16 and fp16 activations are supported (bf16 is
what LGM trains with under accelerate's mixed precision); accumulation is fp32.
CPU tensors (BASELINE config 1, CPU-only inference) take the torch path of lgm_amd/cpu.py, the reference's fallback
attention (core/attention.py:51-64); GPU tensors always run the HIP kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _native as nat
from .linear import linear as _linear16

_DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


def _dtype_code(t: torch.Tensor) -> int:
    if t.dtype not in _DTYPES:
        raise nat.NativeError(f"attention supports float32/bfloat16/float16, got {t.dtype}")
    return _DTYPES[t.dtype]


class _PackedAttention(torch.autograd.Function):
    """o = softmax(scale q k^T) v with q, k, v = qkv.unbind(2), qkv [B, L, 3, H, D] contiguous -> o [B, L, H, D]."""

    @staticmethod
    def forward(ctx, qkv: torch.Tensor, scale: float):
        nat.require_device_tensor(qkv, "qkv")
        qkv = qkv.contiguous()
        B, L, three, H, D = qkv.shape
        if three != 3:
            raise nat.NativeError(f"qkv must be [B, L, 3, H, D], got {tuple(qkv.shape)}")
        dt = _dtype_code(qkv)
        o = torch.empty((B, L, H, D), device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty((B, H, L), device=qkv.device, dtype=torch.float32)
        if B * L * H > 0:
            base, es = qkv.data_ptr(), qkv.element_size()
            L_ = nat.lib()
            nat.check(L_.lgm_attn_forward(dt, B, L, H, D, float(scale), base, base + H * D * es,
                                          base + 2 * H * D * es, 3 * H * D, nat.ptr(o), nat.ptr(lse),
                                          nat.stream_of(qkv.device), nat.diag()), "lgm_attn_forward")
        ctx.save_for_backward(qkv, o, lse)
        ctx.scale = float(scale)
        return o

    @staticmethod
    def backward(ctx, d_o: torch.Tensor):
        qkv, o, lse = ctx.saved_tensors
        B, L, _, H, D = qkv.shape
        d_o = d_o.to(qkv.dtype).contiguous()
        d_qkv = torch.empty_like(qkv)
        if B * L * H > 0:
            dt = _dtype_code(qkv)
            L_ = nat.lib()
            ws_bytes = L_.lgm_attn_workspace_size(dt, B, L, H, D)
            ws = torch.empty(max(ws_bytes, 1), device=qkv.device, dtype=torch.uint8)
            base, dbase, es = qkv.data_ptr(), d_qkv.data_ptr(), qkv.element_size()
            hd = H * D * es
            nat.check(L_.lgm_attn_backward(dt, B, L, H, D, ctx.scale, base, base + hd, base + 2 * hd, 3 * H * D,
                                           nat.ptr(o), nat.ptr(lse), nat.ptr(d_o), dbase, dbase + hd,
                                           dbase + 2 * hd, 3 * H * D, nat.ptr(ws), ws_bytes,
                                           nat.stream_of(qkv.device), nat.diag()), "lgm_attn_backward")
        return d_qkv, None


def packed_attention(qkv: torch.Tensor, scale: float | None = None) -> torch.Tensor:
    """qkv [B, L, 3, H, D] (the reshaped qkv Linear output) -> [B, L, H, D]; scale defaults to D^-1/2.
    GPU tensors run the HIP kernels; CPU tensors the torch path of lgm_amd/cpu.py (BASELINE config 1)."""
    if scale is None:
        scale = qkv.shape[-1] ** -0.5
    if not qkv.is_cuda:
        from .cpu import attention_cpu
        return attention_cpu(qkv, scale)
    return _PackedAttention.apply(qkv, scale)


def memory_efficient_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, attn_bias=None,
                               scale: float | None = None) -> torch.Tensor:
    """xformers.ops.memory_efficient_attention subset used by core/attention.py:79: q, k, v [B, L, H, D], no bias,
    no dropout. Views of one packed [B, L, 3, H, D] tensor (what unbind(qkv, 2) yields) are used in place;
    otherwise the three are stacked first."""
    if attn_bias is not None:
        raise NotImplementedError("attn_bias is not supported (LGM never passes one: core/unet.py:43)")
    if not (q.shape == k.shape == v.shape) or q.dim() != 4:
        raise ValueError("q, k, v must all be [B, L, H, D]")
    B, L, H, D = q.shape
    es = q.element_size()
    packed = (q.dtype == k.dtype == v.dtype and q.stride() == k.stride() == v.stride()
              and q.stride() == (L * 3 * H * D, 3 * H * D, D, 1)
              and k.data_ptr() - q.data_ptr() == H * D * es and v.data_ptr() - q.data_ptr() == 2 * H * D * es)
    if packed:
        qkv = torch.as_strided(q, (B, L, 3, H, D), (L * 3 * H * D, 3 * H * D, H * D, D, 1))
    else:
        qkv = torch.stack([q, k, v], dim=2)
    return packed_attention(qkv, scale)


class Attention(nn.Module):
    """core/attention.py:31-64 (same constructor and parameters)."""

    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = False, proj_bias: bool = True,
                 attn_drop: float = 0.0, proj_drop: float = 0.0) -> None:
        super().__init__()
        self.num_heads = num_heads
        head_dim = dim // num_heads
        self.scale = head_dim ** -0.5
        self.qkv = nn.Linear(dim, dim * 3, bias=qkv_bias)
        self.attn_drop = nn.Dropout(attn_drop)
        self.proj = nn.Linear(dim, dim, bias=proj_bias)
        self.proj_drop = nn.Dropout(proj_drop)
        self.native_wgrad = True  # (a plain attribute: not in the state_dict)

    def _lin(self, lin: nn.Linear, x: torch.Tensor) -> torch.Tensor:
        # 16-bit GPU Linears take their weight gradient from the HIP split-K kernel (lgm_amd/linear.py);
        # native_wgrad = False: torch's autograd through nn.Linear, as upstream
        return _linear16(x, lin) if self.native_wgrad else lin(x)

    def _attend(self, x: torch.Tensor) -> torch.Tensor:
        if self.training and self.attn_drop.p > 0:
            raise NotImplementedError("attention-probability dropout is not implemented (LGM uses attn_drop=0)")
        B, N, C = x.shape
        qkv = self._lin(self.qkv, x).reshape(B, N, 3, self.num_heads, C // self.num_heads)
        y = packed_attention(qkv, self.scale).reshape(B, N, C)
        return self.proj_drop(self._lin(self.proj, y))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self._attend(x)


class MemEffAttention(Attention):
    """core/attention.py:67-84."""

    def forward(self, x: torch.Tensor, attn_bias=None) -> torch.Tensor:
        if attn_bias is not None:
            raise AssertionError("attn_bias (nested tensors) is not supported")
        return self._attend(x)


def _autocast_dtype(dev_type: str):
    if torch.is_autocast_enabled(dev_type):
        return torch.get_autocast_dtype(dev_type)
    return None


class _NormTokens(torch.autograd.Function):
    """GroupNorm of x [B*F, C, H, W] straight into MVAttention's token layout [B, F*H*W, C] (core/unet.py:40-42) in
    one HIP pass (lgm_mva_norm_tokens). Also returns x itself (an alias) for the residual of core/unet.py:47, so the
    residual's gradient arrives here and the backward (lgm_mva_norm_tokens_backward) adds it to the GroupNorm's dx
    in the same pass, instead of autograd summing the two afterwards."""

    @staticmethod
    def forward(ctx, x, weight, bias, F: int, groups: int, eps: float, tok_dtype):
        BF, C, H, W = x.shape
        B, HW = BF // F, H * W
        x = x.contiguous()
        tok = torch.empty((B, F * HW, C), device=x.device, dtype=tok_dtype)
        mean = torch.empty((BF, groups), device=x.device, dtype=torch.float32)
        rstd = torch.empty((BF, groups), device=x.device, dtype=torch.float32)
        w = None if weight is None else weight.detach().float().contiguous()
        b = None if bias is None else bias.detach().float().contiguous()
        L_ = nat.lib()
        ws_bytes = L_.lgm_mva_workspace_size(B, F, C, HW, groups)
        ws = torch.empty(max(ws_bytes, 1), device=x.device, dtype=torch.uint8)
        nat.check(L_.lgm_mva_norm_tokens(_dtype_code(x), _dtype_code(tok), B, F, C, HW, groups, float(eps), nat.ptr(x),
                                         nat.ptr(w), nat.ptr(b), nat.ptr(tok), nat.ptr(mean), nat.ptr(rstd),
                                         nat.ptr(ws), ws_bytes, nat.stream_of(x.device), nat.diag()),
                  "lgm_mva_norm_tokens")
        ctx.save_for_backward(x, weight, mean, rstd)
        ctx.shape = (B, F, C, H, W, groups)
        ctx.set_materialize_grads(False)
        return tok, x

    @staticmethod
    def backward(ctx, d_tok, d_res):
        x, weight, mean, rstd = ctx.saved_tensors
        B, F, C, H, W, groups = ctx.shape
        need_x = ctx.needs_input_grad[0]
        need_w = weight is not None and ctx.needs_input_grad[1]
        need_b = weight is not None and ctx.needs_input_grad[2]
        if d_tok is None:  # only the residual's gradient reached x
            return (d_res if need_x else None), None, None, None, None, None, None
        d_tok = d_tok.contiguous()
        if d_res is not None:
            d_res = d_res.to(x.dtype).contiguous()
        dx = torch.empty_like(x) if need_x else None
        dw = torch.empty(C, device=x.device, dtype=torch.float32) if need_w else None
        db = torch.empty(C, device=x.device, dtype=torch.float32) if need_b else None
        L_ = nat.lib()
        ws_bytes = L_.lgm_mva_backward_workspace_size(B, F, C, H * W, groups)
        ws = torch.empty(max(ws_bytes, 1), device=x.device, dtype=torch.uint8)
        gamma = None if weight is None else weight.detach().float().contiguous()
        nat.check(L_.lgm_mva_norm_tokens_backward(_dtype_code(x), _dtype_code(d_tok), B, F, C, H * W, groups,
                                                  nat.ptr(x), nat.ptr(gamma), nat.ptr(mean), nat.ptr(rstd),
                                                  nat.ptr(d_tok), nat.ptr(d_res), nat.ptr(dx), nat.ptr(dw),
                                                  nat.ptr(db), nat.ptr(ws), ws_bytes, nat.stream_of(x.device),
                                                  nat.diag()), "lgm_mva_norm_tokens_backward")
        dw = None if dw is None else dw.to(weight.dtype)
        db = None if db is None else db.to(weight.dtype)
        return dx, dw, db, None, None, None, None


class _TokensOut(torch.autograd.Function):
    """MVAttention's [B, F*H*W, C] -> [B*F, C, H, W] permute fused with (y + res) * skip_scale (core/unet.py:45-48),
    one HIP pass (lgm_mva_tokens_out); res None: the permute alone. Backward: one HIP pass
    (lgm_mva_tokens_out_backward) writes the tokens' gradient and the residual's."""

    @staticmethod
    def forward(ctx, y, res, F: int, H: int, W: int, skip: float):
        B, L, C = y.shape
        y = y.contiguous()
        out_dtype = y.dtype if res is None else torch.promote_types(y.dtype, res.dtype)
        out = torch.empty((B * F, C, H, W), device=y.device, dtype=out_dtype)
        r = None if res is None else res.contiguous()
        nat.check(nat.lib().lgm_mva_tokens_out(_dtype_code(y), 0 if r is None else _dtype_code(r), _dtype_code(out),
                                               B, F, C, H * W, nat.ptr(y), nat.ptr(r), float(skip), nat.ptr(out),
                                               nat.stream_of(y.device), nat.diag()), "lgm_mva_tokens_out")
        ctx.meta = (B, F, C, H, W, float(skip), y.dtype, None if res is None else res.dtype)
        return out

    @staticmethod
    def backward(ctx, d_out):
        B, F, C, H, W, skip, ydt, rdt = ctx.meta
        d_out = d_out.contiguous()
        d_y = torch.empty((B, F * H * W, C), device=d_out.device, dtype=ydt)
        want_res = rdt is not None and ctx.needs_input_grad[1]
        d_res = torch.empty((B * F, C, H, W), device=d_out.device, dtype=rdt) if want_res else None
        nat.check(nat.lib().lgm_mva_tokens_out_backward(_dtype_code(d_out), _dtype_code(d_y),
                                                        _dtype_code(d_res) if want_res else 0, B, F, C, H * W,
                                                        nat.ptr(d_out), skip if rdt is not None else 1.0,
                                                        nat.ptr(d_y), nat.ptr(d_res), nat.stream_of(d_out.device),
                                                        nat.diag()), "lgm_mva_tokens_out_backward")
        return d_y, d_res, None, None, None, None


class MVAttention(nn.Module):
    """core/unet.py:11-49: self-attention across the tokens of all `num_frames` views of an object.

    num_frames defaults to 4 like the reference (whose UNet never overrides it, core/unet.py:24 'hardcoded');
    here it is a real parameter."""

    def __init__(self, dim: int, num_heads: int = 8, qkv_bias: bool = False, proj_bias: bool = True,
                 attn_drop: float = 0.0, proj_drop: float = 0.0, groups: int = 32, eps: float = 1e-5,
                 residual: bool = True, skip_scale: float = 1, num_frames: int = 4):
        super().__init__()
        self.residual = residual
        self.skip_scale = skip_scale
        self.num_frames = num_frames
        self.norm = nn.GroupNorm(num_groups=groups, num_channels=dim, eps=eps, affine=True)
        self.attn = MemEffAttention(dim, num_heads, qkv_bias, proj_bias, attn_drop, proj_drop)
        self.fused = True  # GPU: the HIP GroupNorm->tokens and tokens->residual kernels (False: torch ops, as upstream)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        BV, C, H, W = x.shape
        if BV % self.num_frames:
            raise ValueError(f"batch {BV} is not a multiple of num_frames={self.num_frames}")
        B = BV // self.num_frames
        if self.fused and x.is_cuda and x.dtype in _DTYPES:
            # fused token layout kernels around the attention core (same math; GroupNorm in fp32 as under autocast)
            ac = _autocast_dtype("cuda")
            tok_dtype = ac if ac is not None else x.dtype
            tok, xres = _NormTokens.apply(x, self.norm.weight, self.norm.bias, self.num_frames, self.norm.num_groups,
                                          self.norm.eps, tok_dtype)
            y = self.attn(tok)
            return _TokensOut.apply(y, xres if self.residual else None, self.num_frames, H, W,
                                    self.skip_scale if self.residual else 1.0)
        res = x
        x = self.norm(x)
        x = x.reshape(B, self.num_frames, C, H, W).permute(0, 1, 3, 4, 2).reshape(B, -1, C)
        x = self.attn(x)
        x = x.reshape(B, self.num_frames, H, W, C).permute(0, 1, 4, 2, 3).reshape(BV, C, H, W)
        if self.residual:
            x = (x + res) * self.skip_scale
        return x
