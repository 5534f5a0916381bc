"""fp32 torch restatement of LGM's multi-view attention -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py may import this module; the product path
(lgm_amd/attention.py) never does. It restates:
  * Attention.forward (core/attention.py:51-64): qkv Linear -> [3, B, H, L, D], softmax(q*scale @ k^T) @ v, proj;
    MemEffAttention (core/attention.py:67-84) computes the same function through xformers;
  * MVAttention.forward (core/unet.py:35-49): GroupNorm, [B*F, C, h, w] -> [B, F*h*w, C] tokens, attention,
    back to [B*F, C, h, w], (x + res) * skip_scale.
Pinned against the reference's own modules through tests/golden/attn_*.npz (tests/test_attention.py).
Parameters are passed as a dict with the reference's state_dict names (qkv.weight, proj.weight, proj.bias,
optional qkv.bias; norm.weight / norm.bias and attn.* for MVAttention).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def attention_core(q, k, v, scale):
    """softmax(scale q k^T) v on [B, H, L, D] tensors (core/attention.py:54-60)."""
    attn = (q * scale) @ k.transpose(-2, -1)
    return attn.softmax(dim=-1) @ v


def attention(x, p, num_heads, prefix=""):
    """x [B, L, C] -> [B, L, C] (core/attention.py:51-64)."""
    B, L, C = x.shape
    qkv = F.linear(x, p[prefix + "qkv.weight"], p.get(prefix + "qkv.bias"))
    qkv = qkv.reshape(B, L, 3, num_heads, C // num_heads).permute(2, 0, 3, 1, 4)
    scale = (C // num_heads) ** -0.5
    y = attention_core(qkv[0], qkv[1], qkv[2], scale)
    y = y.transpose(1, 2).reshape(B, L, C)
    return F.linear(y, p[prefix + "proj.weight"], p.get(prefix + "proj.bias"))


def mv_attention(x, p, num_heads, num_frames, skip_scale=1.0, groups=32, eps=1e-5, residual=True):
    """x [B*F, C, h, w] -> same (core/unet.py:35-49)."""
    BV, C, H, W = x.shape
    B = BV // num_frames
    res = x
    x = F.group_norm(x, groups, p["norm.weight"], p["norm.bias"], eps)
    x = x.reshape(B, num_frames, C, H, W).permute(0, 1, 3, 4, 2).reshape(B, -1, C)
    x = attention(x, p, num_heads, prefix="attn.")
    x = x.reshape(B, num_frames, H, W, C).permute(0, 1, 4, 2, 3).reshape(BV, C, H, W)
    if residual:
        x = (x + res) * skip_scale
    return x
