"""Differentiable float64 restatement of the rasterizer FORWARD -- TEST INFRASTRUCTURE ONLY.

Used to pin the analytic backward of oracle/raster_oracle.c (and through it the HIP backward): torch autograd of
this forward, in float64, must agree with the hand-derived reverse-compositing gradient
wherever the forward is differentiable. The discrete decisions that upstream takes in fp32 (culling, tile rects,
per-tile depth order) are taken from the fp32 oracle so both sides composite the same lists; the continuous
arithmetic (projection, EWA covariance, conic, alpha, compositing) is recomputed here with autograd.

Known non-differentiable points where upstream's analytic gradient is not the true derivative (tests keep inputs
away from them): alpha clamped at 0.99, and |t.x/t.z| or |t.y/t.z| beyond 1.3 tan(fov/2).
"""
from __future__ import annotations

import numpy as np
import torch

from . import oracle as _oracle


def _quat_to_Rm(q: torch.Tensor) -> torch.Tensor:
    """Math-form (row, col) of upstream's glm rotation matrix (= standard quaternion matrix transposed),
    quaternion (r, x, y, z) NOT normalised (as upstream)."""
    r, x, y, z = q.unbind(-1)
    row0 = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y + r * z), 2 * (x * z - r * y)], -1)
    row1 = torch.stack([2 * (x * y - r * z), 1 - 2 * (x * x + z * z), 2 * (y * z + r * x)], -1)
    row2 = torch.stack([2 * (x * z + r * y), 2 * (y * z - r * x), 1 - 2 * (x * x + y * y)], -1)
    return torch.stack([row0, row1, row2], -2)


def render_view(g: torch.Tensor, view16, proj16, tanfov: float, H: int, W: int, bg, scale_modifier: float = 1.0):
    """g [N,14] float64 (requires_grad ok). Returns (color [3,H,W], depth [1,H,W], alpha [1,H,W])."""
    g32 = g.detach().to(torch.float32).numpy()
    ts, ids = _oracle.tile_lists(g32, view16, proj16, tanfov, H, W, scale_modifier)
    dt = g.dtype
    Veff = torch.as_tensor(np.asarray(view16, np.float64).reshape(4, 4).T, dtype=dt)
    Peff = torch.as_tensor(np.asarray(proj16, np.float64).reshape(4, 4).T, dtype=dt)
    bg = torch.as_tensor(np.asarray(bg, np.float64), dtype=dt)
    N = g.shape[0]
    means, opac, scales, q, col = g[:, 0:3], g[:, 3], g[:, 4:7], g[:, 7:11], g[:, 11:14]
    mh = torch.cat([means, torch.ones(N, 1, dtype=dt)], -1)
    hom = mh @ Peff.T
    pw = 1.0 / (hom[:, 3] + 1e-7)
    ppx, ppy = hom[:, 0] * pw, hom[:, 1] * pw
    t = mh @ Veff[:3].T
    fx = W / (2.0 * tanfov)
    fy = H / (2.0 * tanfov)
    lim = 1.3 * tanfov
    tz = t[:, 2]
    tx = torch.clamp(t[:, 0] / tz, -lim, lim) * tz
    ty = torch.clamp(t[:, 1] / tz, -lim, lim) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([torch.stack([fx / tz, zero, -fx * tx / (tz * tz)], -1),
                     torch.stack([zero, fy / tz, -fy * ty / (tz * tz)], -1)], -2)  # [N,2,3]
    A = J @ Veff[:3, :3]
    Rm = _quat_to_Rm(q)
    S2 = torch.diag_embed((scale_modifier * scales) ** 2)
    Sig = Rm.transpose(-1, -2) @ S2 @ Rm
    cov2 = A @ Sig @ A.transpose(-1, -2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    con = torch.stack([c / det, -b / det, a / det], -1)
    px = ((ppx + 1) * W - 1) * 0.5
    py = ((ppy + 1) * H - 1) * 0.5
    depth = t[:, 2]

    gx = (W + 15) // 16
    color = torch.zeros(3, H, W, dtype=dt)
    out_d = torch.zeros(1, H, W, dtype=dt)
    out_a = torch.zeros(1, H, W, dtype=dt)
    rows = []
    for tile in range(len(ts) - 1):
        tyi, txi = divmod(tile, gx)
        ys = torch.arange(tyi * 16, min(tyi * 16 + 16, H))
        xs = torch.arange(txi * 16, min(txi * 16 + 16, W))
        if len(ys) == 0 or len(xs) == 0:
            continue
        yy, xx = torch.meshgrid(ys, xs, indexing="ij")
        pfx, pfy = xx.reshape(-1).to(dt), yy.reshape(-1).to(dt)
        P = pfx.shape[0]
        T = torch.ones(P, dtype=dt)
        C = torch.zeros(P, 3, dtype=dt)
        D = torch.zeros(P, dtype=dt)
        done = torch.zeros(P, dtype=torch.bool)
        for k in range(ts[tile], ts[tile + 1]):
            gi = int(ids[k])
            dx = px[gi] - pfx
            dy = py[gi] - pfy
            power = -0.5 * (con[gi, 0] * dx * dx + con[gi, 2] * dy * dy) - con[gi, 1] * dx * dy
            alpha = torch.clamp(opac[gi] * torch.exp(power), max=0.99)
            with torch.no_grad():
                valid = (~done) & (power <= 0) & (alpha >= 1.0 / 255.0)
                term = valid & (T * (1 - alpha) < 1e-4)
                acc = valid & ~term
                done = done | term
            w = torch.where(acc, alpha * T, torch.zeros_like(T))
            C = C + w[:, None] * col[gi][None, :]
            D = D + w * depth[gi]
            T = torch.where(acc, T * (1 - alpha), T)
        rows.append((yy.reshape(-1), xx.reshape(-1), C, D, T))
    for yy, xx, C, D, T in rows:
        color = color.index_put((torch.arange(3)[:, None], yy[None, :].expand(3, -1), xx[None, :].expand(3, -1)),
                                (C + T[:, None] * bg[None, :]).T)
        out_d = out_d.index_put((torch.zeros_like(yy), yy, xx), D)
        out_a = out_a.index_put((torch.zeros_like(yy), yy, xx), 1 - T)
    return color, out_d, out_a
