"""CPU (PyTorch) path of the render and attention ops, for CPU tensors only -- BASELINE config 1: `infer.py` 'big'
run CPU-only (infer.py:43-47,102-145). The reference cannot do this at all (core/gs.py:20 puts bg on "cuda"; the
rasterizer extension is CUDA-only). This is product code, vectorised torch on the host, separate from the oracle
(oracle/raster_oracle.c, test infrastructure) and parity-tested against it (tests/test_cpu_path.py). GPU tensors
never come here: on a GPU the HIP kernels run, and a missing library raises (lgm_amd/_native.py).

render_cpu follows the upstream algorithm of SURVEY.md §2.3 step by step:
  * preprocess per Gaussian (near cull 0.2, cov3D from the un-normalised quaternion, EWA cov2D with the 1.3 tan-fov
    clamp and 0.3 dilation, 3-sigma radius, ndc2Pix, tile rect);
  * (tile, depth) keys emitted in Gaussian order and sorted stably (ties keep increasing Gaussian id);
  * per tile, front-to-back compositing of its list over its 256 pixels, vectorised over pixels and list chunks:
    alpha = min(0.99, o exp(power)), skipped when power > 0 or alpha < 1/255; a pixel stops at the first accepted
    entry whose T (1 - alpha) would fall below 1e-4 (that entry excluded), exactly the sequential rule, via
    cumulative products of (1 - alpha) along the list.
It is written in differentiable torch ops: autograd gives the backward (the alpha skip / stop decisions are
piecewise-constant masks, as in the reference's backward; the 0.99 alpha cap passes the gradient of o G through, as
upstream's backward does).
"""
from __future__ import annotations

import torch

BLOCK = 16
CHUNK = 512  # list entries composited per step (bounds the [entries x 256 pixels] temporaries)


def _tf(M: torch.Tensor, p: torch.Tensor, rows: int) -> torch.Tensor:
    """The column-major read of a row-major torch 4x4 (core/gs.py:54-55): o[k] = sum_j M[j][k] p_j + M[3][k]."""
    return p @ M[:3, :rows] + M[3, :rows]


def _preprocess(g: torch.Tensor, view: torch.Tensor, proj: torch.Tensor, tanx: float, tany: float, H: int, W: int,
                mod: float):
    f32 = torch.float32
    mean = g[:, 0:3]
    hom = _tf(proj, mean, 4)
    pw = 1.0 / (hom[:, 3] + 0.0000001)
    ppx, ppy = hom[:, 0] * pw, hom[:, 1] * pw
    pv = _tf(view, mean, 3)
    depth = pv[:, 2]
    # cov3D = M^T M, M = S R (glm), un-normalised quaternion (r, x, y, z)
    s = mod * g[:, 4:7]
    r, x, y, z = g[:, 7], g[:, 8], g[:, 9], g[:, 10]
    R = torch.stack([
        torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y)], -1),
        torch.stack([2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x)], -1),
        torch.stack([2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1)], 1)  # R[c][k]
    Mm = R * s[:, None, :]  # M[c][k] = s_k R[c][k]
    Sig = Mm @ Mm.transpose(1, 2)  # Sigma[c][r] = sum_k M[c][k] M[r][k]
    # J with the 1.3 tan-fov clamp on the view-space mean; T = W J (its two non-zero glm columns)
    limx, limy = 1.3 * tanx, 1.3 * tany
    tz = pv[:, 2]
    txtz, tytz = pv[:, 0] / tz, pv[:, 1] / tz
    tx_v, ty_v = txtz.clamp(-limx, limx) * tz, tytz.clamp(-limy, limy) * tz
    # upstream's backward: the clamped t.x (t.y) carries no gradient (x_grad_mul), the unclamped one passes it to the
    # view-space mean only (no chain through t.z); the values are the forward's clamp(t.x / t.z) * t.z
    cx, cy = (txtz < -limx) | (txtz > limx), (tytz < -limy) | (tytz > limy)
    tx = torch.where(cx, tx_v.detach(), pv[:, 0] + (tx_v - pv[:, 0]).detach())
    ty = torch.where(cy, ty_v.detach(), pv[:, 1] + (ty_v - pv[:, 1]).detach())
    fx, fy = W / (2.0 * tanx), H / (2.0 * tany)
    J00, J02 = fx / tz, -(fx * tx) / (tz * tz)
    J11, J12 = fy / tz, -(fy * ty) / (tz * tz)
    Vw = view[:3, :3]  # Vw[r][k]: row r of the torch matrix = glm column
    T0 = Vw[:, 0][None, :] * J00[:, None] + Vw[:, 2][None, :] * J02[:, None]  # T0[r] = view[4r] J00 + view[4r+2] J02
    T1 = Vw[:, 1][None, :] * J11[:, None] + Vw[:, 2][None, :] * J12[:, None]
    s0 = (Sig @ T0[:, :, None])[:, :, 0]
    s1 = (Sig @ T1[:, :, None])[:, :, 0]
    a = (T0 * s0).sum(-1) + 0.3
    b = (T0 * s1).sum(-1)
    c = (T1 * s1).sum(-1) + 0.3
    det = a * c - b * b
    mid = 0.5 * (a + c)
    disc = torch.sqrt(torch.clamp(mid * mid - det, min=0.1))
    rad = torch.ceil(3.0 * torch.sqrt(torch.maximum(mid + disc, mid - disc)))
    px = ((ppx.double() + 1.0) * W - 1.0) * 0.5
    py = ((ppy.double() + 1.0) * H - 1.0) * 0.5
    px, py = px.to(f32), py.to(f32)
    gx, gy = (W + BLOCK - 1) // BLOCK, (H + BLOCK - 1) // BLOCK
    ri = rad.detach().to(torch.int64)
    pxd, pyd = px.detach(), py.detach()
    x0 = ((pxd - ri) / BLOCK).to(torch.int64).clamp(0, gx)
    y0 = ((pyd - ri) / BLOCK).to(torch.int64).clamp(0, gy)
    x1 = ((pxd + ri + BLOCK - 1) / BLOCK).to(torch.int64).clamp(0, gx)
    y1 = ((pyd + ri + BLOCK - 1) / BLOCK).to(torch.int64).clamp(0, gy)
    vis = (depth.detach() > 0.2) & (det.detach() != 0) & ((x1 - x0) * (y1 - y0) > 0)
    inv = 1.0 / torch.where(det == 0, torch.ones_like(det), det)
    conic = torch.stack([c * inv, -b * inv, a * inv], -1)
    return {"px": px, "py": py, "depth": depth, "conic": conic, "vis": vis, "radii": torch.where(vis, ri, 0),
            "rect": torch.stack([x0, y0, x1, y1], -1), "gx": gx, "gy": gy}


def _tile_lists(pre):
    """Upstream's duplicateWithKeys + stable sort on (tile, depth bits): per-tile id lists in compositing order."""
    vis, rect, gx, gy = pre["vis"], pre["rect"], pre["gx"], pre["gy"]
    ids = torch.nonzero(vis).flatten()
    if ids.numel() == 0:
        return torch.zeros(gx * gy + 1, dtype=torch.int64), ids
    r = rect[ids]
    wdt, hgt = r[:, 2] - r[:, 0], r[:, 3] - r[:, 1]
    cnt = wdt * hgt
    gid = torch.repeat_interleave(ids, cnt)
    k = torch.arange(gid.numel()) - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt)
    w_rep, r_rep = torch.repeat_interleave(wdt, cnt), torch.repeat_interleave(r, cnt, dim=0)
    tile = (r_rep[:, 1] + k // w_rep) * gx + r_rep[:, 0] + k % w_rep
    dbits = pre["depth"].detach()[gid].contiguous().view(torch.int32).to(torch.int64)  # positive floats: monotone
    key = tile * (1 << 32) + dbits
    _, order = torch.sort(key, stable=True)  # emitted in Gaussian order: ties keep increasing id
    gid = gid[order]
    start = torch.zeros(gx * gy + 1, dtype=torch.int64)
    start[1:] = torch.cumsum(torch.bincount(tile, minlength=gx * gy), 0)
    return start, gid


def _composite_tile(pre, g, ids, tx, ty, H, W, bg):
    """Front-to-back compositing of one tile's list over its pixels; returns (color [3,P], depth [P], T [P],
    pixel index [P]) for the tile's in-image pixels."""
    ys, xs = torch.meshgrid(torch.arange(ty * BLOCK, min(H, ty * BLOCK + BLOCK)),
                            torch.arange(tx * BLOCK, min(W, tx * BLOCK + BLOCK)), indexing="ij")
    pfx, pfy = xs.flatten().float(), ys.flatten().float()
    P = pfx.numel()
    T = torch.ones(P)
    C = torch.zeros(3, P)
    D = torch.zeros(P)
    done = torch.zeros(P, dtype=torch.bool)
    for c0 in range(0, ids.numel(), CHUNK):
        if bool(done.all()):
            break
        sel = ids[c0:c0 + CHUNK]
        con = pre["conic"][sel]
        dx = pre["px"][sel][:, None] - pfx[None, :]
        dy = pre["py"][sel][:, None] - pfy[None, :]
        power = -0.5 * (con[:, 0:1] * dx * dx + con[:, 2:3] * dy * dy) - con[:, 1:2] * dx * dy
        # min(0.99, o G) with upstream's backward, which differentiates o G even where the cap is active
        og = g[sel, 3][:, None] * torch.exp(power)
        alpha = og + (torch.clamp(og, max=0.99) - og).detach()
        valid = (power <= 0) & (alpha >= 1.0 / 255.0)
        a_eff = torch.where(valid, alpha, torch.zeros_like(alpha))
        # T before / after each entry: the running product in the sequential order (T first, then each factor)
        prod = torch.cumprod(torch.cat([T[None, :], 1 - a_eff], 0), 0)
        Tex, Tin = prod[:-1], prod[1:]
        stop = valid & (Tin < 0.0001)
        first_stop = torch.cumsum(stop.int(), 0) > 0     # at or after the first stopping entry
        keep = valid & ~first_stop & ~done[None, :]
        wgt = torch.where(keep, a_eff * Tex, torch.zeros_like(a_eff))
        C = C + (g[sel, 11:14].T[:, :, None] * wgt[None]).sum(1)
        D = D + (pre["depth"][sel][:, None] * wgt).sum(0)
        # T of each pixel after this chunk: the product up to its last kept entry
        n_keep = keep.int().sum(0)
        lastT = torch.where(keep, Tin, torch.zeros_like(Tin))
        idx = torch.where(keep, torch.arange(sel.numel())[:, None].expand_as(keep), -1).amax(0)
        newT = torch.gather(lastT, 0, idx.clamp(min=0)[None, :])[0]
        T = torch.where(n_keep > 0, newT, T)
        done = done | first_stop.any(0)
    pid = (ys.flatten() * W + xs.flatten())
    return C, D, T, pid


def render_cpu(gaussians, cam_view, cam_view_proj, bg, tanx, tany, H, W, scale_modifier=1.0, clamp=False):
    """[B,N,14] CPU Gaussians -> (image [B,V,3,H,W], depth [B,V,1,H,W], alpha [B,V,1,H,W]); image clamped to
    [0, 1] when clamp (core/gs.py:87)."""
    g_all = gaussians.float()
    B, V = cam_view.shape[0], cam_view.shape[1]
    bgv = torch.as_tensor(bg, dtype=torch.float32).reshape(3)
    imgs, deps, alps = [], [], []
    for b in range(B):
        g = g_all[b]
        for v in range(V):
            pre = _preprocess(g, cam_view[b, v].float(), cam_view_proj[b, v].float(), tanx, tany, H, W,
                              float(scale_modifier))
            start, lst = _tile_lists(pre)
            color = torch.zeros(3, H * W)
            depth = torch.zeros(H * W)
            Tf = torch.ones(H * W)
            for t in range(pre["gx"] * pre["gy"]):
                ids = lst[int(start[t]):int(start[t + 1])]
                if ids.numel() == 0:
                    continue
                C, D, T, pid = _composite_tile(pre, g, ids, t % pre["gx"], t // pre["gx"], H, W, bgv)
                color = color.index_copy(1, pid, C)
                depth = depth.index_copy(0, pid, D)
                Tf = Tf.index_copy(0, pid, T)
            img = color + Tf[None, :] * bgv[:, None]
            imgs.append(img.reshape(3, H, W))
            deps.append(depth.reshape(1, H, W))
            alps.append((1 - Tf).reshape(1, H, W))
    image = torch.stack(imgs).reshape(B, V, 3, H, W)
    if clamp:
        image = image.clamp(0, 1)
    return image, torch.stack(deps).reshape(B, V, 1, H, W), torch.stack(alps).reshape(B, V, 1, H, W)


def attention_cpu(qkv: torch.Tensor, scale: float) -> torch.Tensor:
    """softmax(scale q k^T) v for packed qkv [B, L, 3, H, D] -> [B, L, H, D]: the reference's fallback
    Attention (core/attention.py:51-64: q scaled first, materialised logits), in the input dtype."""
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    attn = (q * scale) @ k.transpose(-2, -1)
    attn = attn.softmax(dim=-1)
    return (attn @ v).transpose(1, 2)


def gaussian_head_cpu(x, weight, bias, B: int, V: int):
    """core/models.py:96-117 in torch ops (the GPU runs lgm_amd/csrc/head.hip)."""
    import torch.nn.functional as F
    y = F.conv2d(x, weight, bias)
    _, C, h, w = y.shape
    y = y.reshape(B, V, C, h, w).permute(0, 1, 3, 4, 2).reshape(B, -1, C)
    return torch.cat([y[..., 0:3].clamp(-1, 1), torch.sigmoid(y[..., 3:4]), 0.1 * F.softplus(y[..., 4:7]),
                      F.normalize(y[..., 7:11]), 0.5 * torch.tanh(y[..., 11:]) + 0.5], dim=-1)


__all__ = ["render_cpu", "attention_cpu", "gaussian_head_cpu"]
