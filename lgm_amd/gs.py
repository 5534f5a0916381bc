"""Drop-in GaussianRenderer (core/gs.py:16-190) on the MI355X-native render path.

Same constructor (reads opt.fovy/znear/zfar at construction like core/gs.py:19-29 and opt.output_size at EVERY
render call like core/gs.py:59-60,92-93, because convert.py:188,265,366 mutate it), same `render` signature and
returned keys ("image" clamped to [0,1] as core/gs.py:87, "alpha"), plus an additive "depth" key, and the same
save_ply / load_ply. The B x V python loop of core/gs.py:42-90 and its B*V per-view extension calls (each with a
device->host sync) are replaced by ONE batched C-ABI call (include/lgm_render.h) per forward and per backward.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import _native
from .ply import read_ply, write_ply

# Slot-mode (sync-free, worst-case B*V*T*N pair slots) workspace when it fits; otherwise the pairs are counted
# exactly first (one host sync per batch -- the reference syncs once per VIEW for num_rendered). The slot workspace
# costs address space, not traffic (only the used part of each tile bucket is touched), but it is held from the
# forward to the backward: up to _WS_FREE_SLOT bytes it is taken without asking (cfg3 needs 1.2 GB, the 8-scene
# pool 9.8 GB); above, only if it fits half of the memory torch could still hand out (free device memory plus
# torch's cached-but-unused blocks) -- LGM 'big' with 20 views at 512^2 needs 25 GB, a 64-view training batch at
# 512^2 34 GB: taken on an idle 288 GB MI355X, counted exactly next to a large model. LGM_AMD_WS_BUDGET_GB fixes
# the limit instead.
_WS_BUDGET = int(float(os.environ["LGM_AMD_WS_BUDGET_GB"]) * (1 << 30)) if "LGM_AMD_WS_BUDGET_GB" in os.environ \
    else None
_WS_FREE_SLOT = 16 << 30


def _slot_fits(ws_bytes: int, dev) -> bool:
    if _WS_BUDGET is not None:
        return ws_bytes <= _WS_BUDGET
    if ws_bytes <= _WS_FREE_SLOT:
        return True
    free, _ = torch.cuda.mem_get_info(dev)
    avail = free + torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)
    return ws_bytes <= avail // 2


def _tiles(H: int, W: int) -> int:
    return ((W + 15) // 16) * ((H + 15) // 16)


class _RasterizeBatched(torch.autograd.Function):
    """Autograd Function over all B x V renders (replaces B*V applications of the EXT _RasterizeGaussians)."""

    @staticmethod
    def forward(ctx, g, cam_view, cam_view_proj, bg, tanx, tany, scale_modifier, H, W, options, gt_img=None,
                gt_mask=None):
        L = _native.lib()
        B, N = g.shape[0], g.shape[1]
        V = cam_view.shape[1]
        dev = g.device
        stream = _native.stream_of(dev)
        cap = 0
        ws_bytes = L.lgm_render_workspace_size_opts(B, V, N, H, W, 0, options)
        if not _slot_fits(ws_bytes, dev):
            # exact pair count (the reference syncs once per view for this; we sync once per batch)
            small = L.lgm_render_workspace_size(B, V, N, H, W, 1)
            ws = torch.empty(small, dtype=torch.uint8, device=dev)
            k = torch.zeros(2, dtype=torch.int64, device=dev)
            _native.check(L.lgm_render_count_pairs(B, V, N, H, W, _native.ptr(g), _native.ptr(cam_view),
                                                   _native.ptr(cam_view_proj), tanx, tany, scale_modifier,
                                                   _native.ptr(ws), small, _native.ptr(k), stream, _native.diag()),
                          "lgm_render_count_pairs")
            # pairs actually binned (upstream's full count with LGM_RENDER_NO_CULL)
            cap = max(int(k[1 if options & _native.RENDER_NO_CULL else 0].item()), 1)
            ws_bytes = L.lgm_render_workspace_size_opts(B, V, N, H, W, cap, options)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        image = torch.empty(B, V, 3, H, W, dtype=torch.float32, device=dev)
        depth = torch.empty(B, V, 1, H, W, dtype=torch.float32, device=dev)
        alpha = torch.empty(B, V, 1, H, W, dtype=torch.float32, device=dev)
        if gt_img is None:
            loss4 = torch.empty(0, dtype=torch.float32, device=dev)
            _native.check(L.lgm_render_forward(B, V, N, H, W, _native.ptr(g), _native.ptr(cam_view),
                                               _native.ptr(cam_view_proj), _native.ptr(bg), tanx, tany, scale_modifier,
                                               _native.ptr(image), _native.ptr(depth), _native.ptr(alpha), None,
                                               _native.ptr(ws), ws_bytes, cap, None, options, stream,
                                               _native.diag()),
                          "lgm_render_forward")
        else:
            # (loss_mse, mse_image, mse_alpha, psnr) of core/models.py:145-148,167, computed by the kernels
            loss4 = torch.empty(4, dtype=torch.float32, device=dev)
            _native.check(L.lgm_render_forward_loss(B, V, N, H, W, _native.ptr(g), _native.ptr(cam_view),
                                                    _native.ptr(cam_view_proj), _native.ptr(bg), tanx, tany,
                                                    scale_modifier, _native.ptr(image), _native.ptr(depth),
                                                    _native.ptr(alpha), _native.ptr(gt_img), _native.ptr(gt_mask),
                                                    _native.ptr(loss4), _native.ptr(ws), ws_bytes, cap, options,
                                                    stream, _native.diag()), "lgm_render_forward_loss")
        # the workspace is saved like an input: autograd frees it after a (non-retain_graph) backward, so a training
        # loop that keeps the previous step's outputs alive does not hold two workspaces
        ctx.save_for_backward(g, cam_view, cam_view_proj, bg, ws, gt_img, gt_mask, loss4)
        ctx.set_materialize_grads(False)  # unused outputs (LGM never uses depth) arrive as None, not zeros
        ctx.ws_bytes, ctx.cap = ws_bytes, cap
        ctx.params = (tanx, tany, scale_modifier, H, W, options)
        ctx.backwards = 0  # a repeated backward (retain_graph) must clear the previous one's accumulators
        return image, depth, alpha, loss4

    @staticmethod
    def backward(ctx, d_image, d_depth, d_alpha, d_loss4):
        g, cam_view, cam_view_proj, bg, ws, gt_img, gt_mask, loss4 = ctx.saved_tensors
        tanx, tany, scale_modifier, H, W, options = ctx.params
        B, N = g.shape[0], g.shape[1]
        V = cam_view.shape[1]
        d_image = None if d_image is None else d_image.float().contiguous()
        d_depth = None if d_depth is None else d_depth.float().contiguous()
        d_alpha = None if d_alpha is None else d_alpha.float().contiguous()
        d_g = torch.empty_like(g)
        L = _native.lib()
        bwd_options = options | (_native.RENDER_BACKWARD_AGAIN if ctx.backwards else 0)
        ctx.backwards += 1
        stream = _native.stream_of(g.device)
        if gt_img is not None and d_loss4 is not None:
            if d_depth is not None:
                raise NotImplementedError("a depth gradient together with the fused loss (LGM's loss has no depth)")
            # d/dmse_image of loss_mse, mse_image and psnr = -10 log10(mse_image); d/dmse_alpha of loss_mse, mse_alpha
            d4 = d_loss4.float()
            # the PSNR term only where psnr is actually differentiated (GaussianRenderer.render detaches it, as the
            # reference computes it under no_grad): an exact fit (mse_image == 0) must not turn 0 / 0 into NaN
            d_psnr = torch.where(d4[3] != 0, d4[3] * (10.0 / math.log(10.0)) / loss4[1], torch.zeros_like(d4[3]))
            s2 = torch.stack([d4[0] + d4[1] - d_psnr, d4[0] + d4[2]]).contiguous()
            _native.check(L.lgm_render_backward_loss(B, V, N, H, W, _native.ptr(g), _native.ptr(cam_view),
                                                     _native.ptr(cam_view_proj), _native.ptr(bg), tanx, tany,
                                                     scale_modifier, _native.ptr(d_image), _native.ptr(d_alpha),
                                                     _native.ptr(gt_img), _native.ptr(gt_mask), _native.ptr(s2),
                                                     _native.ptr(d_g), _native.ptr(ws), ctx.ws_bytes, ctx.cap,
                                                     bwd_options, stream, _native.diag()), "lgm_render_backward_loss")
        else:
            _native.check(L.lgm_render_backward(B, V, N, H, W, _native.ptr(g), _native.ptr(cam_view),
                                                _native.ptr(cam_view_proj), _native.ptr(bg), tanx, tany, scale_modifier,
                                                _native.ptr(d_image), _native.ptr(d_depth), _native.ptr(d_alpha),
                                                _native.ptr(d_g), None, _native.ptr(ws), ctx.ws_bytes, ctx.cap,
                                                bwd_options, stream, _native.diag()), "lgm_render_backward")
        return d_g, None, None, None, None, None, None, None, None, None, None, None


def deterministic_enabled() -> bool:
    """Bit-reproducible render gradients (LGM_RENDER_DETERMINISTIC) when torch's deterministic algorithms are on
    (torch.use_deterministic_algorithms(True)) or LGM_AMD_DETERMINISTIC=1."""
    return torch.are_deterministic_algorithms_enabled() or os.environ.get("LGM_AMD_DETERMINISTIC", "0") == "1"


def rasterize(gaussians, cam_view, cam_view_proj, bg, tanfovx, tanfovy, H, W, scale_modifier=1.0, clamp=False,
              gt_images=None, gt_masks=None, deterministic=None, no_cull=False):
    """Functional form: returns (image [B,V,3,H,W], depth [B,V,1,H,W], alpha [B,V,1,H,W]). The image is
    unclamped unless clamp=True, which applies core/gs.py:87's clamp(0, 1) (and its gradient) inside the kernels.
    With gt_images [B,V,3,H,W] and gt_masks [B,V,1,H,W] a 4th output (loss_mse, mse_image, mse_alpha, psnr) holds
    LGM's training MSE terms (core/models.py:145-148,167), fused into the kernels; it is differentiable.
    no_cull=True bins upstream's full 3-sigma tile rects (LGM_RENDER_NO_CULL: same outputs, more work)."""
    if not gaussians.is_cuda:  # CPU tensors: the torch path of BASELINE config 1 (lgm_amd/cpu.py), never the oracle
        from .cpu import render_cpu
        bgc = torch.as_tensor(bg, dtype=torch.float32).detach().cpu()
        out = render_cpu(gaussians, cam_view.cpu(), cam_view_proj.cpu(), bgc, tanfovx, tanfovy, int(H), int(W),
                         scale_modifier, clamp=clamp)
        if gt_images is None and gt_masks is None:
            return out
        gt_c = gt_images * gt_masks + bgc.view(1, 1, 3, 1, 1) * (1 - gt_masks)  # core/models.py:145
        mi, ma = torch.nn.functional.mse_loss(out[0], gt_c), torch.nn.functional.mse_loss(out[2], gt_masks)
        return out + (torch.stack([mi + ma, mi, ma, -10 * torch.log10(mi)]),)
    for t, n in ((gaussians, "gaussians"), (cam_view, "cam_view"), (cam_view_proj, "cam_view_proj")):
        _native.require_device_tensor(t, n)
    g = gaussians.float().contiguous()
    dev = g.device
    cv = cam_view.to(dev, torch.float32).contiguous()
    cvp = cam_view_proj.to(dev, torch.float32).contiguous()
    bgt = torch.as_tensor(bg, dtype=torch.float32).to(dev).contiguous().detach()
    if g.dim() != 3 or g.shape[-1] != 14:
        raise ValueError(f"gaussians must be [B,N,14], got {tuple(g.shape)}")
    if cv.shape[:2] != cvp.shape[:2] or cv.shape[0] != g.shape[0] or cv.shape[-2:] != (4, 4):
        raise ValueError("cam_view / cam_view_proj must be [B,V,4,4] with B matching gaussians")
    gti = gtm = None
    if gt_images is not None or gt_masks is not None:
        B, V = cv.shape[0], cv.shape[1]
        gti = gt_images.to(dev, torch.float32).contiguous().detach()
        gtm = gt_masks.to(dev, torch.float32).contiguous().detach()
        if tuple(gti.shape) != (B, V, 3, H, W) or tuple(gtm.shape) != (B, V, 1, H, W):
            raise ValueError("gt_images / gt_masks must be [B,V,3,H,W] / [B,V,1,H,W]")
    options = (_native.RENDER_CLAMP_IMAGE if clamp else 0) | (_native.RENDER_NO_CULL if no_cull else 0)
    if deterministic_enabled() if deterministic is None else deterministic:
        options |= _native.RENDER_DETERMINISTIC
    out = _RasterizeBatched.apply(g, cv, cvp, bgt, float(tanfovx), float(tanfovy), float(scale_modifier),
                                  int(H), int(W), options, gti, gtm)
    return out if gti is not None else out[:3]


def count_pairs(gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, H, W, scale_modifier=1.0):
    """(binned, reference) (Gaussian, tile) pair counts over all B x V views (one host sync): `binned` after the
    exact opacity-aware tile culling, `reference` = upstream's num_rendered summed over views (SURVEY §8(d)'s K)."""
    L = _native.lib()
    g = gaussians.float().contiguous()
    B, N, V = g.shape[0], g.shape[1], cam_view.shape[1]
    dev = g.device
    small = L.lgm_render_workspace_size(B, V, N, H, W, 1)
    ws = torch.empty(small, dtype=torch.uint8, device=dev)
    k = torch.zeros(2, dtype=torch.int64, device=dev)
    cv = cam_view.to(dev, torch.float32).contiguous()
    cvp = cam_view_proj.to(dev, torch.float32).contiguous()
    _native.check(L.lgm_render_count_pairs(B, V, N, H, W, _native.ptr(g), _native.ptr(cv), _native.ptr(cvp),
                                           float(tanfovx), float(tanfovy), float(scale_modifier), _native.ptr(ws),
                                           small, _native.ptr(k), _native.stream_of(dev), _native.diag()),
                  "lgm_render_count_pairs")
    kk = k.tolist()
    return int(kk[0]), int(kk[1])


def forward_state(gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, H, W, scale_modifier=1.0, lists=False,
                  no_cull=False, records=False):
    """Runs one forward and returns what it left in its workspace (numpy, one host sync), for parity tests and
    debugging -- the equivalent of reading upstream's saved buffers (radii, point_list/ranges, n_contrib):
      radii [B,V,N] int32; K_binned / K_reference (as count_pairs); tile_counts [B,V,T] int32;
      n_contrib, final_T [B,V,H,W]; with lists=True, ids[b][v] = the view's tile lists concatenated (tile-major,
      each in compositing order); with records=True, the compositing records P, Q [B,V,N,4] and rects [B,V,N,2]
      (uint32) of lgm_render_records. no_cull=True bins upstream's full 3-sigma rects (LGM_RENDER_NO_CULL)."""
    options = _native.RENDER_NO_CULL if no_cull else 0
    L = _native.lib()
    g = gaussians.float().contiguous()
    dev = g.device
    B, N, V = g.shape[0], g.shape[1], cam_view.shape[1]
    cv = cam_view.to(dev, torch.float32).contiguous()
    cvp = cam_view_proj.to(dev, torch.float32).contiguous()
    stream = _native.stream_of(dev)
    ws_bytes = L.lgm_render_workspace_size(B, V, N, H, W, 0)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    bg = torch.zeros(3, device=dev)
    image = torch.empty(B, V, 3, H, W, device=dev)
    depth = torch.empty(B, V, 1, H, W, device=dev)
    alpha = torch.empty(B, V, 1, H, W, device=dev)
    radii = torch.empty(B, V, N, dtype=torch.int32, device=dev)
    stats = torch.zeros(2, dtype=torch.int64, device=dev)
    _native.check(L.lgm_render_forward(B, V, N, H, W, _native.ptr(g), _native.ptr(cv), _native.ptr(cvp),
                                       _native.ptr(bg), float(tanfovx), float(tanfovy), float(scale_modifier),
                                       _native.ptr(image), _native.ptr(depth), _native.ptr(alpha), _native.ptr(radii),
                                       _native.ptr(ws), ws_bytes, 0, _native.ptr(stats), options, stream,
                                       _native.diag()),
                  "lgm_render_forward")
    T = _tiles(H, W)
    counts = torch.empty(B * V * T, dtype=torch.int32, device=dev)
    _native.check(L.lgm_render_tile_lists(B, V, N, H, W, _native.ptr(ws), ws_bytes, 0, _native.ptr(counts), None,
                                          None, stream), "lgm_render_tile_lists")
    n_contrib = torch.empty(B, V, H, W, dtype=torch.int32, device=dev)
    final_T = torch.empty(B, V, H, W, dtype=torch.float32, device=dev)
    _native.check(L.lgm_render_pixel_state(B, V, N, H, W, _native.ptr(ws), ws_bytes, 0, _native.ptr(n_contrib),
                                           _native.ptr(final_T), stream), "lgm_render_pixel_state")
    out = {"radii": radii.cpu().numpy(), "tile_counts": counts.view(B, V, T).cpu().numpy(),
           "n_contrib": n_contrib.cpu().numpy(), "final_T": final_T.cpu().numpy()}
    k = stats.tolist()
    out["K_binned"], out["K_reference"] = int(k[0]), int(k[1])
    if lists:
        c64 = counts.to(torch.int64)
        offsets = (torch.cumsum(c64, 0) - c64).contiguous()
        total = int(c64.sum().item())
        ids = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        _native.check(L.lgm_render_tile_lists(B, V, N, H, W, _native.ptr(ws), ws_bytes, 0, _native.ptr(counts),
                                              _native.ptr(offsets), _native.ptr(ids), stream), "lgm_render_tile_lists")
        flat = ids[:total].cpu().numpy()
        per_view = c64.view(B * V, T).sum(1).tolist()
        bounds = np.concatenate([[0], np.cumsum(per_view)])
        out["ids"] = [[flat[bounds[b * V + v]:bounds[b * V + v + 1]] for v in range(V)] for b in range(B)]
    if records:
        P = torch.empty(B, V, N, 4, device=dev)
        Q = torch.empty(B, V, N, 4, device=dev)
        rects = torch.empty(B, V, N, 2, dtype=torch.int32, device=dev)
        _native.check(L.lgm_render_records(B, V, N, H, W, _native.ptr(ws), ws_bytes, 0, _native.ptr(P), _native.ptr(Q),
                                           _native.ptr(rects), stream), "lgm_render_records")
        out["P"], out["Q"] = P.cpu().numpy(), Q.cpu().numpy()
        out["rects"] = rects.cpu().numpy().view(np.uint32)
    return out


class GaussianRenderer:
    """core/gs.py:16 GaussianRenderer, same API."""

    def __init__(self, opt):
        self.opt = opt
        # core/gs.py:20 creates this on "cuda"; here it follows the Gaussians' device at render time.
        self.bg_color = torch.tensor([1, 1, 1], dtype=torch.float32,
                                     device="cuda" if torch.cuda.is_available() else "cpu")
        self.tan_half_fov = np.tan(0.5 * np.deg2rad(self.opt.fovy))
        self.proj_matrix = torch.zeros(4, 4, dtype=torch.float32)
        self.proj_matrix[0, 0] = 1 / self.tan_half_fov
        self.proj_matrix[1, 1] = 1 / self.tan_half_fov
        self.proj_matrix[2, 2] = (opt.zfar + opt.znear) / (opt.zfar - opt.znear)
        self.proj_matrix[3, 2] = -(opt.zfar * opt.znear) / (opt.zfar - opt.znear)
        self.proj_matrix[2, 3] = 1

    def render(self, gaussians, cam_view, cam_view_proj, cam_pos, bg_color=None, scale_modifier=1, gt_images=None,
               gt_masks=None):
        """core/gs.py:31-98. gaussians [B,N,14]; cam_view, cam_view_proj [B,V,4,4]; cam_pos [B,V,3] (unused without
        SH, as upstream). Additive: with gt_images / gt_masks (the `images_output` / `masks_output` of
        core/models.py:140-141) the result also holds LGM's MSE loss terms, computed in the render kernels:
        "loss_mse" (differentiable: its backward seeds the render backward in-kernel), "mse_image", "mse_alpha"
        and "psnr" (core/models.py:145-148,165-167)."""
        S = int(self.opt.output_size)
        bg = self.bg_color if bg_color is None else bg_color
        tan = float(self.tan_half_fov)
        # core/gs.py:87's clamp(0, 1) and its gradient are applied inside the kernels
        out = rasterize(gaussians, cam_view, cam_view_proj, bg, tan, tan, S, S, scale_modifier, clamp=True,
                        gt_images=gt_images, gt_masks=gt_masks)
        res = {"image": out[0], "alpha": out[2], "depth": out[1]}
        if len(out) == 4:
            loss4 = out[3]
            res.update(loss_mse=loss4[0], mse_image=loss4[1], mse_alpha=loss4[2], psnr=loss4[3].detach())
        return res

    def save_ply(self, gaussians, path, compatible=True):
        """core/gs.py:101-152: B == 1, prune opacity < 0.005, optionally invert activations (3DGS PLY layout)."""
        assert gaussians.shape[0] == 1, "only support batch size 1"
        g = gaussians[0].detach().float().cpu()
        means3D, opacity, scales, rotations = g[:, 0:3], g[:, 3:4], g[:, 4:7], g[:, 7:11]
        shs = g[:, 11:].unsqueeze(1)
        mask = opacity.squeeze(-1) >= 0.005
        means3D, opacity, scales, rotations, shs = means3D[mask], opacity[mask], scales[mask], rotations[mask], shs[mask]
        if compatible:
            o = opacity.clamp(1e-6, 1 - 1e-6)
            opacity = torch.log(o / (1 - o))  # kiui.op.inverse_sigmoid
            scales = torch.log(scales + 1e-8)
            shs = (shs - 0.5) / 0.28209479177387814
        f_dc = shs.transpose(1, 2).flatten(start_dim=1).contiguous()
        names = ["x", "y", "z"] + [f"f_dc_{i}" for i in range(f_dc.shape[1])] + ["opacity"] + \
                [f"scale_{i}" for i in range(scales.shape[1])] + [f"rot_{i}" for i in range(rotations.shape[1])]
        data = torch.cat([means3D, f_dc, opacity, scales, rotations], dim=1).numpy().astype(np.float32)
        write_ply(path, names, data)

    def load_ply(self, path, compatible=True):
        """core/gs.py:154-190: returns a CPU [N,14] tensor."""
        props = read_ply(path)
        xyz = np.stack([props["x"], props["y"], props["z"]], axis=1)
        print("Number of points at loading : ", xyz.shape[0])
        opac = props["opacity"][:, None]
        shs = np.stack([props["f_dc_0"], props["f_dc_1"], props["f_dc_2"]], axis=1)
        sn = sorted([k for k in props if k.startswith("scale_")], key=lambda s: int(s.split("_")[-1]))
        rn = sorted([k for k in props if k.startswith("rot_")], key=lambda s: int(s.split("_")[-1]))
        scales = np.stack([props[k] for k in sn], axis=1)
        rots = np.stack([props[k] for k in rn], axis=1)
        gaussians = torch.from_numpy(np.concatenate([xyz, opac, scales, rots, shs], axis=1).astype(np.float64)).float()
        if compatible:
            gaussians[..., 3:4] = torch.sigmoid(gaussians[..., 3:4])
            gaussians[..., 4:7] = torch.exp(gaussians[..., 4:7])
            gaussians[..., 11:] = 0.28209479177387814 * gaussians[..., 11:] + 0.5
        return gaussians


def tan_half_fov(fovy: float) -> float:
    return math.tan(0.5 * math.radians(fovy))
