"""Camera construction used by every caller of the renderer.

Restates the recipe of core/provider_lvis.py:200-213 (also infer.py:135-142, gui.py:67-73, convert.py:108-114):
OpenGL c2w -> flip up/forward columns -> cam_view = inverse(c2w)^T -> cam_view_proj = cam_view @ proj -> cam_pos = -c2w[:3, 3].
The look-at convention restates kiui.cam.orbit_camera / look_at (EXT, `kiui` is not installed here),
as called by core/models.py:66-71 and infer.py:135.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _normalize(v: np.ndarray) -> np.ndarray:
    return v / max(float(np.linalg.norm(v)), 1e-20)


def look_at(campos: np.ndarray, target: np.ndarray, opengl: bool = True) -> np.ndarray:
    """3x3 camera rotation (columns right, up, forward); kiui.cam.look_at semantics."""
    up = np.array([0, 1, 0], dtype=np.float32)
    if not opengl:
        fwd = _normalize(target - campos)
        right = _normalize(np.cross(fwd, up))
        up = _normalize(np.cross(right, fwd))
    else:
        fwd = _normalize(campos - target)
        right = _normalize(np.cross(up, fwd))
        up = _normalize(np.cross(fwd, right))
    return np.stack([right, up, fwd], axis=1)


def orbit_camera(elevation: float, azimuth: float, radius: float = 1.0, is_degree: bool = True,
                 target=None, opengl: bool = True) -> np.ndarray:
    """[4,4] float32 c2w pose on an orbit (kiui.cam.orbit_camera semantics)."""
    if is_degree:
        elevation = np.deg2rad(elevation)
        azimuth = np.deg2rad(azimuth)
    x = radius * np.cos(elevation) * np.sin(azimuth)
    y = -radius * np.sin(elevation)
    z = radius * np.cos(elevation) * np.cos(azimuth)
    if target is None:
        target = np.zeros([3], dtype=np.float32)
    campos = np.array([x, y, z]) + target
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = look_at(campos, target, opengl)
    T[:3, 3] = campos
    return T


def projection_matrix(fovy: float, znear: float, zfar: float) -> torch.Tensor:
    """The [4,4] proj of core/gs.py:23-29 / core/provider_lvis.py:59-65 (row-major torch layout)."""
    tan_half_fov = np.tan(0.5 * np.deg2rad(fovy))
    P = torch.zeros(4, 4, dtype=torch.float32)
    P[0, 0] = 1 / tan_half_fov
    P[1, 1] = 1 / tan_half_fov
    P[2, 2] = (zfar + znear) / (zfar - znear)
    P[3, 2] = -(zfar * znear) / (zfar - znear)
    P[2, 3] = 1
    return P


def cameras_from_c2w(c2w: torch.Tensor, proj: torch.Tensor):
    """c2w [V,4,4] OpenGL poses -> (cam_view [V,4,4], cam_view_proj [V,4,4], cam_pos [V,3]) per
    core/provider_lvis.py:200-213."""
    c2w = c2w.clone().float()
    c2w[:, :3, 1:3] *= -1
    cam_view = torch.inverse(c2w).transpose(1, 2)
    cam_view_proj = cam_view @ proj
    cam_pos = -c2w[:, :3, 3]
    return cam_view, cam_view_proj, cam_pos


def orbit_cameras(num_views: int, radius: float = 1.5, elevation: float = 0.0, fovy: float = 49.1,
                  znear: float = 0.5, zfar: float = 2.5, azimuth_offset: float = 0.0):
    """V evenly spaced orbit cameras (SURVEY.md §8(d) synthetic cameras): returns cam_view, cam_view_proj,
    cam_pos as [V,4,4], [V,4,4], [V,3] float32 CPU tensors."""
    poses = np.stack([orbit_camera(elevation, azimuth_offset + 360.0 * v / num_views, radius=radius)
                      for v in range(num_views)], axis=0)
    return cameras_from_c2w(torch.from_numpy(poses), projection_matrix(fovy, znear, zfar))


def tan_half_fov(fovy: float) -> float:
    return float(math.tan(0.5 * math.radians(fovy)))


def get_rays(pose: torch.Tensor, h: int, w: int, fovy: float, opengl: bool = True):
    """Per-pixel ray origins and unit directions [h, w, 3] of a c2w pose (core/utils.py:10-43; kiui's
    safe_normalize: x / sqrt(max(x.x, 1e-20)))."""
    x, y = torch.meshgrid(torch.arange(w, device=pose.device), torch.arange(h, device=pose.device), indexing="xy")
    x, y = x.flatten(), y.flatten()
    focal = h * 0.5 / np.tan(0.5 * np.deg2rad(fovy))
    sgn = -1.0 if opengl else 1.0
    dirs = torch.stack([(x - w * 0.5 + 0.5) / focal, (y - h * 0.5 + 0.5) / focal * sgn,
                        torch.full_like(x, sgn, dtype=torch.float32)], -1).float()
    rays_d = dirs @ pose[:3, :3].transpose(0, 1)
    rays_o = pose[:3, 3].unsqueeze(0).expand_as(rays_d)
    rays_d = rays_d / torch.sqrt(torch.clamp((rays_d * rays_d).sum(-1, keepdim=True), min=1e-20))
    return rays_o.reshape(h, w, 3), rays_d.reshape(h, w, 3)


def default_rays(input_size: int, fovy: float = 49.1, radius: float = 1.5, elevation: float = 0.0, device=None):
    """LGM.prepare_default_rays (core/models.py:61-85): the Pluecker ray embeddings [4, 6, h, w] (cross(o, d), d)
    of the 4 input views at azimuths 0 / 90 / 180 / 270."""
    out = []
    for az in (0, 90, 180, 270):
        pose = torch.from_numpy(orbit_camera(elevation, az, radius=radius))
        o, d = get_rays(pose, input_size, input_size, fovy)
        out.append(torch.cat([torch.cross(o, d, dim=-1), d], dim=-1))
    return torch.stack(out, 0).permute(0, 3, 1, 2).contiguous().to(device)


def orbit_cameras_batched(elevation, azimuth, radius: float = 1.5, fovy: float = 49.1, znear: float = 0.5,
                          zfar: float = 2.5, device=None):
    """Device-side batched camera build for the orbit video loops of infer.py:132-145 / app.py:
    elevation and azimuth (degrees; scalars or [V] tensors, broadcast) -> (cam_view [V,4,4], cam_view_proj [V,4,4],
    cam_pos [V,3]) on `device`, in one set of vectorised torch ops instead of V numpy orbit_camera calls, V
    host->device copies and V torch.inverse calls. Same conventions as orbit_camera + cameras_from_c2w (OpenGL
    look-at, up/forward flipped, cam_view = inverse(c2w)^T).

    Precision: the pose is formed in float64 and rounded to float32, as orbit_camera does (numpy float64 into a
    float32 matrix); its inverse is then evaluated in float64 (adjugate of the 3x3 block, exact for the pose as
    rounded) and rounded once, and likewise cam_view @ proj. So every matrix is the correctly rounded value of the
    reference recipe's exact result, where torch.inverse / @ in float32 carry a few ulps of their own rounding."""
    f64 = torch.float64
    el = torch.as_tensor(elevation, dtype=f64, device=device)
    az = torch.as_tensor(azimuth, dtype=f64, device=device)
    el, az = torch.broadcast_tensors(el.reshape(-1), az.reshape(-1))
    el, az = torch.deg2rad(el), torch.deg2rad(az)
    campos = torch.stack([radius * torch.cos(el) * torch.sin(az), -radius * torch.sin(el),
                          radius * torch.cos(el) * torch.cos(az)], -1)  # [V, 3], target at the origin
    up = torch.tensor([0.0, 1.0, 0.0], dtype=f64, device=campos.device).expand_as(campos)
    fwd = torch.nn.functional.normalize(campos, dim=-1, eps=1e-20)
    right = torch.nn.functional.normalize(torch.cross(up, fwd, dim=-1), dim=-1, eps=1e-20)
    upv = torch.nn.functional.normalize(torch.cross(fwd, right, dim=-1), dim=-1, eps=1e-20)
    # the float32 c2w of orbit_camera, up and forward flipped (core/provider_lvis.py:205): exact sign flips
    R = torch.stack([right, -upv, -fwd], -1).float().double()
    t = campos.float().double()
    # inverse of [R t; 0 1] = [R^-1, -R^-1 t]: R^-1 = adj(R) / det(R) in float64
    c0, c1, c2 = R[:, :, 0], R[:, :, 1], R[:, :, 2]
    adj_rows = torch.stack([torch.cross(c1, c2, dim=-1), torch.cross(c2, c0, dim=-1), torch.cross(c0, c1, dim=-1)], 1)
    det = (c0 * adj_rows[:, 0]).sum(-1)
    Rinv = adj_rows / det[:, None, None]
    V = R.shape[0]
    w2c = torch.zeros(V, 4, 4, dtype=f64, device=campos.device)
    w2c[:, :3, :3] = Rinv
    w2c[:, :3, 3] = -(Rinv @ t[:, :, None])[:, :, 0]
    w2c[:, 3, 3] = 1.0
    cam_view = w2c.transpose(1, 2)
    cam_view_proj = cam_view @ projection_matrix(fovy, znear, zfar).to(campos.device, f64)
    return cam_view.float().contiguous(), cam_view_proj.float().contiguous(), -campos.float()


def render_orbit_frames(renderer, gaussians, azimuths, elevation: float = 0.0, radius: float = 1.5,
                        scale_modifier=1.0, chunk: int = 60, cameras=None):
    """infer.py:114-145's video loops (one render per azimuth) as batched renders of up to `chunk` views each, with
    the cameras built on the device: returns uint8 frames [V, H, W, 3] (on the renderer's device), each
    (image * 255) truncated as the reference's .astype(np.uint8). scale_modifier: one float, or one per azimuth
    (infer.py's fancy_video renders azimuth a with min(a / 360, 1), :129-131); consecutive frames with the same
    scale share a call. cameras: (cam_view [V,4,4], cam_view_proj [V,4,4], cam_pos [V,3]) to use instead of the
    device-built orbit."""
    opt = renderer.opt
    dev = gaussians.device
    if cameras is None:
        cv, cvp, cp = orbit_cameras_batched(elevation, azimuths, radius, opt.fovy, opt.znear, opt.zfar, device=dev)
    else:
        cv, cvp, cp = (t.to(dev) for t in cameras)
    V = cv.shape[0]
    sm = np.broadcast_to(np.asarray(scale_modifier, dtype=np.float64), (V,))
    frames = []
    v0 = 0
    while v0 < V:
        v1 = v0 + 1
        while v1 < V and v1 - v0 < chunk and sm[v1] == sm[v0]:
            v1 += 1
        img = renderer.render(gaussians, cv[None, v0:v1], cvp[None, v0:v1], cp[None, v0:v1],
                              scale_modifier=float(sm[v0]))["image"][0]
        frames.append((img.permute(0, 2, 3, 1) * 255).to(torch.uint8))
        v0 = v1
    return torch.cat(frames, 0)
