"""ctypes front-end of the CPU rasterizer oracle (oracle/raster_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module. PARITY UNPINNED for
the rasterizer: see the header of raster_oracle.c. The batched call mirrors core/gs.py:42-93 (B x V loop,
per-(b, v) rasterizer call on the [N,14] slices, results stacked to [B,V,C,H,W]); the image is returned
UNCLAMPED (the clamp of core/gs.py:87 is applied by the caller, exactly as the product path applies it in torch).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liblgm_oracle.so")
_LIB64_PATH = os.path.join(_HERE, "_build", "liblgm_oracle_f64.so")
_libs = {}


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib(f64: bool = False):
    if f64 not in _libs:
        path = _LIB64_PATH if f64 else _LIB_PATH
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        f32p = ctypes.POINTER(ctypes.c_double if f64 else ctypes.c_float)
        rp = ctypes.c_double if f64 else ctypes.c_float
        i32p = ctypes.POINTER(ctypes.c_int)
        i64p = ctypes.POINTER(ctypes.c_longlong)
        L.lgm_oracle_render_batch.restype = ctypes.c_int
        L.lgm_oracle_render_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p, f32p, f32p,
                                              rp, rp, rp, f32p, ctypes.c_int,
                                              ctypes.c_int, f32p, f32p, f32p, i64p, f32p, f32p, f32p, f32p,
                                              ctypes.c_int]
        L.lgm_oracle_render_view.restype = ctypes.c_int
        L.lgm_oracle_render_view.argtypes = [ctypes.c_int, f32p, f32p, f32p, rp, rp,
                                             rp, f32p, ctypes.c_int, ctypes.c_int, f32p, f32p, f32p,
                                             i32p, i64p, f32p, f32p, f32p, f32p, f32p]
        L.lgm_oracle_preprocess_view.restype = ctypes.c_longlong
        L.lgm_oracle_preprocess_view.argtypes = [ctypes.c_int, f32p, f32p, f32p, rp, rp,
                                                 rp, ctypes.c_int, ctypes.c_int, i32p, f32p, f32p,
                                                 f32p, i32p]
        L.lgm_oracle_tile_lists.restype = ctypes.c_longlong
        L.lgm_oracle_tile_lists.argtypes = [ctypes.c_int, f32p, f32p, f32p, rp, rp,
                                            rp, ctypes.c_int, ctypes.c_int, i32p, i32p, ctypes.c_longlong]
        L.lgm_oracle_forward_state.restype = ctypes.c_longlong
        L.lgm_oracle_forward_state.argtypes = [ctypes.c_int, f32p, f32p, f32p, rp, rp, rp, ctypes.c_int,
                                               ctypes.c_int, i32p, f32p]
        L.lgm_oracle_set_tile_threads.restype = None
        L.lgm_oracle_set_tile_threads.argtypes = [ctypes.c_int]
        _libs[f64] = L
    return _libs[f64]


def _f(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _c(a, dtype=np.float32):
    return np.ascontiguousarray(np.asarray(a, dtype=dtype))


def render(gaussians, cam_view, cam_view_proj, tanfov: float, H: int, W: int, bg, scale_modifier: float = 1.0,
           d_image=None, d_depth=None, d_alpha=None, nthreads: int = 0, f64: bool = False, tile_threads: int = 1):
    """Forward (+ optional backward) of B x V renders. nthreads: OpenMP threads over the B x V views;
    tile_threads > 1 instead runs the views in sequence with that many threads over each view's tiles (the CPU
    baseline on all host cores; backward sums in a different order, equal to double rounding).

    gaussians [B,N,14]; cam_view/cam_view_proj [B,V,4,4] (row-major torch layout, as core/gs.py passes them);
    bg [3]. Returns dict with image [B,V,3,H,W] (unclamped), depth/alpha [B,V,1,H,W], K (total pairs),
    evals (pixel-Gaussian evaluations) and, if d_image is given, d_gaussians [B,N,14].
    """
    dt = np.float64 if f64 else np.float32
    g = _c(gaussians, dt)
    B, N = g.shape[0], g.shape[1]
    views = _c(cam_view, dt).reshape(B, -1, 16)
    V = views.shape[1]
    projs = _c(cam_view_proj, dt).reshape(B, V, 16)
    bgv = _c(bg, dt).reshape(3)
    color = np.zeros((B, V, 3, H, W), dt)
    depth = np.zeros((B, V, 1, H, W), dt)
    alpha = np.zeros((B, V, 1, H, W), dt)
    stats = np.zeros(2, np.int64)
    dg = None
    if d_image is not None:
        d_image = _c(d_image, dt).reshape(B, V, 3, H, W)
        d_depth = _c(np.zeros((B, V, 1, H, W)) if d_depth is None else d_depth, dt).reshape(B, V, 1, H, W)
        d_alpha = _c(np.zeros((B, V, 1, H, W)) if d_alpha is None else d_alpha, dt).reshape(B, V, 1, H, W)
        dg = np.zeros((B, N, 14), dt)
    if nthreads <= 0:
        nthreads = min(os.cpu_count() or 1, B * V)
    fp = (lambda a: None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))) if f64 else _f
    lib(f64).lgm_oracle_set_tile_threads(int(tile_threads))
    rc = lib(f64).lgm_oracle_render_batch(B, V, N, fp(g), fp(views), fp(projs), float(tanfov), float(tanfov),
                                       float(scale_modifier), fp(bgv), H, W, fp(color), fp(depth), fp(alpha),
                                       stats.ctypes.data_as(ctypes.POINTER(ctypes.c_longlong)), fp(d_image),
                                       fp(d_depth), fp(d_alpha), fp(dg), int(nthreads))
    lib(f64).lgm_oracle_set_tile_threads(1)
    if rc != 0:
        raise RuntimeError("oracle render failed")
    out = {"image": color, "depth": depth, "alpha": alpha, "K": int(stats[0]), "evals": int(stats[1])}
    if dg is not None:
        out["d_gaussians"] = dg
    return out


def preprocess(g_scene, view16, proj16, tanfov: float, H: int, W: int, scale_modifier: float = 1.0):
    """Per-Gaussian records of one view: radii, xy, depth, conic_opacity, rect, K."""
    g = _c(g_scene)
    N = g.shape[0]
    radii = np.zeros(N, np.int32)
    xy = np.zeros((N, 2), np.float32)
    depth = np.zeros(N, np.float32)
    conic = np.zeros((N, 4), np.float32)
    rect = np.zeros((N, 4), np.int32)
    i32 = ctypes.POINTER(ctypes.c_int)
    K = lib().lgm_oracle_preprocess_view(N, _f(g), _f(_c(view16).reshape(16)), _f(_c(proj16).reshape(16)),
                                         float(tanfov), float(tanfov), float(scale_modifier), H, W,
                                         radii.ctypes.data_as(i32), _f(xy), _f(depth), _f(conic),
                                         rect.ctypes.data_as(i32))
    return {"radii": radii, "xy": xy, "depth": depth, "conic_opacity": conic, "rect": rect, "K": int(K)}


def tile_lists(g_scene, view16, proj16, tanfov: float, H: int, W: int, scale_modifier: float = 1.0):
    """Sorted per-tile Gaussian lists of one view: (tile_start [T+1], ids [K])."""
    g = _c(g_scene)
    N = g.shape[0]
    T = ((W + 15) // 16) * ((H + 15) // 16)
    ts = np.zeros(T + 1, np.int32)
    i32 = ctypes.POINTER(ctypes.c_int)
    args = (N, _f(g), _f(_c(view16).reshape(16)), _f(_c(proj16).reshape(16)), float(tanfov), float(tanfov),
            float(scale_modifier), H, W, ts.ctypes.data_as(i32))
    K = lib().lgm_oracle_tile_lists(*args, None, 0)
    ids = np.zeros(max(K, 1), np.int32)
    lib().lgm_oracle_tile_lists(*args, ids.ctypes.data_as(i32), K)
    return ts, ids[:K]


def forward_state(g_scene, view16, proj16, tanfov: float, H: int, W: int, scale_modifier: float = 1.0):
    """Per-pixel forward state of one view: (n_contrib [H,W] int32, final_T [H,W] float32, K)."""
    g = _c(g_scene)
    N = g.shape[0]
    nc = np.zeros((H, W), np.int32)
    ft = np.zeros((H, W), np.float32)
    K = lib().lgm_oracle_forward_state(N, _f(g), _f(_c(view16).reshape(16)), _f(_c(proj16).reshape(16)),
                                       float(tanfov), float(tanfov), float(scale_modifier), H, W,
                                       nc.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), _f(ft))
    if K < 0:
        raise RuntimeError("oracle forward_state failed")
    return nc, ft, int(K)
