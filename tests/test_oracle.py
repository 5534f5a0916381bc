"""Pins the CPU oracle (oracle/raster_oracle.c) -- the reference rasterizer itself is absent (PARITY UNPINNED
against upstream CUDA). Pins: closed-form single-Gaussian known answers, float64 autograd of the
differentiable restatement (oracle/raster_autograd.py), and the committed golden fixtures."""
import glob
import math
import os

import numpy as np
import pytest
import torch

from oracle import raster_autograd as RA
from tests.render_cases import TAN, rel_l2, scene, upstream


def _single(x, y, z, s, op, rgb, H=32, W=32):
    g = torch.zeros(1, 1, 14)
    g[0, 0, 0:3] = torch.tensor([x, y, z])
    g[0, 0, 3] = op
    g[0, 0, 4:7] = s
    g[0, 0, 7] = 1.0
    g[0, 0, 11:14] = torch.tensor(rgb)
    return g


def test_single_gaussian_known_answer(oracle_mod):
    """Closed form: an isotropic Gaussian at the origin seen from the view-0 orbit camera (r = 1.5, fov 49.1):
    depth 1.5, focal f = W / (2 tan), 2D variance s^2 f^2 / z^2 + 0.3, centre pixel (W - 1) / 2."""
    H = W = 32
    s, op = 0.05, 0.8
    rgb = [0.9, 0.2, 0.4]
    g = _single(0, 0, 0, s, op, rgb, H, W)
    _, cv, cvp = scene(N=1, V=1)
    bg = np.array([0.1, 0.3, 0.5], np.float32)
    out = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg)
    f = W / (2 * TAN)
    var = (s * f / 1.5) ** 2 + 0.3
    c = (W - 1) / 2
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    power = -0.5 * ((xx - c) ** 2 + (yy - c) ** 2) / var
    alpha = np.minimum(0.99, op * np.exp(power))
    alpha[alpha < 1 / 255] = 0
    rad = math.ceil(3 * math.sqrt(var + math.sqrt(0.1) if False else var))  # isotropic: lambda_max = var
    img = np.stack([rgb[k] * alpha + (1 - alpha) * bg[k] for k in range(3)])
    assert np.abs(out["image"][0, 0] - img).max() < 2e-6
    assert np.abs(out["alpha"][0, 0, 0] - alpha).max() < 2e-6
    assert np.abs(out["depth"][0, 0, 0] - 1.5 * alpha).max() < 5e-6
    assert rad > 0


def test_two_gaussians_front_to_back(oracle_mod):
    """Two overlapping Gaussians on the optical axis: front one composited first (depth order)."""
    H = W = 16
    g = torch.cat([_single(0, 0, 0.3, 0.08, 0.6, [1, 0, 0], H, W), _single(0, 0, -0.3, 0.08, 0.7, [0, 0, 1], H, W)], 1)
    _, cv, cvp = scene(N=1, V=1)
    out = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, np.zeros(3, np.float32))
    c = (W - 1) / 2
    i = int(c)
    img = out["image"][0, 0, :, i, i]
    # at the pixel nearest the centre the red (front, z=+0.3 is closer to the camera at z=1.5) dominates
    assert img[0] > img[2] > 0


@pytest.mark.parametrize("seed,V,mod", [(3, 2, 1.0), (4, 1, 0.8), (5, 3, 1.2)])
def test_analytic_backward_matches_float64_autograd(oracle_mod, seed, V, mod):
    H = W = 40
    g, cv, cvp = scene(N=30, V=V, seed=seed, shrink=0.5, scale_mul=3.0, max_opacity=0.9)
    d_img, d_dep, d_alp, bg = upstream(1, V, H, W, seed=seed)
    ref = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), scale_modifier=mod,
                            d_image=d_img.numpy(), d_depth=d_dep.numpy(), d_alpha=d_alp.numpy())
    gd = g[0].double().clone().requires_grad_(True)
    loss = 0
    for v in range(V):
        c, d, a = RA.render_view(gd, cv[0, v].numpy().reshape(16), cvp[0, v].numpy().reshape(16), TAN, H, W,
                                 bg.numpy(), mod)
        assert rel_l2(c.detach().numpy(), ref["image"][0, v]) < 1e-5
        assert rel_l2(a.detach().numpy(), ref["alpha"][0, v]) < 1e-5
        assert rel_l2(d.detach().numpy(), ref["depth"][0, v]) < 1e-5
        loss = loss + (c * d_img[0, v].double()).sum() + (a * d_alp[0, v].double()).sum() + (d * d_dep[0, v].double()).sum()
    loss.backward()
    for name, sl in {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11),
                     "rgb": slice(11, 14)}.items():
        e = rel_l2(ref["d_gaussians"][0, :, sl], gd.grad.numpy()[:, sl])
        assert e < 2e-4, (name, e)


def test_permutation_invariance(oracle_mod):
    """Distinct depths: rendering does not depend on the order of the Gaussians in the array."""
    g, cv, cvp = scene(N=500, V=2, seed=8)
    perm = torch.randperm(500, generator=torch.Generator().manual_seed(0))
    bg = np.ones(3, np.float32)
    a = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, 48, 48, bg)
    b = oracle_mod.render(g[:, perm].numpy(), cv.numpy(), cvp.numpy(), TAN, 48, 48, bg)
    assert np.array_equal(a["image"], b["image"]) and a["K"] == b["K"]


def test_zero_opacity_is_background(oracle_mod):
    g, cv, cvp = scene(N=200, V=1, seed=1)
    g[..., 3] = 0
    bg = np.array([0.3, 0.4, 0.5], np.float32)
    a = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, 32, 32, bg)
    assert np.allclose(a["image"][0, 0], bg[:, None, None]) and np.all(a["alpha"] == 0)


def test_alpha_range(oracle_mod):
    g, cv, cvp = scene(N=3000, V=2, seed=2)
    a = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, 64, 64, np.ones(3, np.float32))
    assert a["alpha"].min() >= 0 and a["alpha"].max() <= 1
    assert a["image"].min() >= -1e-6 and a["image"].max() <= 1 + 1e-6


GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "render_*.npz")))


@pytest.mark.parametrize("path", GOLDEN, ids=[os.path.basename(p) for p in GOLDEN])
def test_oracle_reproduces_golden(oracle_mod, path):
    z = np.load(path)
    out = oracle_mod.render(z["gaussians"], z["cam_view"], z["cam_view_proj"], float(z["tanfov"]), int(z["H"]),
                            int(z["W"]), z["bg"], float(z["scale_modifier"]), d_image=z["d_image"],
                            d_depth=z["d_depth"], d_alpha=z["d_alpha"])
    for k in ("image", "depth", "alpha", "d_gaussians"):
        assert np.array_equal(out[k], z[k]), k
    assert out["K"] == int(z["K"])


def test_golden_present():
    assert len(GOLDEN) >= 4
