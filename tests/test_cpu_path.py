"""The CPU (torch) path of BASELINE config 1 (lgm_amd/cpu.py: GaussianRenderer / attention / head on CPU tensors)
against the oracles: the render against oracle/raster_oracle.c (forward 1e-4 relative L2, radii bit-exact,
gradients by autograd within max(1e-4, 2 x the fp32 oracle's own error) of the fp64 oracle), the attention against
the reference-generated fixtures (1e-4). CPU-only: these run in the driver's `-m "not gpu"` tier."""
import glob
import os

import numpy as np
import pytest
import torch

from lgm_amd import GaussianRenderer, Options
from lgm_amd.cpu import _preprocess, render_cpu
from tests.render_cases import TAN, rel_l2, scene, upstream

GROUPS = {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11), "rgb": slice(11, 14)}


@pytest.mark.parametrize("B,N,V,H,W,mod,elev", [(1, 1, 1, 32, 32, 1.0, 0.0), (1, 400, 2, 48, 48, 1.0, 15.0),
                                                 (2, 800, 2, 40, 56, 0.8, -20.0), (1, 3000, 1, 64, 64, 1.0, 0.0)])
def test_cpu_render_matches_oracle(oracle_mod, B, N, V, H, W, mod, elev):
    g, cv, cvp = scene(B=B, N=N, V=V, seed=N + 1, elevation=elev)
    d_img, d_dep, d_alp, bg = upstream(B, V, H, W, seed=N)
    gd = g.clone().requires_grad_(True)
    img, dep, alp = render_cpu(gd, cv, cvp, bg, TAN, TAN, H, W, mod)
    ((img * d_img).sum() + (dep * d_dep).sum() + (alp * d_alp).sum()).backward()
    kw = dict(scale_modifier=mod, d_image=d_img.numpy(), d_depth=d_dep.numpy(), d_alpha=d_alp.numpy())
    ref = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), **kw)
    truth = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, W, bg.numpy(), f64=True, **kw)
    for k, t in (("image", img), ("depth", dep), ("alpha", alp)):
        assert rel_l2(t.detach().numpy(), ref[k]) < 1e-4, k
    for name, sl in GROUPS.items():
        e = rel_l2(gd.grad.numpy()[..., sl], truth["d_gaussians"][..., sl])
        e32 = rel_l2(ref["d_gaussians"][..., sl], truth["d_gaussians"][..., sl])
        assert e < max(1e-4, 2 * e32), (name, e, e32)
    for b in range(B):
        for v in range(V):
            pre = _preprocess(g[b], cv[b, v], cvp[b, v], TAN, TAN, H, W, mod)
            o = oracle_mod.preprocess(g[b].numpy(), cv[b, v].numpy(), cvp[b, v].numpy(), TAN, H, W, mod)
            assert np.array_equal(pre["radii"].numpy(), o["radii"])


def test_renderer_api_on_cpu_tensors(oracle_mod):
    """GaussianRenderer.render with CPU tensors (infer.py on a CPU-only host): clamped image, alpha, depth."""
    opt = Options(output_size=32)
    r = GaussianRenderer(opt)
    g, cv, cvp = scene(N=500, V=2, seed=3)
    out = r.render(g, cv, cvp, torch.zeros(1, 2, 3), bg_color=torch.ones(3))
    ref = oracle_mod.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, 32, 32, np.ones(3, np.float32))
    assert out["image"].shape == (1, 2, 3, 32, 32) and not out["image"].is_cuda
    assert rel_l2(out["image"].numpy(), np.clip(ref["image"], 0, 1)) < 1e-4
    assert rel_l2(out["alpha"].numpy(), ref["alpha"]) < 1e-4


def test_cpu_attention_matches_reference_fixtures():
    """The CPU (torch) attention path against the reference-generated fixtures: four small ones and the two seeded
    ones at LGM's real widths (C = 512 / 1024, 16 heads)."""
    from lgm_amd.attention import MemEffAttention, MVAttention
    from tests.test_attention import _err, _load
    paths = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "attn_*.npz")))
    seeded = [p for p in paths if "_h16_" in p]
    for path in [p for p in paths if p not in seeded][:4] + seeded:
        meta, z, params, _ = _load(path)
        if meta["kind"] == "memeff":
            m = MemEffAttention(meta["dim"], meta["num_heads"], qkv_bias=False, proj_bias=True)
        else:
            m = MVAttention(meta["dim"], meta["num_heads"], num_frames=meta["num_frames"],
                            skip_scale=meta["skip_scale"])
        m.load_state_dict(params)
        x = torch.from_numpy(z["x"]).requires_grad_(True)
        y = m(x)
        y.backward(torch.from_numpy(z["gy"]))
        assert _err(y.detach().numpy(), z["y"]) < 1e-4, path
        assert _err(x.grad.numpy(), z["dx"]) < 1e-4, path
