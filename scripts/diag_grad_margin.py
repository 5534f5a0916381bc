"""Gradient error margins vs the fp64 truth (per parameter group) for the library in LGM_AMD_LIB, at cfg3 and at a
small config, next to the fp32 oracle's own error: the quantity the GPU parity tests bound."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgm_amd.gs import rasterize  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.render_cases import TAN, rel_l2, scene, upstream  # noqa: E402

dev = torch.device("cuda:0")
GROUPS = {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11), "rgb": slice(11, 14)}
for (B, N, V, H) in [(1, 100000, 6, 256), (2, 2000, 3, 64)]:
    g, cv, cvp = scene(B=B, N=N, V=V, seed=N + V)
    d_img, d_dep, d_alp, bg = upstream(B, V, H, H, seed=3)
    gd = g.to(dev).requires_grad_(True)
    img, dep, alp = rasterize(gd, cv.to(dev), cvp.to(dev), bg.to(dev), TAN, TAN, H, H)
    torch.autograd.backward([img, alp], [d_img.to(dev), d_alp.to(dev)])
    G = gd.grad.cpu().numpy()
    kw = dict(d_image=d_img.numpy(), d_alpha=d_alp.numpy())
    o32 = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, H, bg.numpy(), **kw)["d_gaussians"]
    o64 = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, H, H, bg.numpy(), f64=True, **kw)["d_gaussians"]
    print(f"B{B} N{N} V{V} {H}^2: total GPU {rel_l2(G, o64):.2e} oracle32 {rel_l2(o32, o64):.2e}")
    for n, sl in GROUPS.items():
        eg, eo = rel_l2(G[..., sl], o64[..., sl]), rel_l2(o32[..., sl], o64[..., sl])
        print(f"   {n:8s} GPU {eg:.2e}  oracle32 {eo:.2e}  bar {max(1e-4, 2 * eo):.2e}  margin {max(1e-4, 2 * eo) / eg:.1f}x")
