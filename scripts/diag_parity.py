"""cfg3 parity diagnostics: per-group rel L2 GPU vs oracle, GPU run-to-run (float-atomic order), and the
Gaussians that dominate the gradient error."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgm_amd.gs import rasterize  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.render_cases import TAN, rel_l2, scene, upstream  # noqa: E402

dev = torch.device("cuda:0")
g, cv, cvp = scene(N=100000, V=6, seed=1)
d_img, d_dep, d_alp, bg = upstream(1, 6, 256, 256, seed=2)
use_depth = "--no-depth" not in sys.argv


def gpu():
    gd = g.to(dev).requires_grad_(True)
    img, dep, alp = rasterize(gd, cv.to(dev), cvp.to(dev), bg.to(dev), TAN, TAN, 256, 256)
    outs, grads = [img, alp], [d_img.to(dev), d_alp.to(dev)]
    if use_depth:
        outs.append(dep)
        grads.append(d_dep.to(dev))
    torch.autograd.backward(outs, grads)
    torch.cuda.synchronize()
    return img.detach().cpu().numpy(), gd.grad.cpu().numpy()


img1, g1 = gpu()
img2, g2 = gpu()
ref = O.render(g.numpy(), cv.numpy(), cvp.numpy(), TAN, 256, 256, bg.numpy(), d_image=d_img.numpy(),
               d_depth=d_dep.numpy() if use_depth else None, d_alpha=d_alp.numpy())
R = ref["d_gaussians"]
print("image rel", rel_l2(img1, ref["image"]), "total grad rel", rel_l2(g1, R), "gpu-vs-gpu", rel_l2(g1, g2))
for name, sl in {"mean": slice(0, 3), "opacity": slice(3, 4), "scale": slice(4, 7), "rot": slice(7, 11),
                 "rgb": slice(11, 14)}.items():
    print(f"  {name:8s} rel {rel_l2(g1[..., sl], R[..., sl]):.3e}  gpu-vs-gpu {rel_l2(g1[..., sl], g2[..., sl]):.3e}"
          f"  |ref| {np.linalg.norm(R[..., sl]):.3e}")
err = np.linalg.norm((g1 - R)[0], axis=1)
tot = np.linalg.norm(g1 - R)
idx = np.argsort(-err)[:10]
pre = O.preprocess(g[0].numpy(), cv[0, 0].numpy(), cvp[0, 0].numpy(), TAN, 256, 256)
print("top error Gaussians (share of total error^2):")
for i in idx:
    print(f"  {i:6d} err {err[i]:.3e} share {err[i]**2 / tot**2:.3f} |ref| {np.linalg.norm(R[0, i]):.3e} "
          f"op {g[0, i, 3]:.3f} scale {g[0, i, 4:7].numpy().round(4)} radius(v0) {pre['radii'][i]} "
          f"pos {g[0, i, 0:3].numpy().round(3)}")
