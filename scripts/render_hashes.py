"""Hashes of every render output for the library in LGM_AMD_LIB (or the default): bench.py's pool (fwd + bwd,
deterministic gradients), a cfg5-like fused-loss render at 512^2, a ragged small case and
one 256^2 view (the launches of at most 256 tiles: k_render_fwd's small-launch form) -- so kernel variants that
must be bitwise equal can be compared across child processes (scripts/gpu_ab.sh prints them per variant)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("LGM_AMD_DETERMINISTIC", "1")
import torch  # noqa: E402

from lgm_amd import GaussianRenderer, Options  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402


def h(t):
    return hashlib.sha1(t.detach().float().contiguous().cpu().numpy().tobytes()).hexdigest()[:10]


dev = torch.device("cuda:0")
out = {}
for name, (B, N, V, S, seed) in {"pool": (8, 100000, 6, 256, 2), "ragged": (2, 3000, 3, 72, 5),
                                    "one_view": (1, 50000, 1, 256, 3)}.items():
    r = GaussianRenderer(Options(output_size=S))
    g = synthetic_gaussians(B, N, seed=seed).to(dev).requires_grad_(True)
    cv, cvp, cp = (t[None].expand(B, *t.shape).contiguous().to(dev) for t in orbit_cameras(V, elevation=10.0))
    d_img, _, d_alpha, bg = synthetic_upstream_grads(B, V, S, S, seed=seed + 1000)
    o = r.render(g, cv, cvp, cp, bg_color=bg.to(dev))
    torch.autograd.backward([o["image"], o["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
    out[name] = {"image": h(o["image"]), "alpha": h(o["alpha"]), "depth": h(o["depth"]), "grad": h(g.grad)}
# fused loss at 512^2 (k_render_fwd<true> and the loss backward)
r = GaussianRenderer(Options(output_size=512))
g = synthetic_gaussians(1, 60000, seed=9).to(dev).requires_grad_(True)
cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(4, elevation=-10.0))
gen = torch.Generator().manual_seed(10)
gt = torch.rand(1, 4, 3, 512, 512, generator=gen).to(dev)
mask = (torch.rand(1, 4, 1, 512, 512, generator=gen) > 0.5).float().to(dev)
o = r.render(g, cv, cvp, cp, bg_color=torch.ones(3, device=dev), gt_images=gt, gt_masks=mask)
o["loss_mse"].backward()
out["loss"] = {"loss": float(o["loss_mse"]), "image": h(o["image"]), "grad": h(g.grad)}
print(json.dumps(out))
