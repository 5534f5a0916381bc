"""Section shares of k_render_bwd from the LGM_BWD_STAMPS diagnostic build (shader-clock cycles summed over
waves): python scripts/diag_bwd_stamps.py with LGM_AMD_LIB pointing at that build. Shares only, not time."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(1, 100000, seed=1).to(dev).requires_grad_(True)
cv, cvp, cp = orbit_cameras(6)
d_img, _, d_alpha, bg = synthetic_upstream_grads(1, 6, 256, 256, seed=1001)
L = _native.lib()
cnt = torch.zeros(8 + 8 * 6 * 256 + 8 * 6 * 200 + 4 * 5 * 6 * 256, dtype=torch.int64, device=dev)
for it in range(6):
    o = r.render(g, cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev), bg_color=bg.to(dev))
    torch.cuda.synchronize()
    if it == 5:
        cnt.zero_()
    with _native.diagnostics(render_counters=cnt if it == 5 else None):
        torch.autograd.backward([o["image"], o["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
        torch.cuda.synchronize()
    g.grad = None
c = cnt[:10].tolist()
names = ["stage", "compact", "entries", "flush", "tail"]
tot = sum(c[2:7])
res = {n: {"Gcyc": round(v / 1e9, 3), "share": round(v / max(tot, 1), 3)} for n, v in zip(names, c[2:7])}
res["quadrant_imbalance_max_over_mean"] = round(c[9] / max(c[8], 1), 3)
print(json.dumps(res))
