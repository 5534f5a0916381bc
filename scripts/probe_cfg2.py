"""BASELINE config 2 forward renders only (50k Gaussians, one 256^2 view, bench.py's seed), for rocprofv3 counter
passes on the small-launch k_render_fwd: python scripts/probe_cfg2.py [STEPS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from lgm_amd import GaussianRenderer, Options  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda:0")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(1, 50_000, seed=bench.CFG2_SEED).to(dev)
cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(1))
bg = torch.ones(3, device=dev)
with torch.no_grad():
    for _ in range(steps):
        r.render(g, cv, cvp, cp, bg_color=bg)
    torch.cuda.synchronize()
print("ok")
