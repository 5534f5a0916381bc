"""Largest tile list of the bench workloads (pool seed 2, cfg3 seed 1): the bound a capped slot stride must exceed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from bench import CFG3_SEED, N_GAUSS, POOL_SCENES, POOL_SEED, RES, VIEWS  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.gs import forward_state  # noqa: E402
from lgm_amd import GaussianRenderer, Options  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda", 0)
tan = float(GaussianRenderer(Options(output_size=RES)).tan_half_fov)
cv, cvp, _ = orbit_cameras(VIEWS)
for name, B, seed in (("pool", POOL_SCENES, POOL_SEED), ("cfg3", 1, CFG3_SEED)):
    g = synthetic_gaussians(B, N_GAUSS, seed=seed).to(dev)
    st = forward_state(g, cv[None].expand(B, -1, -1, -1).contiguous().to(dev),
                       cvp[None].expand(B, -1, -1, -1).contiguous().to(dev), tan, tan, RES, RES)
    c = st["tile_counts"]
    print(name, "max", int(c.max()), "mean", float(c.mean()), "p99", float(sorted(c.ravel())[int(0.99 * c.size)]))
