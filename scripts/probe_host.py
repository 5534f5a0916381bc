"""Host-side cost of one render step (fwd + image/alpha bwd): cProfile of 300 single-view steps (GPU work is
small there, so the host path dominates), top functions by own time, plus the ctypes entry points' wall times."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
r = GaussianRenderer(Options(output_size=256))
cv0, cvp0, cp0 = orbit_cameras(6)
V = int(sys.argv[1]) if len(sys.argv) > 1 else 1
g = synthetic_gaussians(1, 100_000, seed=2).to(dev).requires_grad_(True)
d_img, _, d_alpha, bg = synthetic_upstream_grads(1, V, 256, 256, seed=1001)
cv, cvp, cp = cv0[None, :V].contiguous().to(dev), cvp0[None, :V].contiguous().to(dev), cp0[None, :V].contiguous().to(dev)
di, da, bgd = d_img.to(dev), d_alpha.to(dev), bg.to(dev)


def step():
    out = r.render(g, cv, cvp, cp, bg_color=bgd)
    torch.autograd.backward([out["image"], out["alpha"]], [di, da])
    g.grad = None


_calls = {}


def _wrap(name):
    L = _native.lib()
    f = getattr(L, name)

    def w(*a):
        t0 = time.perf_counter()
        rv = f(*a)
        _calls.setdefault(name, []).append(time.perf_counter() - t0)
        return rv
    setattr(L, name, w)


for _n in ("lgm_render_forward", "lgm_render_backward", "lgm_render_workspace_size_opts"):
    _wrap(_n)
for _ in range(5):
    step()
torch.cuda.synchronize()
# wall time of the pieces, GPU idle before each
parts = {"render": [], "backward": [], "zero_grad": []}
for _ in range(50):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = r.render(g, cv, cvp, cp, bg_color=bgd)
    t1 = time.perf_counter()
    torch.autograd.backward([out["image"], out["alpha"]], [di, da])
    t2 = time.perf_counter()
    g.grad = None
    t3 = time.perf_counter()
    parts["render"].append(t1 - t0)
    parts["backward"].append(t2 - t1)
    parts["zero_grad"].append(t3 - t2)
torch.cuda.synchronize()
print({k: round(1e6 * sorted(v)[len(v) // 2], 1) for k, v in parts.items()}, "us (median)", flush=True)
print("C-ABI calls (median us):", {k: round(1e6 * sorted(v)[len(v) // 2], 1) for k, v in _calls.items()}, flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(300):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
