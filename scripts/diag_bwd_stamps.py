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
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # 1: cfg3 (seed 1); 8: bench.py's pool (seed 2)
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(B, 100000, seed=1 if B == 1 else 2).to(dev).requires_grad_(True)
cv, cvp, cp = (t[None].expand(B, *t.shape).contiguous().to(dev) for t in orbit_cameras(6))
d_img, _, d_alpha, bg = synthetic_upstream_grads(B, 6, 256, 256, seed=1001 if B == 1 else 1002)
L = _native.lib()
M = B * 6 * 256
cnt = torch.zeros(8 + 8 * M + 8 * B * 6 * 200 + 4 * 5 * M, dtype=torch.int64, device=dev)
for it in range(6):
    o = r.render(g, cv, cvp, cp, bg_color=bg.to(dev))
    torch.cuda.synchronize()
    if it == 5:
        cnt.zero_()
    with _native.diagnostics(render_counters=cnt if it == 5 else None):
        torch.autograd.backward([o["image"], o["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
        torch.cuda.synchronize()
    g.grad = None
c = cnt[:8].tolist()
names = ["prologue", "top_barrier", "chunk_head", "entries", "barrier_partials", "dma_wait", "flush_barrier",
         "atomics"]
tot = sum(c)
res = {n: {"Gcyc": round(v / 1e9, 3), "share": round(v / max(tot, 1), 3)} for n, v in zip(names, c)}
res["B"] = B
print(json.dumps(res))
