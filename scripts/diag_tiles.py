"""Per-tile list length n (k_sort) vs entries the forward actually walks (k_render_fwd), cfg3: how much of each
sorted list is ever consumed. -> gpurun_out/tiles.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(1, 100000, seed=1).to(dev)
cv, cvp, cp = orbit_cameras(6)
M = 6 * 256
NB = 6 * ((100000 + 511) // 512)
cnt = torch.zeros(8 + 8 * M + 8 * NB + 4 * 5 * M + 32 * M, dtype=torch.int64, device=dev)
L = _native.lib()
r.render(g, cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev))
torch.cuda.synchronize()
with _native.diagnostics(render_counters=cnt):
    r.render(g, cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev))
    torch.cuda.synchronize()
tl = np.array(cnt[8: 8 + 8 * M].tolist(), dtype=np.int64).reshape(M, 8)
n, staged = tl[:, 6] & 0xFFFFFFFF, tl[:, 7] & 0xFFFFFFFF
res = {"n_mean": float(n.mean()), "n_max": int(n.max()), "staged_mean": float(staged.mean()),
       "staged_max": int(staged.max()), "frac_consumed": float(staged.sum() / max(1, n.sum()))}
for K in (256, 512, 768, 1024, 1536, 2048):
    need = staged > K
    res[f"tiles_staged_over_{K}"] = int(need.sum())
    res[f"sort_work_if_prefix_{K}"] = float(np.minimum(n, K).sum() / n.sum())
res["staged_hist_256"] = np.bincount(staged // 256).tolist()
res["n_hist_256"] = np.bincount(n // 256).tolist()
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/tiles.json", "w"), indent=1)
