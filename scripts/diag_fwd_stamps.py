"""Per-tile section cycles of k_render_fwd from the LGM_FWD_STAMPS diagnostic build (LGM_AMD_LIB pointing at it):
BASELINE config 2 (50k Gaussians, one 256^2 view, forward only). For each tile, wave 0's shader cycles in the chunk
head (termination count, DMA, wait, entry tests, barrier), the checkpoint / compaction step and the compositing loop,
the whole chunk loop, and the tile's wall span; the slowest tiles and the means. -> stdout JSON"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians  # noqa: E402

dev = torch.device("cuda:0")
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(1, 50_000, seed=seed).to(dev)
cv, cvp, cp = (t[None].to(dev) for t in orbit_cameras(1))
bg = torch.ones(3, device=dev)
M = 256
NB = (50_000 + 511) // 512
cnt = torch.zeros(8 + 8 * M + 8 * NB + 4 * 5 * M + 32 * M, dtype=torch.int64, device=dev)
with torch.no_grad():
    for _ in range(5):
        r.render(g, cv, cvp, cp, bg_color=bg)
    torch.cuda.synchronize()
    with _native.diagnostics(render_counters=cnt):
        r.render(g, cv, cvp, cp, bg_color=bg)
        torch.cuda.synchronize()
tl = np.array(cnt[8: 8 + 8 * M].tolist(), dtype=np.int64).reshape(M, 8)
span_us = (tl[:, 1] - tl[:, 0]) / 100.0  # s_memrealtime: 100 MHz
t0 = tl[:, 0].min()
start_us, end_us = (tl[:, 0] - t0) / 100.0, (tl[:, 1] - t0) / 100.0
head, mid, comp, loop = tl[:, 2], tl[:, 3], tl[:, 4], tl[:, 5]
n = tl[:, 6] & 0xFFFFFFFF
staged = tl[:, 7] & 0xFFFFFFFF
steps = (tl[:, 7] >> 32) & 0xFFFFFF
order = np.argsort(-end_us)
rows = []
for t in order[:12]:
    rows.append({"tile": int(t), "start_us": round(float(start_us[t]), 2), "end_us": round(float(end_us[t]), 2),
                 "span_us": round(float(span_us[t]), 2), "n": int(n[t]), "staged": int(staged[t]),
                 "w0_entries": int(steps[t]), "head_kcyc": round(head[t] / 1e3, 1), "mid_kcyc": round(mid[t] / 1e3, 1),
                 "comp_kcyc": round(comp[t] / 1e3, 1), "loop_kcyc": round(loop[t] / 1e3, 1)})
res = {"slowest": rows,
       "mean": {"span_us": round(float(span_us.mean()), 2), "head_kcyc": round(head.mean() / 1e3, 1),
                "mid_kcyc": round(mid.mean() / 1e3, 1), "comp_kcyc": round(comp.mean() / 1e3, 1),
                "loop_kcyc": round(loop.mean() / 1e3, 1), "staged": float(staged.mean()),
                "w0_entries": float(steps.mean())},
       "launch_us": round(float(end_us.max()), 2), "last_start_us": round(float(start_us.max()), 2)}
print(json.dumps(res, indent=1))
