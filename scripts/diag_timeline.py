"""Whole-step timeline of one render fwd+bwd from the per-workgroup stamps (lgm_diag.render_counters): raw start /
end of every binning, sort, forward, backward-item and preprocess-backward workgroup on one clock, dumped as
gpurun_out/timeline_B{B}.npz for offline analysis (scripts/timeline_report.py), plus a short summary.
    python scripts/diag_timeline.py [B]     (B = 1: cfg3, seed 1; B = 8: bench.py's pool, seed 2)"""
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
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
N, V = 100000, 6
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(B, N, seed=1 if B == 1 else 2).to(dev).requires_grad_(True)
cv, cvp, cp = (t[None].expand(B, *t.shape).contiguous().to(dev) for t in orbit_cameras(V))
d_img, _, d_alpha, bg = synthetic_upstream_grads(B, V, 256, 256, seed=1001 if B == 1 else 1002)
d_img, d_alpha, bg = d_img.to(dev), d_alpha.to(dev), bg.to(dev)
M = B * V * 256
NB = B * V * ((N + 511) // 512)  # binning records reserved (k_bin uses B * ceil(V / 3) * ceil(N / 512))
NI = 3 * M + 16  # backward work items: one per tile (rounded up to 8) and one per checkpoint slot (include/lgm_render.h)
cnt = torch.zeros(8 + 8 * M + 8 * NB + 4 * NI, dtype=torch.int64, device=dev)


def step(diag):
    if diag:
        with _native.diagnostics(render_counters=cnt):
            out = r.render(g, cv, cvp, cp, bg_color=bg)
            torch.autograd.backward([out["image"], out["alpha"]], [d_img, d_alpha])
    else:
        out = r.render(g, cv, cvp, cp, bg_color=bg)
        torch.autograd.backward([out["image"], out["alpha"]], [d_img, d_alpha])
    g.grad = None


for _ in range(5):
    step(False)
torch.cuda.synchronize()
runs = []
for rep in range(3):  # three instrumented steps: their spread says how much one timeline can be trusted
    cnt.zero_()
    step(True)
    torch.cuda.synchronize()
    runs.append(cnt.cpu().numpy().copy())
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/timeline_B{B}.npz", runs=np.stack(runs), M=M, NB=NB, NI=NI, B=B, V=V, N=N)
c = runs[-1]
tl = c[8:8 + 8 * M].reshape(M, 8)
bt = c[8 + 8 * M:8 + 8 * M + 8 * NB].reshape(NB, 8)
it = c[8 + 8 * M + 8 * NB:].reshape(NI, 4)
t0 = bt[bt[:, 0] > 0, 0].min()
us = lambda x: round(float(x - t0) * 0.01, 2)  # noqa: E731
summ = {}
for name, st, en in (("bin", bt[:, 0], bt[:, 4]), ("sort", tl[:, 4], tl[:, 5]), ("fwd", tl[:, 0], tl[:, 1]),
                     ("bwd", it[:, 0], it[:, 1]), ("preproc_bwd", tl[:, 2], tl[:, 3])):
    ok = en > 0
    if ok.any():
        dur = (en[ok] - st[ok]) * 0.01
        summ[name] = {"first_start": us(st[ok].min()), "last_start": us(st[ok].max()), "end": us(en[ok].max()),
                      "wgs": int(ok.sum()), "dur_p50": round(float(np.median(dur)), 2),
                      "dur_max": round(float(dur.max()), 2), "dur_sum": round(float(dur.sum()), 1)}
print(json.dumps(summ))
json.dump(summ, open(f"gpurun_out/timeline_B{B}.json", "w"), indent=1)
