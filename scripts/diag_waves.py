"""Per-wave timeline of the wave-independent compositing kernels on one cfg3 step (diagnostic counters):
per-SIMD / per-CU busy spans and work, to tell imbalance from throughput limits. -> gpurun_out/waves.json"""
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
g = synthetic_gaussians(1, 100000, seed=1).to(dev).requires_grad_(True)
cv, cvp, cp = orbit_cameras(6)
d_img, _, d_alpha, bg = synthetic_upstream_grads(1, 6, 256, 256, seed=1001)
M = 6 * 256
NB = 6 * ((100000 + 511) // 512)
W0 = 8 + 8 * M + 8 * NB + 4 * 5 * M
cnt = torch.zeros(W0 + 2 * 4 * 4 * M, dtype=torch.int64, device=dev)
L = _native.lib()


def step():
    o = r.render(g, cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev), bg_color=bg.to(dev))
    torch.autograd.backward([o["image"], o["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
    g.grad = None


for _ in range(5):
    step()
torch.cuda.synchronize()
L.lgm_render_debug_counters(_native.ptr(cnt))
for _ in range(3):
    step()
torch.cuda.synchronize()
L.lgm_render_debug_counters(None)
c = np.array(cnt.tolist(), dtype=np.int64)
res = {}
for pi, name in enumerate(["fwd", "bwd"]):
    w = c[W0 + pi * 16 * M: W0 + (pi + 1) * 16 * M].reshape(4 * M, 4)
    ok = w[:, 1] > 0
    w = w[ok]
    t0 = w[:, 0].min()
    st, en = (w[:, 0] - t0) * 0.01, (w[:, 1] - t0) * 0.01
    nlist = w[:, 3] >> 32
    w[:, 3] &= 0xFFFFFFFF
    hw = w[:, 2] & 0xFFFFFFFF
    xcc = (w[:, 2] >> 32) & 0xF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    cu_key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    simd_key = cu_key * 4 + simd
    dur = en - st
    out = {"waves": int(len(w)), "span_us": round(float(en.max()), 2), "start_spread_us": round(float(st.max()), 2),
           "dur_p50": round(float(np.median(dur)), 2), "dur_p90": round(float(np.percentile(dur, 90)), 2),
           "dur_max": round(float(dur.max()), 2), "work_mean": round(float(w[:, 3].mean()), 1),
           "work_max": int(w[:, 3].max())}
    cc = np.corrcoef(w[:, 3], dur)[0, 1]
    out["corr_work_dur"] = round(float(cc), 3)
    for kname, key in [("cu", cu_key), ("simd", simd_key)]:
        u = np.unique(key)
        endt = np.array([en[key == k].max() for k in u])
        work = np.array([w[key == k, 3].sum() for k in u])
        nw = np.array([(key == k).sum() for k in u])
        out[f"{kname}_count"] = int(len(u))
        out[f"{kname}_end_p10_p50_max"] = [round(float(np.percentile(endt, 10)), 2), round(float(np.median(endt)), 2),
                                           round(float(endt.max()), 2)]
        out[f"{kname}_work_min_mean_max"] = [int(work.min()), round(float(work.mean()), 1), int(work.max())]
        out[f"{kname}_waves_min_max"] = [int(nw.min()), int(nw.max())]
        out[f"{kname}_corr_work_end"] = round(float(np.corrcoef(work, endt)[0, 1]), 3)
    # how busy over time: fraction of waves still running at 25/50/75/90 % of the span
    sp = en.max()
    out["running_at_frac"] = {str(f): int(((st <= f * sp) & (en >= f * sp)).sum()) for f in (0.1, 0.25, 0.5, 0.75, 0.9)}
    top = np.argsort(-dur)[:12]
    out["longest"] = [[round(float(dur[i]), 1), int(w[i, 3]), int(nlist[i]), round(float(st[i]), 1)] for i in top]
    out["work_dur_by_decile"] = []
    qs = np.percentile(w[:, 3], np.arange(0, 101, 10))
    for a, b in zip(qs[:-1], qs[1:]):
        m = (w[:, 3] >= a) & (w[:, 3] <= b)
        if m.any():
            out["work_dur_by_decile"].append([int(a), int(b), round(float(dur[m].mean()), 1), round(float(dur[m].max()), 1)])
    res[name] = out
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/waves.json", "w"), indent=1)
