"""Work counters of one cfg3 forward+backward (lgm_render_debug_counters) -> gpurun_out/counters.json."""
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
M = 6 * 256
cnt = torch.zeros(8 + 4 * M, dtype=torch.int64, device=dev)
L = _native.lib()
L.lgm_render_debug_counters(_native.ptr(cnt))
out = r.render(g, cv[None].to(dev), cvp[None].to(dev), cp[None].to(dev), bg_color=bg.to(dev))
torch.autograd.backward([out["image"], out["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
torch.cuda.synchronize()
L.lgm_render_debug_counters(None)
c = cnt.tolist()
names = ["fwd_wave_iters", "fwd_contribs", "bwd_wave_iters", "bwd_contribs", "bwd_dense", "bwd_sparse",
         "fwd_entries_staged", "fwd_max_wave_iters"]
res = dict(zip(names, c[:8]))
import numpy as np  # noqa: E402
tl = np.array(c[8:], dtype=np.int64).reshape(M, 4)
for name, (a, b) in {"fwd": (0, 1), "bwd": (2, 3)}.items():
    st, en = tl[:, a], tl[:, b]
    ok = en > 0
    st, en = st[ok], en[ok]
    t0 = st.min()
    dur = (en - st) * 0.01  # us
    res[f"{name}_span_us"] = float((en.max() - t0) * 0.01)
    res[f"{name}_wg_us_p50"] = float(np.median(dur))
    res[f"{name}_wg_us_p99"] = float(np.percentile(dur, 99))
    res[f"{name}_wg_us_max"] = float(dur.max())
    res[f"{name}_start_spread_us"] = float((st.max() - t0) * 0.01)
    res[f"{name}_wg_sum_us"] = float(dur.sum())
    order = np.argsort(-dur)[:5]
    res[f"{name}_slowest_tiles"] = [(int(np.nonzero(ok)[0][i]), float(dur[i])) for i in order]
res["fwd_lane_util"] = c[1] / max(1, 64 * c[0])
res["bwd_lane_util"] = c[3] / max(1, 64 * c[2])
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open("gpurun_out/counters.json", "w"), indent=1)
