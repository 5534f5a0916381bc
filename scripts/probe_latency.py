"""Latency vs throughput probe: per-kernel times of the render step (fwd + image/alpha bwd) as the batch grows
(1 scene x 1/2/3/6 views, 2/4/8 scenes x 6 views). Kernels whose time stays flat as work shrinks are latency-bound
(critical path / partial waves), those that scale are throughput-bound. Prints one JSON line per workload."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
r = GaussianRenderer(Options(output_size=256))
cv0, cvp0, cp0 = orbit_cameras(6)
steps = 20
for B, V in [(int(a), int(b)) for a, b in (x.split('x') for x in (sys.argv[1:] or ['1x1', '1x2', '1x3', '1x6', '2x6', '4x6', '8x6']))]:
    g = synthetic_gaussians(B, 100_000, seed=2).to(dev).requires_grad_(True)
    d_img, _, d_alpha, bg = synthetic_upstream_grads(B, V, 256, 256, seed=1001)
    cv = cv0[None, :V].expand(B, -1, -1, -1).contiguous().to(dev)
    cvp = cvp0[None, :V].expand(B, -1, -1, -1).contiguous().to(dev)
    cp = cp0[None, :V].expand(B, -1, -1).contiguous().to(dev)
    di, da, bgd = d_img.to(dev), d_alpha.to(dev), bg.to(dev)

    def step():
        out = r.render(g, cv, cvp, cp, bg_color=bgd)
        torch.autograd.backward([out["image"], out["alpha"]], [di, da])
        g.grad = None

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(steps):
        step()
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / steps
    import time
    host = []
    for _ in range(10):  # host issue time of one step with an idle GPU queue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        host.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    prof = _native.KernelProfiler()
    with prof:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    k = prof.summary()
    prof.close()
    print(json.dumps({"B": B, "V": V, "ms": round(ms, 4), "us_per_view": round(1e3 * ms / (B * V), 2),
                      "host_us_min": round(1e6 * min(host), 1), "host_us_med": round(1e6 * sorted(host)[5], 1),
                      "kernels_us": {n: round(1e3 * ms_ / cnt, 1) for n, (cnt, ms_) in k.items()}}), flush=True)
