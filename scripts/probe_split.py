"""Probe: one cfg3 scene (100k Gaussians x 6 views x 256^2, fwd+bwd through the C ABI) as ONE call vs its views split
into halves / thirds rendered as independent calls -- on one stream (the cost of the smaller launches) and on two or
three streams (whether concurrent half-size chains fill each other's kernel tails). GPU span per step from events on
the main stream (the side streams fork from and join into it each step); host enqueue time alongside."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lgm_amd import _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.gs import tan_half_fov  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
L = _native.lib()
N, V, R = 100_000, 6, 256
g = synthetic_gaussians(1, N, seed=1).to(dev)
cv, cvp, _ = orbit_cameras(V)
cv, cvp = cv[None].to(dev), cvp[None].to(dev)
d_img, _, d_alpha, bg = synthetic_upstream_grads(1, V, R, R, seed=1001)
d_img, d_alpha, bg = d_img.to(dev), d_alpha.to(dev), bg.to(dev)
tan = tan_half_fov(49.1)
OPT = 2  # LGM_RENDER_CLAMP_IMAGE


class Part:
    def __init__(self, v0, v1):
        self.v0, self.v1, self.V = v0, v1, v1 - v0
        self.cv, self.cvp = cv[:, v0:v1].contiguous(), cvp[:, v0:v1].contiguous()
        self.di, self.da = d_img[:, v0:v1].contiguous(), d_alpha[:, v0:v1].contiguous()
        self.ws_bytes = L.lgm_render_workspace_size_opts(1, self.V, N, R, R, 0, OPT)
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        self.img = torch.empty(1, self.V, 3, R, R, device=dev)
        self.dep = torch.empty(1, self.V, 1, R, R, device=dev)
        self.alp = torch.empty(1, self.V, 1, R, R, device=dev)
        self.dg = torch.empty_like(g)

    def run(self, stream):
        st = stream.cuda_stream
        p = _native.ptr
        _native.check(L.lgm_render_forward(1, self.V, N, R, R, p(g), p(self.cv), p(self.cvp), p(bg), tan, tan, 1.0,
                                           p(self.img), p(self.dep), p(self.alp), None, p(self.ws), self.ws_bytes, 0,
                                           None, OPT, st, None), "fwd")
        _native.check(L.lgm_render_backward(1, self.V, N, R, R, p(g), p(self.cv), p(self.cvp), p(bg), tan, tan, 1.0,
                                            p(self.di), None, p(self.da), p(self.dg), None, p(self.ws), self.ws_bytes,
                                            0, OPT, st, None), "bwd")


def measure(parts, streams, steps=60):
    main = torch.cuda.current_stream()
    total = torch.empty_like(g)

    def step():
        ev = torch.cuda.Event()
        ev.record(main)
        for i, pt in enumerate(parts):
            s = streams[i % len(streams)]
            if s is not main:
                s.wait_event(ev)
            pt.run(s)
        for s in streams:
            if s is not main:
                e2 = torch.cuda.Event()
                e2.record(s)
                main.wait_event(e2)
        if len(parts) > 1:
            torch.sum(torch.stack([pt.dg for pt in parts]), 0, out=total)
    for _ in range(30):
        step()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    st.record(main)
    for _ in range(steps):
        step()
    en.record(main)
    host = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    return {"gpu_ms_per_step": round(st.elapsed_time(en) / steps, 4), "host_ms_per_step": round(host, 4)}


main = torch.cuda.current_stream()
side = [torch.cuda.Stream(device=dev) for _ in range(2)]
full = [Part(0, 6)]
halves = [Part(0, 3), Part(3, 6)]
thirds = [Part(0, 2), Part(2, 4), Part(4, 6)]
res = {}
for rnd in range(2):
    res[f"full_r{rnd}"] = measure(full, [main])
    res[f"halves_1stream_r{rnd}"] = measure(halves, [main])
    res[f"halves_2streams_r{rnd}"] = measure(halves, [main, side[0]])
    res[f"thirds_3streams_r{rnd}"] = measure(thirds, [main, side[0], side[1]])
print(json.dumps(res))
