"""Probe: the 8-scene scaling pool (100k Gaussians x 6 views x 256^2 per scene, fwd+bwd through the C ABI) as ONE
call vs its scenes split into halves / quarters rendered as independent calls -- on one stream (the cost of the
smaller launches) and on two streams (whether concurrent half-size chains fill each other's kernel tails and
mid-kernel hand-over gaps, DESIGN.md §4 timeline). GPU span per step from events on the main stream (the side
stream forks from and joins into it each step). scripts/probe_split.py is the same probe on one scene's views."""
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
S, N, V, R = 8, 100_000, 6, 256
g = synthetic_gaussians(S, N, seed=2).to(dev)
cv, cvp, _ = orbit_cameras(V)
cv = cv[None].expand(S, -1, -1, -1).contiguous().to(dev)
cvp = cvp[None].expand(S, -1, -1, -1).contiguous().to(dev)
d_img, _, d_alpha, bg = synthetic_upstream_grads(S, V, R, R, seed=1002)
d_img, d_alpha, bg = d_img.to(dev), d_alpha.to(dev), bg.to(dev)
tan = tan_half_fov(49.1)
OPT = 2  # LGM_RENDER_CLAMP_IMAGE


class Part:
    def __init__(self, s0, s1):
        self.B = s1 - s0
        self.g = g[s0:s1]  # (contiguous: a slice of whole scenes)
        self.cv, self.cvp = cv[s0:s1], cvp[s0:s1]
        self.di, self.da = d_img[s0:s1], d_alpha[s0:s1]
        self.ws_bytes = L.lgm_render_workspace_size_opts(self.B, V, N, R, R, 0, OPT)
        self.ws = torch.empty(self.ws_bytes, dtype=torch.uint8, device=dev)
        self.img = torch.empty(self.B, V, 3, R, R, device=dev)
        self.dep = torch.empty(self.B, V, 1, R, R, device=dev)
        self.alp = torch.empty(self.B, V, 1, R, R, device=dev)
        self.dg = torch.empty_like(self.g)

    def run(self, stream):
        st = stream.cuda_stream
        p = _native.ptr
        _native.check(L.lgm_render_forward(self.B, V, N, R, R, p(self.g), p(self.cv), p(self.cvp), p(bg), tan, tan,
                                           1.0, p(self.img), p(self.dep), p(self.alp), None, p(self.ws),
                                           self.ws_bytes, 0, None, OPT, st, None), "fwd")
        _native.check(L.lgm_render_backward(self.B, V, N, R, R, p(self.g), p(self.cv), p(self.cvp), p(bg), tan, tan,
                                            1.0, p(self.di), None, p(self.da), p(self.dg), None, p(self.ws),
                                            self.ws_bytes, 0, OPT, st, None), "bwd")


def measure(parts, streams, steps=40):
    main = torch.cuda.current_stream()

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
    for _ in range(20):
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
side = torch.cuda.Stream(device=dev)
full = [Part(0, 8)]
halves = [Part(0, 4), Part(4, 8)]
res = {}
for rnd in range(2):
    res[f"full_r{rnd}"] = measure(full, [main])
    res[f"halves_1stream_r{rnd}"] = measure(halves, [main])
    res[f"halves_2streams_r{rnd}"] = measure(halves, [main, side])
    print(json.dumps(res), flush=True)
# the halves' gradients against the full call's (float atomics: equal to rounding)
ref = full[0].dg
got = torch.cat([pt.dg for pt in halves])
res["halves_vs_full_rel_l2"] = float((got - ref).norm() / ref.norm())
print(json.dumps(res), flush=True)
