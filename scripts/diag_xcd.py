"""XCD balance of one cfg3 scene (bench.py's single-scene line): per XCD, the forward's tiles and the backward's work
items -- count, summed workgroup time, first start and last end -- from the lgm_diag.render_counters timelines.
An XCD whose work ends last sets the kernel's time; bench.py's single scene runs 1,536 tiles in one round.
Usage: python scripts/diag_xcd.py -> JSON on stdout."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import CFG3_SEED  # noqa: E402
from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(1, 100000, seed=CFG3_SEED).to(dev).requires_grad_(True)
cv, cvp, cp = (t[None].contiguous().to(dev) for t in orbit_cameras(6))
d_img, _, d_alpha, bg = synthetic_upstream_grads(1, 6, 256, 256, seed=CFG3_SEED + 1000)
d_img, d_alpha, bg = d_img.to(dev), d_alpha.to(dev), bg.to(dev)
M = 6 * 256
NB = 6 * ((100000 + 511) // 512)
NI = 3 * M + 16
cnt = torch.zeros(8 + 8 * M + 8 * NB + 4 * NI, dtype=torch.int64, device=dev)
for _ in range(200):  # clocks up
    o = r.render(g, cv, cvp, cp, bg_color=bg)
    torch.autograd.backward([o["image"], o["alpha"]], [d_img, d_alpha])
    g.grad = None
res = {}
for rep in range(3):
    cnt.zero_()
    torch.cuda.synchronize()
    for _ in range(30):  # keep the clocks up right before the instrumented step
        o = r.render(g, cv, cvp, cp, bg_color=bg)
        torch.autograd.backward([o["image"], o["alpha"]], [d_img, d_alpha])
        g.grad = None
    with _native.diagnostics(render_counters=cnt):
        o = r.render(g, cv, cvp, cp, bg_color=bg)
        torch.autograd.backward([o["image"], o["alpha"]], [d_img, d_alpha])
        g.grad = None
    torch.cuda.synchronize()
    c = np.array(cnt.tolist(), dtype=np.int64)
    tl = c[8:8 + 8 * M].reshape(M, 8)
    st, en, xcc, nl = tl[:, 0], tl[:, 1], (tl[:, 7] >> 56) & 0xFF, tl[:, 6] & 0xFFFFFFFF
    t0 = st.min()
    fwd = {}
    for x in range(8):
        m = xcc == x
        fwd[x] = [int(m.sum()), round(float(((en[m] - st[m]) * 0.01).sum()), 1), round(float((st[m].min() - t0) * 0.01), 2),
                  round(float((en[m].max() - t0) * 0.01), 2), int(nl[m].sum())]
    it = c[8 + 8 * M + 8 * NB: 8 + 8 * M + 8 * NB + 4 * NI].reshape(NI, 4)
    it = it[it[:, 1] > 0]
    b0 = it[:, 0].min()
    bx = it[:, 3] & 0xFF
    bwd = {}
    for x in range(8):
        m = bx == x
        bwd[x] = [int(m.sum()), round(float(((it[m, 1] - it[m, 0]) * 0.01).sum()), 1),
                  round(float((it[m, 0].min() - b0) * 0.01), 2), round(float((it[m, 1].max() - b0) * 0.01), 2)]
    res[f"rep{rep}"] = {"fwd_per_xcd [tiles, sum_wg_us, first_start_us, last_end_us, list_entries]": fwd,
                        "fwd_span_us": round(float((en.max() - t0) * 0.01), 2),
                        "bwd_per_xcd [items, sum_item_us, first_start_us, last_end_us]": bwd,
                        "bwd_span_us": round(float((it[:, 1].max() - b0) * 0.01), 2)}
print(json.dumps(res))
