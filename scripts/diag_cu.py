"""Per-CU balance of one cfg3 scene (bench.py's single-scene line), from the lgm_diag.render_counters timelines:
for the forward's tiles and the backward's work items, per CU (XCC_ID, HW_ID SE/SH/CU bits): item count, summed list
entries (forward), summed workgroup time and last end. Says whether the kernels' ends are set by a CU whose summed
work is above the mean (an assignment imbalance an order could fix) or by one long item.
Usage: python scripts/diag_cu.py -> JSON on stdout."""
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


def step():
    o = r.render(g, cv, cvp, cp, bg_color=bg)
    torch.autograd.backward([o["image"], o["alpha"]], [d_img, d_alpha])
    g.grad = None


def per_cu(key, st, en, weight):
    """key: CU id per item; returns the per-CU table and the summary."""
    t0 = st.min()
    cus = np.unique(key)
    rows = []
    for k in cus:
        m = key == k
        rows.append((int(k), int(m.sum()), int(weight[m].sum()), float(((en[m] - st[m]) * 0.01).sum()),
                     float((en[m].max() - t0) * 0.01), float(((en[m] - st[m]) * 0.01).max())))
    a = np.array([x[1:] for x in rows], dtype=np.float64)
    last = int(np.argmax(a[:, 3]))
    return {
        "n_cu": len(rows),
        "items_per_cu [min, mean, max]": [a[:, 0].min(), round(a[:, 0].mean(), 2), a[:, 0].max()],
        "weight_per_cu [min, mean, max]": [a[:, 1].min(), round(a[:, 1].mean(), 1), a[:, 1].max()],
        "sum_wg_us_per_cu [min, mean, max]": [round(a[:, 2].min(), 1), round(a[:, 2].mean(), 1), round(a[:, 2].max(), 1)],
        "last_end_us [min, p50, p90, max]": [round(np.percentile(a[:, 3], q), 2) for q in (0, 50, 90, 100)],
        "last_cu": {"items": a[last, 0], "weight": a[last, 1], "sum_wg_us": round(a[last, 2], 1),
                    "longest_item_us": round(a[last, 4], 2), "weight_rank": int((a[:, 1] > a[last, 1]).sum())},
        "corr(weight, last_end)": round(float(np.corrcoef(a[:, 1], a[:, 3])[0, 1]), 3),
        "corr(sum_wg_us, last_end)": round(float(np.corrcoef(a[:, 2], a[:, 3])[0, 1]), 3),
        "longest_item_us": round(float(((en - st) * 0.01).max()), 2),
    }


for _ in range(200):  # clocks up
    step()
res = {}
for rep in range(3):
    cnt.zero_()
    torch.cuda.synchronize()
    for _ in range(30):
        step()
    with _native.diagnostics(render_counters=cnt):
        step()
    torch.cuda.synchronize()
    c = np.array(cnt.tolist(), dtype=np.int64)
    tl = c[8:8 + 8 * M].reshape(M, 8)
    st, en = tl[:, 0], tl[:, 1]
    xcc, hw, nl = (tl[:, 7] >> 56) & 0xFF, (tl[:, 6] >> 32) & 0xFFFFFFFF, tl[:, 6] & 0xFFFFFFFF
    fkey = xcc * 256 + ((hw >> 8) & 0xFF)
    it = c[8 + 8 * M + 8 * NB: 8 + 8 * M + 8 * NB + 4 * NI].reshape(NI, 4)
    it = it[it[:, 1] > 0]
    bkey = (it[:, 3] & 0xFF) * 256 + ((it[:, 3] >> 16) & 0xFF)
    blen = it[:, 2] & 0xFFFFF
    c_list, c_iter = tl[:, 7] & 0xFFFFFFFF, (tl[:, 7] >> 32) & 0xFFFFFF
    dur = (en - st) * 0.01
    top = np.argsort(-dur)[:6]
    res[f"rep{rep}"] = {"fwd": per_cu(fkey, st, en, nl), "bwd": per_cu(bkey, it[:, 0], it[:, 1], blen),
                        "fwd_longest [tile, us, list, staged, wave0_steps, start_us]": [
                            [int(t), round(float(dur[t]), 2), int(nl[t]), int(c_list[t]), int(c_iter[t]),
                             round(float((st[t] - st.min()) * 0.01), 2)] for t in top]}
    if rep == 0:  # per-tile raw record of one run: CU key, start / end (us), list, staged, wave-0 entries
        res["tiles_rep0 [cu_key, start_us, end_us, list, staged, wave0_entries]"] = [
            [int(fkey[t]), round(float((st[t] - st.min()) * 0.01), 2), round(float((en[t] - st.min()) * 0.01), 2),
             int(nl[t]), int(c_list[t]), int(c_iter[t])] for t in range(M)]
print(json.dumps(res))
