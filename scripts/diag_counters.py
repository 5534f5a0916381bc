"""Work counters of one cfg3 forward+backward (lgm_diag.render_counters) -> gpurun_out/counters.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from lgm_amd import GaussianRenderer, Options, _native  # noqa: E402
from lgm_amd.cameras import orbit_cameras  # noqa: E402
from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1  # 1: cfg3 (seed 1); 8: bench.py's pool (seed 2)
r = GaussianRenderer(Options(output_size=256))
g = synthetic_gaussians(B, 100000, seed=1 if B == 1 else 2).to(dev).requires_grad_(True)
cv, cvp, cp = (t[None].expand(B, *t.shape).contiguous().to(dev) for t in orbit_cameras(6))
d_img, _, d_alpha, bg = synthetic_upstream_grads(B, 6, 256, 256, seed=1001 if B == 1 else 1002)
M = B * 6 * 256
NB = B * 6 * ((100000 + 511) // 512)  # binning records reserved (k_bin uses the first B*ceil(6/3)*ceil(N/512): 3 views per workgroup)
NI = 12 * M + 256  # backward work-item capacity (the one-wave backward: 4 items per tile and per checkpoint slot)
cnt = torch.zeros(8 + 8 * M + 8 * NB + 4 * NI, dtype=torch.int64, device=dev)
L = _native.lib()
for _ in range(5):  # warm up (clocks, caches, code objects) before the instrumented step
    o = r.render(g, cv, cvp, cp, bg_color=bg.to(dev))
    torch.autograd.backward([o["image"], o["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
    g.grad = None
torch.cuda.synchronize()
with _native.diagnostics(render_counters=cnt):
    out = r.render(g, cv, cvp, cp, bg_color=bg.to(dev))
    torch.autograd.backward([out["image"], out["alpha"]], [d_img.to(dev), d_alpha.to(dev)])
    torch.cuda.synchronize()
c = cnt.tolist()
# [0..7] hold only the LGM_BWD_STAMPS build's backward section cycles (scripts/diag_bwd_stamps.py reads them);
# the forward no longer writes aggregate counters there (include/lgm_render.h)
res = {"bwd_section_cycles_stamps_build": c[:8]} if any(c[:8]) else {}
import numpy as np  # noqa: E402
tl = np.array(c[8:8 + 8 * M], dtype=np.int64).reshape(M, 8)
nl = tl[:, 6] & 0xFFFFFFFF
res["tile_list_max"] = int(nl.max())
res["tile_list_p50"] = float(np.median(nl))
res["tile_list_mean"] = float(nl.mean())
res["tile_list_hist_1k"] = np.bincount(nl // 1024).tolist()
for name, (a, b) in {"fwd": (0, 1), "preproc_bwd": (2, 3), "sort": (4, 5)}.items():
    st, en = tl[:, a], tl[:, b]
    ok = en > 0
    if not ok.any():  # no per-workgroup timeline for this kernel (the backward records none)
        continue
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
st7 = np.array(c[8:8 + 8 * M], dtype=np.int64).reshape(M, 8)[:, 7]
res["fwd_entries_staged"] = int((st7 & 0xFFFFFFFF).sum())  # [+7] low 32 bits per tile
res["fwd_wave0_steps"] = int(((st7 >> 32) & 0xFFFFFF).sum())  # [+7] bits 32-55
print(json.dumps(res, indent=1))
os.makedirs("gpurun_out", exist_ok=True)
json.dump(res, open(f"gpurun_out/counters_B{B}.json", "w"), indent=1)
st, en = tl[:, 4], tl[:, 5]
ok = en > 0
dur = (en - st) * 0.01 if ok.any() else np.zeros(len(st))
res2 = {}
for k in range(int(nl.max()) // 512 + 1):
    m = ok & (nl // 512 == k)
    if m.any():
        res2[f"{512 * k}-{512 * k + 511}"] = [int(m.sum()), round(float(dur[m].mean()), 2), round(float(dur[m].max()), 2)]
print("sort us by list length [tiles, mean, max]:", json.dumps(res2))
res["sort_us_by_n"] = res2
json.dump(res, open(f"gpurun_out/counters_B{B}.json", "w"), indent=1)

bt = np.array(c[8 + 8 * M: 8 + 8 * M + 8 * NB], dtype=np.int64).reshape(NB, 8)
ok = bt[:, 4] > 0
bt = bt[ok]
t0 = bt[:, 0].min()
# [1..3]: summed durations of the preprocess / tile-test / reservation phases over the workgroup's batches
tot = (bt[:, 4] - bt[:, 0]) * 0.01
phd = {"preproc": bt[:, 1] * 0.01, "tests": bt[:, 2] * 0.01, "reserve": bt[:, 3] * 0.01}
phd["emit"] = tot - phd["preproc"] - phd["tests"] - phd["reserve"]
phd["total"] = tot
binres = {k: [round(float(np.median(v)), 2), round(float(v.max()), 2)] for k, v in phd.items()}
binres["span_us"] = round(float((bt[:, 4].max() - t0) * 0.01), 2)
binres["start_spread_us"] = round(float((bt[:, 0].max() - t0) * 0.01), 2)
binres["hits_median"] = float(np.median(bt[:, 5]))
print("k_bin phases [median us, max us]:", json.dumps(binres))
res["k_bin_phases"] = binres
json.dump(res, open(f"gpurun_out/counters_B{B}.json", "w"), indent=1)

it = np.array(c[8 + 8 * M + 8 * NB: 8 + 8 * M + 8 * NB + 4 * NI], dtype=np.int64).reshape(NI, 4)
ok = it[:, 1] > 0
it = it[ok]
if len(it):
    t0 = it[:, 0].min()
    dur = (it[:, 1] - it[:, 0]) * 0.01
    ln = it[:, 2] & 0xFFFFF
    lo = (it[:, 2] >> 20) & 0xFFFFF
    tl_ = it[:, 2] >> 40
    first = lo == 0
    ir = {"items": int(len(it)), "span_us": round(float((it[:, 1].max() - t0) * 0.01), 2),
          "dur_p50": round(float(np.median(dur)), 2), "dur_max": round(float(dur.max()), 2),
          "first_seg_p50": round(float(np.median(dur[first])), 2), "first_seg_max": round(float(dur[first].max()), 2),
          "other_seg_p50": round(float(np.median(dur[~first])), 2) if (~first).any() else None,
          "sum_dur_us": round(float(dur.sum()), 1),
          "last_start_us": round(float((it[:, 0].max() - t0) * 0.01), 2)}
    order_ = np.argsort(-dur)[:8]
    ir["slowest"] = [(int(tl_[i]), int(lo[i]), int(ln[i]), round(float(dur[i]), 2), int(it[i, 3]),
                      round(float((it[i, 0] - t0) * 0.01), 2)) for i in order_]
    print("bwd items:", json.dumps(ir))
    res["bwd_items"] = ir
    json.dump(res, open(f"gpurun_out/counters_B{B}.json", "w"), indent=1)
