"""Where the forward's tiles ran (per-tile HW_ID / XCC_ID stamps of k_render_fwd, scripts/diag_timeline.py with a
build that records them) and how the work and the durations spread over the CUs: does the longest tile share its CU
with other heavy tiles?
    python scripts/placement_report.py gpurun_out/timeline_B1_hw.npz"""
import collections
import sys

import numpy as np

z = np.load(sys.argv[1])
c = z["runs"][-1]
M = int(z["M"])
tl = c[8:8 + 8 * M].reshape(M, 8)
hw = (tl[:, 6] >> 32).astype(np.int64)
xcc = (tl[:, 7] >> 56).astype(np.int64) & 0xF
steps = (tl[:, 7] >> 32) & 0xFFFFFF
dur = (tl[:, 1] - tl[:, 0]) * 0.01
cu, sh, se, simd, slot = (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7, (hw >> 4) & 3, hw & 0xF
key = xcc * 1000 + se * 100 + sh * 16 + cu
cus = collections.defaultdict(list)
for t in range(M):
    cus[int(key[t])].append(t)
print(f"{len(cus)} distinct CUs used by {M} tiles; tiles per CU: {collections.Counter(len(v) for v in cus.values())}")
load = {k: int(steps[v].sum()) for k, v in cus.items()}
end = {k: float(dur[v].max()) for k, v in cus.items()}
ks = sorted(cus, key=lambda k: -load[k])
print("heaviest CUs (xcc.se.sh.cu: sum of wave-0 steps, longest tile us, tiles):")
for k in ks[:8]:
    print(f"  {k}: {load[k]}, {end[k]:.1f}, {[int(t) for t in cus[k]]}")
print("lightest CUs:")
for k in ks[-4:]:
    print(f"  {k}: {load[k]}, {end[k]:.1f}, {[int(t) for t in cus[k]]}")
la, ea = np.array([load[k] for k in cus]), np.array([end[k] for k in cus])
print(f"CU load (steps) mean {la.mean():.0f} max {la.max()} min {la.min()}; corr(load, longest tile) "
      f"{np.corrcoef(la, ea)[0, 1]:.2f}")
# dispatch order vs CU: block b of tile t (XCD order), consecutive blocks of one XCC
blk = np.zeros(M, np.int64)
q, r = M >> 3, M & 7
for b in range(M):
    g, i = b & 7, b >> 3
    blk[(g * (q + 1) if g < r else r * (q + 1) + (g - r) * q) + i] = b
order = np.argsort(blk)
print("first 40 blocks -> (xcc, se, sh, cu):", [(int(xcc[t]), int(se[t]), int(sh[t]), int(cu[t])) for t in order[:40]])
