"""How much of k_render_bwd's per-wave work contributes: for one cfg3 scene (seed 1, as bench.py) and the oracle's
tile lists and n_contrib, per 8x8 quadrant: R = list positions before the quadrant's largest n_contrib whose
alpha >= 1/255 ellipse meets the quadrant (the backward's per-wave list; the continuous-rectangle test approximated
on a 0.25-px grid), U = those with alpha >= 1/255 at some pixel centre before that pixel's last contributor, the
8-entry batches each needs per 64-entry chunk, and the share of (entry, pixel) evaluations that contribute.
Usage: python scripts/diag_bwd_useful.py [views]  (CPU only; ~1 min per view)"""
import sys, numpy as np, math
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from lgm_amd.synthetic import synthetic_gaussians
from lgm_amd.cameras import orbit_cameras
from oracle import oracle as O
O.build()
g = synthetic_gaussians(1, 100_000, seed=1)[0].numpy()
cv, cvp, cp = orbit_cameras(6)
tan = math.tan(math.radians(49.1) / 2)
H = W = 256
tot_R = tot_U = tot_bR = tot_bU = tot_pe = 0
for v in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1):
    pre = O.preprocess(g, cv[v].numpy(), cvp[v].numpy(), tan, H, W)
    ts, ids = O.tile_lists(g, cv[v].numpy(), cvp[v].numpy(), tan, H, W)
    nc, ft, K = O.forward_state(g, cv[v].numpy(), cvp[v].numpy(), tan, H, W)
    xy = pre['xy'].astype(np.float64); co = pre['conic_opacity'].astype(np.float64)
    gx = W // 16
    for t in range(len(ts) - 1):
        lst = ids[ts[t]:ts[t + 1]]
        if len(lst) == 0: continue
        tx0, ty0 = (t % gx) * 16, (t // gx) * 16
        for q in range(4):
            qx, qy = tx0 + (q & 1) * 8, ty0 + (q >> 1) * 8
            ncq = nc[qy:qy + 8, qx:qx + 8].reshape(-1)          # per pixel last (count)
            wl = int(ncq.max())
            if wl == 0: continue
            L = lst[:wl]
            X = xy[L]; A, B, C, o = co[L, 0], co[L, 1], co[L, 2], co[L, 3]
            px = np.arange(8) + qx; py = np.arange(8) + qy
            PX, PY = np.meshgrid(px, py); PX = PX.reshape(-1); PY = PY.reshape(-1)
            dx = X[:, 0:1] - PX[None]; dy = X[:, 1:2] - PY[None]
            power = -0.5 * (A[:, None] * dx * dx + C[:, None] * dy * dy) - B[:, None] * dx * dy
            alpha = np.minimum(0.99, o[:, None] * np.exp(power))
            contrib = (power <= 0) & (alpha >= 1 / 255) & (np.arange(wl)[:, None] < ncq[None])
            U = contrib.any(1)
            # rect test: min over integer pixels of the quadrant of q = A dx^2 + 2B dx dy + C dy^2 vs tau = 2 ln(255 o)
            # (pixel-exact minimum over the 64 centres is a lower bound of the GPU's continuous-rect test)
            qf = (A[:, None] * dx * dx + 2 * B[:, None] * dx * dy + C[:, None] * dy * dy)
            tau = 2 * np.log(np.maximum(255 * o, 1e-30))
            # continuous rect: sample finer grid (0.25 px) to approximate the continuous minimum
            fx = np.arange(0, 7.01, 0.25) + qx; fy = np.arange(0, 7.01, 0.25) + qy
            FX, FY = np.meshgrid(fx, fy); FX = FX.reshape(-1); FY = FY.reshape(-1)
            ddx = X[:, 0:1] - FX[None]; ddy = X[:, 1:2] - FY[None]
            qq = (A[:, None] * ddx * ddx + 2 * B[:, None] * ddx * ddy + C[:, None] * ddy * ddy).min(1)
            R = qq <= tau
            tot_R += R.sum(); tot_U += U.sum(); tot_pe += contrib.sum()
            # batches: per 64-position chunk, ceil(cnt/8)
            for c0 in range(0, wl, 64):
                tot_bR += -(-R[c0:c0 + 64].sum() // 8); tot_bU += -(-U[c0:c0 + 64].sum() // 8)
    print('view', v, 'R (rect hits before wlast)', tot_R, 'U (contributing)', tot_U, 'ratio %.3f' % (tot_U / tot_R),
          'batches R %d U %d ratio %.3f' % (tot_bR, tot_bU, tot_bU / tot_bR), 'useful (entry,pixel) per R-entry-pixel %.3f' % (tot_pe / (64 * tot_R)), flush=True)
