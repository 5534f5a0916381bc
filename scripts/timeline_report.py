"""Report on a whole-step timeline (scripts/diag_timeline.py -> gpurun_out/timeline_B{B}.npz): per kernel the span,
the gap before it, how many workgroups run over time (in 5 % slices of the span), the longest workgroups and,
for the backward, head items vs checkpoint items.
    python scripts/timeline_report.py gpurun_out/timeline_B1.npz [run]"""
import sys

import numpy as np

z = np.load(sys.argv[1])
run = int(sys.argv[2]) if len(sys.argv) > 2 else -1
c = z["runs"][run]
M, NB, NI = int(z["M"]), int(z["NB"]), int(z["NI"])
tl = c[8:8 + 8 * M].reshape(M, 8)
bt = c[8 + 8 * M:8 + 8 * M + 8 * NB].reshape(NB, 8)
it = c[8 + 8 * M + 8 * NB:].reshape(NI, 4)
okb = bt[:, 4] > 0
t0 = bt[okb, 0].min()
ks = {"bin": (bt[okb, 0], bt[okb, 4], None), "sort": (tl[:, 4], tl[:, 5], tl[:, 6] & 0xFFFFFFFF),
      "fwd": (tl[:, 0], tl[:, 1], tl[:, 7] & 0xFFFFFFFF)}
oki = it[:, 1] > 0
ks["bwd"] = (it[oki, 0], it[oki, 1], it[oki, 2] & 0xFFFFF)
okp = tl[:, 3] > 0
ks["preproc_bwd"] = (tl[okp, 2], tl[okp, 3], None)
prev_end = None
for name, (st, en, w) in ks.items():
    ok = en > 0
    st, en = (st[ok] - t0) * 0.01, (en[ok] - t0) * 0.01
    dur = en - st
    span0, span1 = st.min(), en.max()
    gap = span0 - prev_end if prev_end is not None else 0.0
    prev_end = span1
    # active workgroups in 20 slices of the span
    edges = np.linspace(span0, span1, 21)
    mids = 0.5 * (edges[:-1] + edges[1:])
    active = [int(((st <= m) & (en > m)).sum()) for m in mids]
    print(f"{name:12s} start {span0:7.2f} end {span1:7.2f} span {span1 - span0:7.2f} us  gap-before {gap:5.2f}  "
          f"wgs {len(st)}  dur p50 {np.median(dur):6.2f} p90 {np.percentile(dur, 90):6.2f} max {dur.max():6.2f}  "
          f"sum {dur.sum():9.1f}  last-start {st.max() - span0:6.2f}")
    print(f"{'':12s} active per 5% slice: {active}")
    if name == "bwd":
        lo = (it[oki, 2] >> 20) & 0xFFFFF
        head = lo[ok] == 0
        print(f"{'':12s} head items {head.sum()} dur p50 {np.median(dur[head]):.2f} max {dur[head].max():.2f} "
              f"start-max {st[head].max() - span0:.2f} | ck items {(~head).sum()} dur p50 "
              f"{np.median(dur[~head]) if (~head).any() else 0:.2f} start-min "
              f"{(st[~head].min() - span0) if (~head).any() else 0:.2f}")
        # items ending last: what are they
        order = np.argsort(-en)[:10]
        tile = (it[oki, 2] >> 40)[ok]
        print(f"{'':12s} last to end (tile, chunk, entries, start, dur):",
              [(int(tile[i]), int(lo[ok][i]), int(w[ok][i]), round(float(st[i] - span0), 1), round(float(dur[i]), 1))
               for i in order])
    if name == "fwd":
        order = np.argsort(-dur)[:8]
        idx = np.nonzero(ok)[0]
        print(f"{'':12s} longest (tile, staged, steps_w0, dur):",
              [(int(idx[i]), int(w[ok][i]), int((tl[idx[i], 7] >> 32) & 0xFFFFFF), round(float(dur[i]), 1)) for i in order])
    if name == "sort":
        order = np.argsort(-en)[:8]
        idx = np.nonzero(ok)[0]
        print(f"{'':12s} last to end (tile, n, start, dur):",
              [(int(idx[i]), int(w[ok][i]), round(float(st[i] - span0), 1), round(float(dur[i]), 1)) for i in order])
print(f"step (bin start -> preproc_bwd end): {prev_end:.2f} us")
