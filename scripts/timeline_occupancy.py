"""Occupancy of a whole-step timeline (scripts/diag_timeline.py -> gpurun_out/timeline_B{B}.npz): for k_render_bwd the
active head / checkpoint items every 20 us and the starts per 20 us, per-CU items at one instant and per-XCD totals,
and for every kernel its span against the sum of its workgroup durations over its residency slots.
    python scripts/timeline_occupancy.py [gpurun_out/timeline_B8.npz]"""
import sys
import numpy as np
z = np.load(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/timeline_B8.npz')
c = z["runs"][-1]; M, NB, NI = int(z["M"]), int(z["NB"]), int(z["NI"])
tl = c[8:8 + 8 * M].reshape(M, 8); bt = c[8 + 8 * M:8 + 8 * M + 8 * NB].reshape(NB, 8); it = c[8 + 8 * M + 8 * NB:].reshape(NI, 4)
okb = bt[:, 4] > 0; t0 = bt[okb, 0].min()
oki = it[:, 1] > 0
st = (it[oki, 0] - t0) * 0.01; en = (it[oki, 1] - t0) * 0.01
lo = (it[oki, 2] >> 20) & 0xFFFFF; head = lo == 0; ent = it[oki, 2] & 0xFFFFF
s0 = st.min(); e1 = en.max()
print('bwd span', s0, e1, e1 - s0, 'items', len(st), 'head', head.sum(), 'ck', (~head).sum())
print('sum dur head %.0f ck %.0f  -> ideal at 1024 slots %.1f us' % ((en-st)[head].sum(), (en-st)[~head].sum(), (en-st).sum()/1024))
for tt in np.arange(s0, e1, 20):
    a = ((st <= tt) & (en > tt)); 
    print('t=%6.1f active %4d (head %4d ck %4d)  starts in next 20us: head %4d ck %4d' % (tt - s0, a.sum(), (a & head).sum(), (a & ~head).sum(), ((st >= tt) & (st < tt + 20) & head).sum(), ((st >= tt) & (st < tt + 20) & ~head).sum()))
# fwd
st2 = (tl[:, 0] - t0) * 0.01; en2 = (tl[:, 1] - t0) * 0.01; ok = tl[:,1] > 0
st2, en2 = st2[ok], en2[ok]
print('fwd span %.1f ideal %.1f' % (en2.max() - st2.min(), (en2 - st2).sum() / 1792))
st3 = bt[okb,0]; en3 = bt[okb,4]
st3 = (st3 - t0)*0.01; en3 = (en3 - t0)*0.01
print('bin span %.1f ideal(512) %.1f' % (en3.max()-st3.min(), (en3-st3).sum()/512))
st4 = (tl[:, 4] - t0) * 0.01; en4 = (tl[:, 5] - t0) * 0.01; ok4 = tl[:,5]>0
print('sort span %.1f ideal(1024) %.1f' % (en4[ok4].max()-st4[ok4].min(), (en4[ok4]-st4[ok4]).sum()/1024))
okp = tl[:, 3] > 0; st5 = (tl[okp,2]-t0)*0.01; en5=(tl[okp,3]-t0)*0.01
print('preproc span %.1f ideal(1024) %.1f' % (en5.max()-st5.min(), (en5-st5).sum()/1024))
print('--- per XCD / per CU (bwd)')
x = (it[oki, 3] & 0xff).astype(int); hw = (it[oki, 3] >> 8).astype(np.int64)
# HW_ID fields (gfx9): wave_id[3:0], simd_id[5:4], pipe[7:6], cu_id[11:8], sh_id[12], se_id[15:13] (approx)
cu = (hw >> 8) & 0xf; sh = (hw >> 12) & 1; se = (hw >> 13) & 7
cuk = x * 1000 + se * 100 + sh * 16 + cu
tt = s0 + 300.0
a = (st <= tt) & (en > tt)
print('active at t=300:', a.sum())
import collections
cnt = collections.Counter(cuk[a])
vals = np.array(list(cnt.values()))
print('CUs seen active', len(cnt), 'items per CU hist', collections.Counter(vals.tolist()))
print('unique CU keys overall', len(set(cuk.tolist())))
for xx in range(8):
    print('xcd', xx, 'active', (a & (x == xx)).sum(), 'items', (x == xx).sum(), 'ck', ((x == xx) & ~head).sum(), 'end %.1f' % (en[x == xx].max() - s0), 'sumdur %.0f' % (en - st)[x == xx].sum())
