// lgm_amd/csrc/render_bin.hip -- per-(view, Gaussian) preprocess + tile binning + per-tile depth sort.
//
// Replaces upstream's preprocess -> InclusiveSum -> D2H(num_rendered) -> duplicateWithKeys -> 41-bit global LSD
// radix sort -> identifyTileRanges, once per (b, v), with one launch sequence over all
// B x V views and no host synchronisation:
//   k_bin<EMIT_SLOT>   preprocess + emit each Gaussian's (depth_bits << 32 | id) key into the slot bucket of every
//                      tile it can reach (LDS tile histogram -> one global atomic reservation per touched tile per
//                      workgroup -> LDS-local positions). Slot buckets need no count pass and no scan.
//   k_bin<COUNT>/k_scan/k_bin<EMIT_PACKED>   the same with exact packing (large workloads).
//   k_sort             one workgroup per tile: one MSD bucket pass on the top 11 bits of the tile's depth span,
//                      then each entry ranked inside its (small) bucket on (depth, id); clustered depths fall back
//                      to LDS LSD radix passes (wave ballot multisplit ranks, per-wave chunks => stable). Ties are
//                      ordered by Gaussian id, which is exactly upstream's order: its LSD sort is stable on
//                      index-ordered pairs. Buckets > RS_CAP (4032) use an in-place bitonic network on the u64
//                      composite key (LDS blocks + global merge stages).
#include "render_common.h"

namespace lgm {
namespace {

enum BinMode { COUNT = 0, EMIT_SLOT = 1, EMIT_PACKED = 2 };

// Inclusive wavefront scans on the DPP network (row shifts inside each 16-lane row, then the row_bcast:15 /
// row_bcast:31 carries across rows): VALU only, no LDS permute round trips. A lane whose DPP source does not
// exist takes `old` (the operation's identity).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dpp_src(int old, int v) {
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, 0xf, false);
}
__device__ __forceinline__ int wave_incl_scan(int x, int /*lane*/) {
    x += dpp_src<0x111>(0, x);       // row_shr:1
    x += dpp_src<0x112>(0, x);       // row_shr:2
    x += dpp_src<0x114>(0, x);       // row_shr:4
    x += dpp_src<0x118>(0, x);       // row_shr:8
    x += dpp_src<0x142, 0xa>(0, x);  // row_bcast:15 into rows 1, 3
    x += dpp_src<0x143, 0xc>(0, x);  // row_bcast:31 into rows 2, 3
    return x;
}

// ------------------------------------------------------------------------------------------------------------
// k_bin: grid (ceil(N / BIN_G), B * ceil(V / BIN_ITERS)), block BIN_THREADS, one Gaussian per thread; the workgroup
// bins its BIN_G Gaussians into BIN_ITERS views of one scene, one view (batch) after the other. A workgroup's LDS
// tile histogram aggregates its BIN_G Gaussians before one global reservation per touched tile of the view.
//
// Load balance: a Gaussian's work is the tile rows of its candidate rectangle (1 to tens). Each wavefront
// flattens the rows of its 64 Gaussians into one list and takes 64 at a time (lane -> (Gaussian, row); the owner
// Gaussian found by a head-flag max-scan), so no lane idles behind a large Gaussian; a lane computes its row's exact
// tile range (BinRec) and records the hits in an LDS hit list with their rank in the tile (returned by the
// histogram atomic). The emission after the global reservation is a flat loop over that list.
// A workgroup's BIN_ITERS batches are BIN_ITERS VIEWS of the same BIN_G Gaussians: each Gaussian row is loaded once
// per workgroup instead of once per view (pool 199 -> 193 us, single scene 40.6 -> 38.8 us; 1 / 2 / 6 views per
// workgroup measured slower).
constexpr int BIN_THREADS = 512, BIN_G = BIN_THREADS, BIN_ITERS = 3;
constexpr int BIN_HITCAP = BIN_THREADS * 6;  // hit-list capacity (typical: ~4 hits per Gaussian)
static_assert(BIN_THREADS <= 512, "owner index packs into 9 bits");

// One Gaussian's emit record in LDS (48 B). The tiles a Gaussian can reach are found ROW BY ROW: for the tile row's
// pixel band dy in [dy0, dy0 + BY - 1] the culling ellipse q = A dx^2 + 2B dx dy + C dy^2 <= tau spans
//   x in [x - kB e' - sqrt(k0 - k1 e'^2), x - kB e + sqrt(k0 - k1 e^2)],
//   kB = B / A, k0 = tau / A, k1 = det / A^2, e = clamp(dys, band), e' = clamp(-dys, band),
// where dys = -B hx / C is the dy of the ellipse's rightmost point (hx = sqrt(tau C / det)): the exact x-extent of
// (ellipse ∩ band), so the row's tiles are one contiguous range -- the same tiles as testing every candidate tile's
// rectangle (ellipse_hits_rect), at one evaluation per row instead of per tile. Never-culled Gaussians (tau >= 3e38)
// take k0 = inf: whole rows of the 3-sigma rect.
struct BinRec {
    float x, y, kB, k0, k1, dys, mg;  // mg: conservative margin (pixels) added on both sides
    unsigned c0;                      // cx0 | cy0 << 16
    unsigned cx1;
    unsigned pad_;
    unsigned long long key;
};

__device__ __forceinline__ int wave_incl_max(int v, int /*lane*/) {
    constexpr int LO = -2147483647 - 1;
    v = max(v, dpp_src<0x111>(LO, v));
    v = max(v, dpp_src<0x112>(LO, v));
    v = max(v, dpp_src<0x114>(LO, v));
    v = max(v, dpp_src<0x118>(LO, v));
    v = max(v, dpp_src<0x142, 0xa>(LO, v));
    v = max(v, dpp_src<0x143, 0xc>(LO, v));
    return v;
}

// k_sort's tile order: the tiles of a view by distance from the image centre, nearest first.
// The centre tiles carry the longest lists (the object sits in the middle of the frame), so with the views
// interleaved (workgroup b sorts rank b / BV of view b % BV) the long sorts start in the first residency round and
// the short ones fill the second. One binning workgroup writes it at its end: a counting sort of the tiles on their
// squared centre distance quantised to min(T, BIN_THREADS) buckets, in LDS (hk: >= that + RS-wave sums ints). Ties
// take atomic slots -- the order only schedules the sorts, every order gives the same result.
__device__ void center_order(int gx, int T, int *__restrict__ corder, int *hk) {
    const int gy = (T + gx - 1) / gx, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int K = min(T, BIN_THREADS);
    const long long maxkey = (long long)(gx - 1) * (gx - 1) + (long long)(gy - 1) * (gy - 1);
    auto key = [&](int t) {
        const int y = t / gx, x = t - y * gx, dx = 2 * x - (gx - 1), dy = 2 * y - (gy - 1);
        return maxkey ? (int)(((long long)dx * dx + (long long)dy * dy) * (K - 1) / maxkey) : 0;
    };
    __syncthreads();  // (hk is the binning histogram's LDS)
    if (tid < K) hk[tid] = 0;
    __syncthreads();
    for (int t = tid; t < T; t += BIN_THREADS) atomicAdd(&hk[key(t)], 1);
    __syncthreads();
    const int v = tid < K ? hk[tid] : 0;
    const int incl = wave_incl_scan(v, lane);
    if (lane == 63) hk[K + w] = incl;
    __syncthreads();
    int run = incl - v;
    for (int ww = 0; ww < w; ww++) run += hk[K + ww];
    __syncthreads();
    if (tid < K) hk[tid] = run;
    __syncthreads();
    for (int t = tid; t < T; t += BIN_THREADS) corder[atomicAdd(&hk[key(t)], 1)] = t;
}

template <int MODE>
__global__ __launch_bounds__(BIN_THREADS) void k_bin(Dims d, const float *__restrict__ gauss, const float *__restrict__ views,
                                                     const float *__restrict__ projs, float4 *__restrict__ gP,
                                                     float4 *__restrict__ gQ,
                                                     uint2 *__restrict__ rects, int *__restrict__ radii_out,
                                                     int *__restrict__ tile_count, const int *__restrict__ tile_start,
                                                     unsigned long long *__restrict__ pairs, long long slot_stride,
                                                     unsigned long long *__restrict__ misc, float *__restrict__ accum,
                                                     int *__restrict__ corder) {
    extern __shared__ int hist[];  // [T] per-tile hit counts, [T] reserved global bases, [T] fallback cursors
    __shared__ BinRec srec[BIN_THREADS];
    __shared__ int sHead[BIN_THREADS], sExcl[BIN_THREADS];
    __shared__ unsigned sHit[BIN_HITCAP];         // owner | tile << 9
    __shared__ unsigned short sRank[BIN_HITCAP];  // rank of the hit within its tile (this workgroup)
    __shared__ int s_nhit;
    __shared__ unsigned long long s_tot[2];
    const int T = d.T, tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int vgroups = (d.V + BIN_ITERS - 1) / BIN_ITERS;
    const int b = blockIdx.y / vgroups, vg0 = (blockIdx.y - b * vgroups) * BIN_ITERS;
    int bv = b * d.V + vg0;  // the batch's view (updated per batch; `dest` reads it by reference)
    const bool lds = T <= LDS_HIST_MAX;
    int *hbase = hist + T, *fill = hist + 2 * T;
    int *cur = tile_count + (size_t)bv * T;
    if (tid < 2) s_tot[tid] = 0;
    auto dest = [&](int t, int pos) -> long long {
        return (MODE == EMIT_SLOT ? ((long long)bv * T + t) * slot_stride
                                  : (long long)tile_start[(size_t)bv * T + t]) + pos;
    };
    // diagnostics: per-workgroup phase stamps after the per-tile records (see lgm_diag.render_counters)
    unsigned long long *stamp = d.counters ? d.counters + 8 + 8 * (size_t)d.BV * T +
                                             8 * ((size_t)blockIdx.y * gridDim.x + blockIdx.x)
                                           : nullptr;
    // (stamps: [0] start, [1..3] the summed durations of the preprocess, tile-test and reservation phases over the
    // batches, [4] end, [5] the last batch's hits)
    unsigned long long t_ph = 0, ph_acc[3] = {0, 0, 0};
    if (stamp && tid == 0) stamp[0] = t_ph = __builtin_amdgcn_s_memrealtime();
    auto phase = [&](int k) {
        if (stamp && tid == 0) {
            const unsigned long long t = __builtin_amdgcn_s_memrealtime();
            if (k >= 0) ph_acc[k] += t - t_ph;
            t_ph = t;
        }
    };
    // BIN_ITERS batches per workgroup, one after the other: fewer, longer workgroups (2 per CU: 106 VGPRs at 8 waves
    // per workgroup) fit the single scene's launch into one round of residency. The batches are views of the same
    // Gaussians, whose rows are loaded once.
    const int i = blockIdx.x * BIN_G + tid;
    float g[14];
    if (i < d.N) load_gaussian(gauss + ((size_t)b * d.N + i) * 14, g);
    for (int it = 0; it < BIN_ITERS; it++) {
    if (vg0 + it >= d.V) break;  // workgroup-uniform (the last view group of a scene may be short)
    bv = b * d.V + vg0 + it;
    cur = tile_count + (size_t)bv * T;
    if (tid == 0) s_nhit = 0;
    if (lds)
        for (int t = tid; t < T; t += BIN_THREADS) hist[t] = 0;
    // ---- preprocess, one Gaussian per thread
    Geo o;
    bool vis = false;
    if (i < d.N) {
        vis = preprocess_one(g, views + 16 * bv, projs + 16 * bv, d, o);
        if (MODE != COUNT) {
            const size_t k = (size_t)bv * d.N + i;
            if (vis) {
                const float4 rp = rec_p(o.x, o.y, o.A, o.B), rq = rec_q(o.C, o.opacity, o.tau, o.depth);
                gP[k] = rp;  // pre-scaled compositing records (render_common.h)
                gQ[k] = rq;
                const bool side = !(d.options & LGM_RENDER_DETERMINISTIC) && rec_needle(rp.z, rp.w, rq.x);
                rects[k] = make_uint2((unsigned)o.x0 | ((unsigned)o.y0 << 16),
                                      (unsigned)o.x1 | ((unsigned)o.y1 << 16) | (side ? 0x80000000u : 0u));
                if (side) {  // the record's fp64 conic accumulators (acc_side_offset)
                    double *sd = reinterpret_cast<double *>(accum + acc_side_offset(d.B, d.V, d.N)) + k * 3;
                    sd[0] = 0.0; sd[1] = 0.0; sd[2] = 0.0;
                }
            } else {
                gP[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                gQ[k] = make_float4(0.f, -INFINITY, -1.f, 0.f);
                rects[k] = make_uint2(0u, 0u);
            }
            if (radii_out) radii_out[k] = vis ? o.radius : 0;
        }
    }
    int nc = 0;
    unsigned long long nref = 0;
    if (vis) {
        BinRec r;
        r.x = o.x; r.y = o.y;
        const float detq = o.A * o.C - o.B * o.B;
        if (o.tau >= 3.0e38f || !(detq > 0.f) || !(o.A > 0.f) || !(o.C > 0.f)) {  // never culled: whole rows
            r.kB = 0.f; r.k0 = INFINITY; r.k1 = 0.f; r.dys = 0.f; r.mg = 0.f;
        } else {
            // (1-ulp reciprocals: the interval ends carry the margin mg, far above their rounding)
            const float iA = __builtin_amdgcn_rcpf(o.A);
            r.kB = o.B * iA;
            r.k0 = fmaxf(o.tau, 0.f) * iA;
            r.k1 = detq * iA * iA;
            const float hxe = sqrtf(fmaxf(o.tau, 0.f) * o.C * __builtin_amdgcn_rcpf(detq));
            r.dys = -o.B * hxe * __builtin_amdgcn_rcpf(o.C);
            r.mg = 1e-3f * hxe + 1e-2f;  // >> the fp32 error of the interval ends (sqrt cancellation at the edge)
        }
        r.c0 = (unsigned)o.cx0 | ((unsigned)o.cy0 << 16);
        r.cx1 = (unsigned)o.cx1;
        r.key = ((unsigned long long)__float_as_uint(o.depth) << 32) | (unsigned)i;
        srec[tid] = r;
        nc = o.cx1 > o.cx0 ? o.cy1 - o.cy0 : 0;  // candidate tile rows
        nref = (unsigned long long)((o.x1 - o.x0) * (o.y1 - o.y0));
    }
#pragma unroll
    for (int o2 = 32; o2 > 0; o2 >>= 1) nref += __shfl_xor(nref, o2, 64);
    if (lane == 0 && nref) atomicAdd(&s_tot[1], nref);
    // ---- flattened (Gaussian, tile row) items of the wavefront: each lane finds its row's tile range
    const int incl = wave_incl_scan(nc, lane), excl = incl - nc;
    const int total = __builtin_amdgcn_readlane(incl, 63);
    sExcl[tid] = excl;
    __syncthreads();  // histogram zeroed; records and exclusive offsets visible
    phase(0);
    unsigned long long nemit = 0;  // wave-uniform
    // Pass 0: histogram (LDS rank per hit) + the hit list (or, without the LDS histogram, direct emission). Pass 1
    // (only after a hit-list overflow -- a dense batch, e.g. 512^2 views where a Gaussian covers ~10 tiles): the
    // same rows again, each hit emitted at hbase[t] + an LDS fill rank.
    auto flat_tests = [&](int pass) {
    int carry = 0;
    for (int base0 = 0; base0 < total; base0 += 64) {
        sHead[tid] = -1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (nc > 0 && excl >= base0 && excl < base0 + 64) sHead[w * 64 + excl - base0] = lane;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        int v = sHead[tid];
        if (lane == 0 && v < 0) v = carry;
        v = wave_incl_max(v, lane);
        carry = __builtin_amdgcn_readlane(v, 63);
        const int c = base0 + lane;
        int ta = 0, cnt = 0, trow = 0, owner = 0;
        if (c < total) {
            owner = w * 64 + v;
            const BinRec &e = srec[owner];
            const int ty = (int)(e.c0 >> 16) + (c - sExcl[owner]);
            const float dy0 = (float)(ty * BY) - e.y, dy1 = dy0 + (float)(BY - 1);
            const float e1 = fminf(fmaxf(e.dys, dy0), dy1), e2 = fminf(fmaxf(-e.dys, dy0), dy1);
            const float xh = e.x - e.kB * e1 + sqrtf(fmaxf(e.k0 - e.k1 * e1 * e1, 0.f)) + e.mg;
            const float xl = e.x - e.kB * e2 - sqrtf(fmaxf(e.k0 - e.k1 * e2 * e2, 0.f)) - e.mg;
            // tiles [BX t, BX t + BX - 1] meeting [xl, xh], within the candidate rect
            const int cx0 = (int)(e.c0 & 0xffffu), cx1 = (int)e.cx1;
            const float fa = ceilf((xl - (float)(BX - 1)) * (1.0f / BX)), fb = floorf(xh * (1.0f / BX)) + 1.f;
            ta = (int)fminf(fmaxf(fa, (float)cx0), (float)cx1);  // (float clamps: +-inf and NaN safe)
            const int tb = (int)fminf(fmaxf(fb, (float)ta), (float)cx1);
            cnt = tb - ta;
            trow = ty * d.gx;
        }
        if (pass == 1) {
            for (int k = 0; k < cnt; k++) {
                const int t = trow + ta + k;
                pairs[dest(t, hbase[t] + atomicAdd(&fill[t], 1))] = srec[owner].key;
            }
            continue;
        }
        const int hincl = wave_incl_scan(cnt, lane);
        const int htot = __builtin_amdgcn_readlane(hincl, 63);
        nemit += (unsigned)htot;
        if (!htot) continue;
        if (lds) {
            int slot0 = 0;
            if (MODE != COUNT && lane == 0) slot0 = atomicAdd(&s_nhit, htot);
            slot0 = __builtin_amdgcn_readlane(slot0, 0) + hincl - cnt;
            for (int k = 0; k < cnt; k++) {
                const int t = trow + ta + k;
                const int rk = atomicAdd(&hist[t], 1);
                if (MODE != COUNT) {
                    const int slot = slot0 + k;
                    if (slot < BIN_HITCAP) {
                        sHit[slot] = (unsigned)owner | ((unsigned)t << 9);
                        sRank[slot] = (unsigned short)rk;
                    }
                }
            }
        } else {
            for (int k = 0; k < cnt; k++) {
                const int t = trow + ta + k;
                const int pos = atomicAdd(&cur[t], 1);
                if (MODE != COUNT) pairs[dest(t, pos)] = srec[owner].key;
            }
        }
    }
    };
    flat_tests(0);
    if (lane == 0 && nemit) atomicAdd(&s_tot[0], nemit);
    if (lds) {
        __syncthreads();
        phase(1);
        for (int t = tid; t < T; t += BIN_THREADS) {
            const int c = hist[t];
            if (c) {
                if (MODE == COUNT) atomicAdd(&cur[t], c);
                else hbase[t] = atomicAdd(&cur[t], c);
            }
            fill[t] = 0;
        }
        __syncthreads();
        phase(2);
        if (MODE != COUNT) {
            const int H = s_nhit;
            if (H <= BIN_HITCAP) {
                for (int h = tid; h < H; h += BIN_THREADS) {
                    const unsigned e2 = sHit[h];
                    const int t = (int)(e2 >> 9);
                    pairs[dest(t, hbase[t] + sRank[h])] = srec[e2 & 511u].key;
                }
            } else {
                flat_tests(1);  // hit-list overflow: the wave's tests again, emitting with LDS fill ranks
            }
        }
    }
    __syncthreads();
    phase(-1);  // (the emit phase: the rest of the batch)
    if (stamp && tid == 0) {
        stamp[1] = ph_acc[0];
        stamp[2] = ph_acc[1];
        stamp[3] = ph_acc[2];
        stamp[4] = t_ph;
        stamp[5] = (unsigned long long)s_nhit;
        stamp[6] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID (SE / CU / SIMD / wave slot)
        stamp[7] = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
    }
    }  // batches
    if (tid == 0) {
        atomicAdd(&misc[0], s_tot[0]);
        atomicAdd(&misc[1], s_tot[1]);
    }
    if (corder && blockIdx.x == 0 && blockIdx.y == 0) center_order(d.gx, T, corder, hist);
}

// k_scan: one workgroup of 1024 threads; exclusive scan of the M tile counts -> tile_start[0..M].
__global__ __launch_bounds__(1024) void k_scan(const int *__restrict__ count, int M, int *__restrict__ start) {
    __shared__ long long wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (M + 1023) / 1024;
    const int lo = min(M, tid * per), hi = min(M, lo + per);
    long long s = 0;
    for (int i = lo; i < hi; i++) s += count[i];
    long long x = s;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const long long y = __shfl_up(x, dd, 64);
        if (lane >= dd) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (wid == 0) {
        long long w = lane < 16 ? wsum[lane] : 0;
#pragma unroll
        for (int dd = 1; dd < 16; dd <<= 1) {
            const long long y = __shfl_up(w, dd, 64);
            if (lane >= dd) w += y;
        }
        if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    long long run = x - s + (wid > 0 ? wsum[wid - 1] : 0);
    for (int i = lo; i < hi; i++) {
        start[i] = (int)run;
        run += count[i];
    }
    if (tid == 1023) start[M] = (int)wsum[15];
}

// ------------------------------------------------------------------------------------------------------------
// Per-tile sort: up to RS_CAP entries sorted in LDS (larger buckets take sort_oversized): u32 keys, u16 bucket
// positions and per-wave 512-bucket counters; 8 rows per lane.
// RS_CAP is 4032, not 4096: the workgroup's whole LDS (the dynamic image, RS_CAP * 8 + 8 KB on the MSD path, plus
// ~400 B of static __shared__) must stay <= 40 KB for 4 workgroups per CU (160 KB). At 4096 it was 41,360 B and
// the kernel ran 3 per CU; lists of 4033..4096 entries now take the (rare) oversized path.
constexpr int RS_THREADS = 512, RS_WAVES = RS_THREADS / 64, RS_CAP = 4032,
              RS_MAXR = (RS_CAP + RS_THREADS - 1) / RS_THREADS;
constexpr int RS_OBLK = 4096;  // sort_oversized's LDS block (a power of two), u64 keys over the image
static_assert(RS_CAP <= RS_OBLK && RS_CAP % 64 == 0, "sort image layout");
constexpr int RS_DBITS = 9, RS_B = 1 << RS_DBITS;  // digit width: a typical 26-bit depth span takes 3 passes
typedef unsigned short RsCnt;  // per-wave digit counters as u16 (they never exceed RS_CAP): halves their LDS
// (the MSD path below takes RS_CAP * 8 + 2048 * 4 bytes of the same block)
constexpr int RS_LDS_LSD = RS_CAP * 4 + RS_CAP * 2 + RS_WAVES * RS_B * (int)sizeof(RsCnt);
constexpr int RS_LDS = RS_LDS_LSD > RS_CAP * 8 + 2048 * 4 ? RS_LDS_LSD : RS_CAP * 8 + 2048 * 4;
static_assert(RS_CAP < 65536, "u16 counters");
static_assert(RS_LDS >= RS_OBLK * 8, "sort_oversized reuses the image as u64[RS_OBLK]");
static_assert(RS_LDS + 512 <= 160 * 1024 / 4, "4 sort workgroups per CU (with the static __shared__ words)");
static_assert(RS_B % RS_THREADS == 0 || RS_THREADS % RS_B == 0, "bucket scan layout");

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// Lanes of the wavefront holding the same nbits-bit digit as this lane (restricted to valid lanes).
__device__ __forceinline__ unsigned long long match_digit(unsigned dgt, bool valid, int nbits) {
    unsigned long long peers = __ballot(valid);
    for (int b = 0; b < nbits; b++) {
        const bool bit = (dgt >> b) & 1u;
        const unsigned long long m = __ballot(bit);
        peers &= bit ? m : ~m;
    }
    return peers;
}

__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    return v;
}
__device__ __forceinline__ unsigned wave_max_u32(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, (unsigned)__shfl_xor((int)v, o, 64));
    return v;
}

// One stable LSD pass over the nbits-bit digit (kr >> shift) of the per-wave chunks held in registers, writing the permuted keys / bucket positions to sk / sp. Ranks come from ballot
// matching (one leader per digit updates the wave's counter: no contended LDS atomics) and are kept in registers
// for the scatter. All threads of the block call it.
__device__ __forceinline__ void radix_pass(const unsigned (&kr)[RS_MAXR], const unsigned short (&pr)[RS_MAXR],
                                          int shift, int nbits, int n, int c0, int R, unsigned *sk,
                                          unsigned short *sp, RsCnt *cnt, int *s_wsum) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const unsigned mask = (1u << nbits) - 1u;
    RsCnt *my = cnt + w * RS_B;
    for (int q = lane; q < RS_B; q += 64) my[q] = 0;
    const unsigned long long lt = lanemask_lt(lane);
    int lr[RS_MAXR];
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        lr[r] = 0;
        if (r < R) {
            const int e = c0 + r * 64 + lane;
            const bool valid = e < n;
            const unsigned dgt = (kr[r] >> shift) & mask;
            const unsigned long long peers = match_digit(dgt, valid, nbits);
            if (valid) {
                const int rk = __popcll(peers & lt);
                const int b0 = my[dgt];  // same address for all peers: broadcast read
                lr[r] = b0 + rk;
                if (rk == 0) my[dgt] = (RsCnt)(b0 + __popcll(peers));
            }
        }
    }
    __syncthreads();
    // exclusive bases, bucket-major then wave: base(w, d) = sum_{d' < d} total(d') + sum_{w' < w} cnt[w'][d]
    constexpr int BPT = RS_B / RS_THREADS > 0 ? RS_B / RS_THREADS : 1;  // buckets per thread (contiguous)
    int tot = 0;
    if (tid * BPT < RS_B) {
#pragma unroll
        for (int j = 0; j < BPT; j++)
            for (int ww = 0; ww < RS_WAVES; ww++) tot += cnt[ww * RS_B + tid * BPT + j];
    }
    const int incl = wave_incl_scan(tot, lane);
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    if (tid * BPT < RS_B) {
        int run = incl - tot;
        for (int ww = 0; ww < w; ww++) run += s_wsum[ww];
#pragma unroll
        for (int j = 0; j < BPT; j++)
            for (int ww = 0; ww < RS_WAVES; ww++) {
                const int x = cnt[ww * RS_B + tid * BPT + j];
                cnt[ww * RS_B + tid * BPT + j] = (RsCnt)run;
                run += x;
            }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        if (r < R) {
            const int e = c0 + r * 64 + lane;
            if (e < n) {
                const int pos = my[(kr[r] >> shift) & mask] + lr[r];
                sk[pos] = kr[r];
                sp[pos] = pr[r];
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void cas64(unsigned long long *s, int lo, int hi) {
    const unsigned long long a = s[lo], b = s[hi];
    if (a > b) { s[lo] = b; s[hi] = a; }
}

// Buckets larger than RS_CAP: bitonic network ("flip + half-cleaner" form, all comparators ascending, entries at
// index >= n act as +inf) on the u64 composite keys in place: LDS blocks of RS_OBLK for short distances, global
// memory for long ones. Rare (only huge central tiles); correct for any n.
__device__ void sort_oversized(unsigned long long *seg, int n, unsigned long long *sk) {
    const int C = RS_OBLK;
    int m = 1;
    while (m < n) m <<= 1;
    for (int c0 = 0; c0 < n; c0 += C) {  // sort each LDS block
        const int nb = min(C, n - c0);
        for (int q = threadIdx.x; q < nb; q += blockDim.x) sk[q] = seg[c0 + q];
        __syncthreads();
        for (int k = 2; k <= C; k <<= 1) {
            for (int p = threadIdx.x; p < (C >> 1); p += blockDim.x) {
                const int half = k >> 1, lo = (p / half) * k + (p % half), hi = lo ^ (k - 1);
                if (hi < nb) cas64(sk, lo, hi);
            }
            __syncthreads();
            for (int j = k >> 2; j > 0; j >>= 1) {
                for (int p = threadIdx.x; p < (C >> 1); p += blockDim.x) {
                    const int lo = 2 * p - (p & (j - 1)), hi = lo + j;
                    if (hi < nb) cas64(sk, lo, hi);
                }
                __syncthreads();
            }
        }
        for (int q = threadIdx.x; q < nb; q += blockDim.x) seg[c0 + q] = sk[q];
        __syncthreads();
    }
    for (int k = 2 * C; k <= m; k <<= 1) {
        for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
            const int half = k >> 1, lo = (p / half) * k + (p % half), hi = lo ^ (k - 1);
            if (hi < n) cas64(seg, lo, hi);
        }
        __syncthreads();
        for (int j = k >> 2; j >= C; j >>= 1) {
            for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
                const int lo = 2 * p - (p & (j - 1)), hi = lo + j;
                if (hi < n) cas64(seg, lo, hi);
            }
            __syncthreads();
        }
        for (int c0 = 0; c0 < n; c0 += C) {
            const int nb = min(C, n - c0);
            for (int q = threadIdx.x; q < nb; q += blockDim.x) sk[q] = seg[c0 + q];
            __syncthreads();
            for (int j = C >> 1; j > 0; j >>= 1) {
                for (int p = threadIdx.x; p < (C >> 1); p += blockDim.x) {
                    const int lo = 2 * p - (p & (j - 1)), hi = lo + j;
                    if (hi < nb) cas64(sk, lo, hi);
                }
                __syncthreads();
            }
            for (int q = threadIdx.x; q < nb; q += blockDim.x) seg[c0 + q] = sk[q];
            __syncthreads();
        }
    }
    // ids in place: u32 id i lives in u64 slot i/2; chunk c's writes only touch slots of chunks <= c (already read)
    unsigned *ids = reinterpret_cast<unsigned *>(seg);
    unsigned *sid = reinterpret_cast<unsigned *>(sk);
    for (int c0 = 0; c0 < n; c0 += C) {
        const int nb = min(C, n - c0);
        for (int q = threadIdx.x; q < nb; q += blockDim.x) sid[q] = (unsigned)seg[c0 + q];
        __syncthreads();
        for (int q = threadIdx.x; q < nb; q += blockDim.x) ids[c0 + q] = sid[q];
        __syncthreads();
    }
}

// MSD bucket sort of one tile (the common case): ONE histogram / scan / scatter pass on the top MSD_BITS bits of
// the tile's depth-key span (2048 buckets: ~1 entry per bucket at the typical 1.5k-entry list), then every entry
// takes its final position = bucket start + its rank among the bucket's entries on (key, id), found by one thread
// scanning the (few) bucket entries in LDS -- no serial insertion chains, no further passes. Exact and stable by
// construction (equal keys share a bucket and are ranked by id), so the result is upstream's order, written as
// ids straight into the tile's range. Returns false -- nothing written -- when some bucket holds more than
// MSD_LIMIT entries (clustered depths, e.g. a flat layer facing the camera); the caller then runs the LSD passes.
// LDS: (key, id) u64 entries [RS_CAP] over the image, counters hc [MSD_B] u32 (40 KB: 4 workgroups per CU, as the
// 64-VGPR cap allows anyway).
constexpr int MSD_BITS = 11, MSD_B = 1 << MSD_BITS, MSD_LIMIT = 48;
static_assert(MSD_B % RS_THREADS == 0, "scan layout");

__device__ __forceinline__ bool msd_sort(const unsigned (&kr)[RS_MAXR], const unsigned (&ir)[RS_MAXR], int n,
                                         int c0, int R, int kbits, unsigned *sk, unsigned *hc, int *s_wsum,
                                         int *s_flag, unsigned *__restrict__ ids_out) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int shift = kbits > MSD_BITS ? kbits - MSD_BITS : 0;
    constexpr int BPT = MSD_B / RS_THREADS;
    // (hc and *s_flag were zeroed by sort_tile under its span barrier)
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        const int e = c0 + r * 64 + lane;
        if (r < R && e < n) atomicAdd(&hc[kr[r] >> shift], 1u);
    }
    __syncthreads();
    // exclusive scan of the bucket counts (BPT consecutive buckets per thread), and the largest bucket
    unsigned loc[BPT], sum = 0u, mx = 0u;
#pragma unroll
    for (int j = 0; j < BPT; j++) {
        loc[j] = hc[tid * BPT + j];
        sum += loc[j];
        mx = max(mx, loc[j]);
    }
    const int incl = wave_incl_scan((int)sum, lane);
    if (lane == 63) s_wsum[w] = incl;
    if (mx > (unsigned)MSD_LIMIT) *s_flag = 1;  // benign race: every writer stores 1
    __syncthreads();
    if (*s_flag) return false;  // workgroup-uniform
    unsigned run = (unsigned)(incl - (int)sum);
    for (int ww = 0; ww < w; ww++) run += (unsigned)s_wsum[ww];
#pragma unroll
    for (int j = 0; j < BPT; j++) {
        hc[tid * BPT + j] = run;
        run += loc[j];
    }
    __syncthreads();
    // scatter (arbitrary order inside a bucket); afterwards hc[b] is the END of bucket b (= start of b + 1)
    // key and id side by side (the sk / si image read as one u64 array): one 8-B LDS write per entry here and one
    // 8-B read per bucket entry in the ranking, on the composite (key << 32 | id) order
    unsigned long long *skv = reinterpret_cast<unsigned long long *>(sk);
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        const int e = c0 + r * 64 + lane;
        if (r < R && e < n) {
            const unsigned pos = atomicAdd(&hc[kr[r] >> shift], 1u);
            skv[pos] = ((unsigned long long)kr[r] << 32) | ir[r];
        }
    }
    __syncthreads();
    for (int q = tid; q < n; q += RS_THREADS) {
        const unsigned long long cq = skv[q];
        const unsigned bq = (unsigned)(cq >> 32) >> shift;
        const int lo = bq ? (int)hc[bq - 1] : 0, hi = (int)hc[bq];
        int rank = lo;
        for (int z = lo; z < hi; z++) rank += skv[z] < cq ? 1 : 0;
        ids_out[rank] = (unsigned)cq;
    }
    return true;
}

// One tile's bucket: LDS LSD radix sort (see the file header); all threads of the block call it.
__device__ __forceinline__ void sort_tile(long long base, int n, unsigned long long *__restrict__ pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned *sk = reinterpret_cast<unsigned *>(smem);
    unsigned short *sp = reinterpret_cast<unsigned short *>(sk + RS_CAP);
    RsCnt *cnt = reinterpret_cast<RsCnt *>(sp + RS_CAP);
    __shared__ unsigned s_vmax;
    __shared__ int s_wsum[RS_WAVES], s_long, s_flag;
    if (n <= 1) return;  // a single id already sits in place (low half of its key)
    unsigned long long *seg = pairs + base;
    if (n > RS_CAP) {
        sort_oversized(seg, n, reinterpret_cast<unsigned long long *>(smem));
        return;
    }
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int C = ((n + RS_THREADS - 1) / RS_THREADS) * 64;  // per-wave chunk, a multiple of 64
    const int R = C >> 6, c0 = w * C;
    unsigned kr[RS_MAXR], ir[RS_MAXR];
    unsigned short pr[RS_MAXR];
    unsigned lmin = 0xffffffffu, lmax = 0u, vmax = 0u;
    // every row's load issued before the first use (clamped index, no per-row branch around the load): with the
    // load inside the per-row branch each row waited for its own round trip (vmcnt(0) per row, R serial trips)
    unsigned long long xv[RS_MAXR];
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        const int e = c0 + r * 64 + lane;
        if (r < R) xv[r] = seg[min(e, n - 1)];  // (r < R is workgroup-uniform)
    }
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        kr[r] = 0u;
        ir[r] = 0u;
        const int e = c0 + r * 64 + lane;
        if (r < R && e < n) {
            const unsigned long long x = xv[r];
            kr[r] = (unsigned)(x >> 32);
            ir[r] = (unsigned)x;
            lmin = min(lmin, kr[r]);
            lmax = max(lmax, kr[r]);
            vmax = max(vmax, (unsigned)x);
        }
    }
    // the span is reduced through per-wave LDS slots (no initialised LDS atomics, one barrier), and the MSD bucket
    // counters are zeroed under that barrier (none at the start of msd_sort): k_sort 152 -> 150 us on the pool
    if (tid == 0) { s_long = 0; s_flag = 0; }
    {
        unsigned *hc0 = reinterpret_cast<unsigned *>(smem) + 2 * RS_CAP;
        for (int q = tid; q < MSD_B; q += RS_THREADS) hc0[q] = 0u;
    }
    __shared__ unsigned s_wmm[3][RS_WAVES];
    lmin = wave_min_u32(lmin);
    lmax = wave_max_u32(lmax);
    vmax = wave_max_u32(vmax);
    if (lane == 0) { s_wmm[0][w] = lmin; s_wmm[1][w] = lmax; s_wmm[2][w] = vmax; }
    __syncthreads();
    unsigned kmin = s_wmm[0][0], kmax = s_wmm[1][0], vall = s_wmm[2][0];
#pragma unroll
    for (int ww = 1; ww < RS_WAVES; ww++) {
        kmin = min(kmin, s_wmm[0][ww]);
        kmax = max(kmax, s_wmm[1][ww]);
        vall = max(vall, s_wmm[2][ww]);
    }
    if (tid == 0) s_vmax = vall;  // (read after later barriers, by the tie path only)
    const unsigned span = kmax - kmin;
    const int kbits = span ? 32 - __clz(span) : 0;
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) kr[r] -= kmin;
    auto reload = [&]() {
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            if (r < R) {
                const int e = c0 + r * 64 + lane;
                if (e < n) { kr[r] = sk[e]; pr[r] = sp[e]; }
            }
        }
    };
    // (kr holds key - kmin: the MSD buckets split the tile's span)
    if (kbits > 0 && msd_sort(kr, ir, n, c0, R, kbits, sk, reinterpret_cast<unsigned *>(smem) + 2 * RS_CAP, s_wsum,
                              &s_flag, reinterpret_cast<unsigned *>(seg)))
        return;
    unsigned idr[RS_MAXR];
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) pr[r] = (unsigned short)(c0 + r * 64 + lane);  // bucket positions
    for (int sh = 0; sh < kbits; sh += RS_DBITS) {
        radix_pass(kr, pr, sh, min(RS_DBITS, kbits - sh), n, c0, R, sk, sp, cnt, s_wsum);
        reload();
    }
    if (kbits == 0) {
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            if (r < R) {
                const int e = c0 + r * 64 + lane;
                if (e < n) { sk[e] = kr[r]; sp[e] = pr[r]; }
            }
        }
        __syncthreads();
    }
    // Ties (equal depth bits) must end in increasing id order, as upstream's stable sort leaves them.
    for (int q = tid + 32; q < n; q += RS_THREADS)
        if (sk[q] == sk[q - 32]) s_long = 1;
    __syncthreads();
    if (s_long) {
        // long runs of equal depth (e.g. a flat layer facing the camera): full LSD on (key, id) from the bucket
        // order: the id digits first (the ids themselves serve as the keys), then the depth digits
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            const int e = c0 + r * 64 + lane;
            if (r < R && e < n) { kr[r] = (unsigned)seg[e]; pr[r] = (unsigned short)e; }
        }
        const int vbits = s_vmax ? 32 - __clz(s_vmax) : 0;
        for (int sh = 0; sh < vbits; sh += RS_DBITS) {
            radix_pass(kr, pr, sh, min(RS_DBITS, vbits - sh), n, c0, R, sk, sp, cnt, s_wsum);
            reload();
        }
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            const int e = c0 + r * 64 + lane;
            if (r < R && e < n) kr[r] = (unsigned)(seg[pr[r]] >> 32) - kmin;
        }
        for (int sh = 0; sh < kbits; sh += RS_DBITS) {
            radix_pass(kr, pr, sh, min(RS_DBITS, kbits - sh), n, c0, R, sk, sp, cnt, s_wsum);
            reload();
        }
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            idr[r] = 0u;
            const int e = c0 + r * 64 + lane;
            if (r < R && e < n) idr[r] = (unsigned)seg[pr[r]];
        }
    } else {
        // short runs (<= 32): gather the ids in key order, then order each run of equal keys by id
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            idr[r] = 0u;
            const int e = c0 + r * 64 + lane;
            if (r < R && e < n) idr[r] = (unsigned)seg[sp[e]];
        }
        bool any_tie = false;
        for (int q = tid; q + 1 < n; q += RS_THREADS) any_tie |= sk[q] == sk[q + 1];
        if (__syncthreads_or(any_tie)) {
            unsigned *ids_l = reinterpret_cast<unsigned *>(sp);  // sp + cnt = RS_CAP u32, free after the gather
#pragma unroll
            for (int r = 0; r < RS_MAXR; r++) {
                const int e = c0 + r * 64 + lane;
                if (r < R && e < n) ids_l[e] = idr[r];
            }
            __syncthreads();
            for (int q = tid; q < n; q += RS_THREADS) {
                if (q + 1 < n && sk[q] == sk[q + 1] && (q == 0 || sk[q - 1] != sk[q])) {
                    int e = q + 1;
                    while (e < n && sk[e] == sk[q]) e++;
                    for (int a2 = q + 1; a2 < e; a2++) {
                        const unsigned v = ids_l[a2];
                        int z = a2 - 1;
                        while (z >= q && ids_l[z] > v) { ids_l[z + 1] = ids_l[z]; z--; }
                        ids_l[z + 1] = v;
                    }
                }
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < RS_MAXR; r++) {
                const int e = c0 + r * 64 + lane;
                if (r < R && e < n) idr[r] = ids_l[e];
            }
        }
    }
    __syncthreads();  // every read of the bucket (seg) is done before the ids overwrite it in place
    unsigned *ids = reinterpret_cast<unsigned *>(seg);
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        const int e = c0 + r * 64 + lane;
        if (r < R && e < n) ids[e] = idr[r];
    }
}

// k_sort: grid (B*V*T), block RS_THREADS, dynamic LDS RS_LDS bytes; workgroup b sorts tile xcd_item(b), or with
// the centre-first table (center_order) tile corder[b / BV] of view b % BV. 8 waves per SIMD: <= 64 VGPRs, 4
// workgroups per CU with the u16 counters.
__global__ __launch_bounds__(RS_THREADS) __attribute__((amdgpu_waves_per_eu(8))) void k_sort(
    int M, long long slot_stride, const int *__restrict__ tile_start, const int *__restrict__ tile_count,
    unsigned long long *__restrict__ pairs, unsigned long long *__restrict__ counters, int BV, int T,
    const int *__restrict__ corder) {
    int tile = xcd_item(blockIdx.x, M);
    if (corder) {  // centre-first, views interleaved (center_order)
        const int r = (int)blockIdx.x / BV, v = (int)blockIdx.x - r * BV;
        tile = v * T + corder[r];
    }
    long long base;
    int n;
    tile_range(tile, slot_stride, tile_start, tile_count, base, n);
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    if (counters && threadIdx.x == 0) {  // per-workgroup timeline + bucket size (see lgm_diag.render_counters)
        counters[8 + 8 * (size_t)tile + 4] = t_start;
        counters[8 + 8 * (size_t)tile + 6] = (unsigned long long)n;
    }
    sort_tile(base, n, pairs);
    if (counters) {
        __syncthreads();
        if (threadIdx.x == 0) counters[8 + 8 * (size_t)tile + 5] = __builtin_amdgcn_s_memrealtime();
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------------------------
int launch_binning(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                   char *ws, const Layout &L, int *radii_out, long long *stats_out, bool count_only,
                   hipStream_t st) {
    const size_t M = (size_t)d.BV * d.T;
    // tile counters and the misc counters are adjacent in the layout: one memset
    if (hipMemsetAsync(ws + L.tile_count, 0, L.misc + 64 - L.tile_count, st) != hipSuccess) {
        set_error("hipMemsetAsync failed");
        return LGM_E_HIP;
    }
    float4 *gP = (float4 *)(ws + L.gP), *gQ = (float4 *)(ws + L.gQ);
    uint2 *rects = (uint2 *)(ws + L.rects);
    int *tcount = (int *)(ws + L.tile_count), *tstart = (int *)(ws + L.tile_start);
    unsigned long long *pairs = (unsigned long long *)(ws + L.pairs), *misc = (unsigned long long *)(ws + L.misc);
    float *accum = (float *)(ws + L.accum);
    const size_t lds = d.T <= LDS_HIST_MAX ? 3 * (size_t)d.T * 4 : 0;
    // k_sort's centre-first tile table (the first T ints of the order buffer; the binning histogram's 3T ints of LDS
    // hold its counting sort)
    int *corder = lds && d.T >= 8 ? (int *)(ws + L.order) : nullptr;
    dim3 grid((d.N + BIN_G - 1) / BIN_G, d.B * ((d.V + BIN_ITERS - 1) / BIN_ITERS));
    if (d.N > 0) {
        if (count_only || !L.slot) {
            LGM_LAUNCH("k_bin_count", st, (k_bin<COUNT><<<grid, BIN_THREADS, lds, st>>>(d, gaussians, cam_view, cam_view_proj,
                       gP, gQ, rects, nullptr, tcount, tstart, pairs, 0, misc, accum, nullptr)));
        }
        if (!count_only) {
            if (L.slot) {
                LGM_LAUNCH("k_bin", st, (k_bin<EMIT_SLOT><<<grid, BIN_THREADS, lds, st>>>(d, gaussians, cam_view, cam_view_proj,
                           gP, gQ, rects, radii_out, tcount, tstart, pairs, (long long)d.N, misc, accum, corder)));
            } else {
                LGM_LAUNCH("k_scan", st, (k_scan<<<1, 1024, 0, st>>>(tcount, (int)M, tstart)));
                if (hipMemsetAsync(ws + L.tile_count, 0, L.misc + 64 - L.tile_count, st) != hipSuccess) {
                    set_error("hipMemsetAsync failed");
                    return LGM_E_HIP;
                }
                LGM_LAUNCH("k_bin", st, (k_bin<EMIT_PACKED><<<grid, BIN_THREADS, lds, st>>>(d, gaussians, cam_view,
                           cam_view_proj, gP, gQ, rects, radii_out, tcount, tstart, pairs, 0, misc, accum, corder)));
            }
            LGM_LAUNCH("k_sort", st, (k_sort<<<(unsigned)M, RS_THREADS, RS_LDS, st>>>(
                                         (int)M, L.slot ? (long long)d.N : -1LL, tstart, tcount, pairs, d.counters,
                                         d.BV, d.T, corder)));
        }
    }
    if (d.N == 0 && !L.slot && hipMemsetAsync(ws + L.tile_start, 0, (M + 1) * 4, st) != hipSuccess) {
        set_error("hipMemsetAsync failed");  // packed mode with no Gaussians: every tile range is empty
        return LGM_E_HIP;
    }
    if (stats_out && hipMemcpyAsync(stats_out, ws + L.misc, 16, hipMemcpyDeviceToDevice, st) != hipSuccess) {
        set_error("hipMemcpyAsync failed");
        return LGM_E_HIP;
    }
    return LGM_OK;
}

}  // namespace lgm
