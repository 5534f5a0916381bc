// lgm_amd/csrc/render_bin.hip -- per-(view, Gaussian) preprocess + tile binning + per-tile depth sort.
//
// Replaces upstream's preprocess -> InclusiveSum -> D2H(num_rendered) -> duplicateWithKeys -> 41-bit global LSD
// radix sort -> identifyTileRanges, once per (b, v), with one launch sequence over all
// B x V views and no host synchronisation:
//   k_bin<EMIT_SLOT>   preprocess + emit each Gaussian's (depth_bits << 32 | id) key into the slot bucket of every
//                      tile it can reach (LDS tile histogram -> one global atomic reservation per touched tile per
//                      workgroup -> LDS-local positions). Slot buckets need no count pass and no scan.
//   k_bin<COUNT>/k_scan/k_bin<EMIT_PACKED>   the same with exact packing (large workloads).
//   k_sort             one workgroup per tile: LDS LSD radix sort of the bucket on the varying depth bits (wave
//                      ballot multisplit ranks, per-wave chunks => stable), ties ordered by Gaussian id. The result
//                      is exactly upstream's order: its LSD sort is stable on index-ordered pairs, so equal depths
//                      keep increasing Gaussian id. Buckets > 8192 use an in-place bitonic network on the u64
//                      composite key (LDS blocks + global merge stages).
#include "render_common.h"

namespace lgm {
namespace {

enum BinMode { COUNT = 0, EMIT_SLOT = 1, EMIT_PACKED = 2 };

// ------------------------------------------------------------------------------------------------------------
// k_bin: grid (ceil(N / BIN_G), B*V), block 256; every thread handles BIN_GPT Gaussians of one view so that a
// workgroup's LDS tile histogram aggregates 1024 Gaussians before its one global reservation per touched tile.
constexpr int BIN_GPT = 4, BIN_G = 256 * BIN_GPT;

struct EmitGeo {
    float x, y, A, B, C, iA, iC, tau;
    int cx0, cy0, cx1, cy1;
    unsigned long long hitmask;  // candidate tiles (row-major in the candidate rect) that pass the exact test
    unsigned long long key;
};

template <int MODE>
__global__ __launch_bounds__(256) void k_bin(Dims d, const float *__restrict__ gauss, const float *__restrict__ views,
                                             const float *__restrict__ projs, float4 *__restrict__ gA,
                                             float4 *__restrict__ gB, float *__restrict__ gD,
                                             uint2 *__restrict__ rects, int *__restrict__ radii_out,
                                             int *__restrict__ tile_count, const int *__restrict__ tile_start,
                                             unsigned long long *__restrict__ pairs, long long slot_stride,
                                             unsigned long long *__restrict__ misc) {
    extern __shared__ int hist[];  // [T] counts, then [T] reserved bases
    __shared__ unsigned long long s_tot[2];
    const int bv = blockIdx.y, b = bv / d.V, T = d.T;
    const bool lds = T <= LDS_HIST_MAX;
    int *hbase = hist + T;
    int *cur = tile_count + (size_t)bv * T;
    if (threadIdx.x < 2) s_tot[threadIdx.x] = 0;
    if (lds)
        for (int t = threadIdx.x; t < T; t += blockDim.x) hist[t] = 0;
    __syncthreads();
    auto dest = [&](int t, int pos) -> long long {
        return (MODE == EMIT_SLOT ? ((long long)bv * T + t) * slot_stride
                                  : (long long)tile_start[(size_t)bv * T + t]) + pos;
    };
    EmitGeo em[BIN_GPT];
    unsigned long long nemit = 0, nref = 0;
#pragma unroll
    for (int r = 0; r < BIN_GPT; r++) {
        const int i = blockIdx.x * BIN_G + r * 256 + threadIdx.x;
        Geo o;
        bool vis = false;
        if (i < d.N) {
            float g[14];
            load_gaussian(gauss + ((size_t)b * d.N + i) * 14, g);
            vis = preprocess_one(g, views + 16 * bv, projs + 16 * bv, d, o);
            if (MODE != COUNT) {
                const size_t k = (size_t)bv * d.N + i;
                if (vis) {
                    gA[k] = make_float4(o.x, o.y, o.tau, 0.f);
                    gB[k] = make_float4(o.A, o.B, o.C, o.opacity);
                    gD[k] = o.depth;
                    rects[k] = make_uint2((unsigned)o.x0 | ((unsigned)o.y0 << 16),
                                          (unsigned)o.x1 | ((unsigned)o.y1 << 16));
                } else {
                    gA[k] = make_float4(0.f, 0.f, -1.f, 0.f);
                    gB[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                    gD[k] = 0.f;
                    rects[k] = make_uint2(0u, 0u);
                }
                if (radii_out) radii_out[k] = vis ? o.radius : 0;
            }
        }
        EmitGeo &e = em[r];
        e.hitmask = 0ull;
        if (!vis) {
            e.cx0 = e.cx1 = e.cy0 = e.cy1 = 0;
            e.key = 0ull;
            continue;
        }
        nref += (unsigned long long)((o.x1 - o.x0) * (o.y1 - o.y0));
        e.x = o.x; e.y = o.y; e.A = o.A; e.B = o.B; e.C = o.C; e.tau = o.tau;
        e.iA = 1.0f / o.A;
        e.iC = 1.0f / o.C;
        e.cx0 = o.cx0; e.cy0 = o.cy0; e.cx1 = o.cx1; e.cy1 = o.cy1;
        e.key = ((unsigned long long)__float_as_uint(o.depth) << 32) | (unsigned)i;
        int bit = 0;
        for (int y = e.cy0; y < e.cy1; y++)
            for (int x = e.cx0; x < e.cx1; x++, bit++) {
                if (!ellipse_hits_rect(e.x, e.y, e.A, e.B, e.C, e.iA, e.iC, e.tau, (float)(x * BX),
                                       (float)(x * BX + BX - 1), (float)(y * BY), (float)(y * BY + BY - 1)))
                    continue;
                nemit++;
                if (bit < 64) e.hitmask |= 1ull << bit;
                const int t = y * d.gx + x;
                if (lds) {
                    atomicAdd(&hist[t], 1);
                } else {
                    const int pos = atomicAdd(&cur[t], 1);
                    if (MODE != COUNT) pairs[dest(t, pos)] = e.key;
                }
            }
    }
    if (nemit) atomicAdd(&s_tot[0], nemit);
    if (nref) atomicAdd(&s_tot[1], nref);
    if (lds) {
        __syncthreads();
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            const int c = hist[t];
            if (MODE == COUNT) {
                if (c) atomicAdd(&cur[t], c);
            } else {
                if (c) hbase[t] = atomicAdd(&cur[t], c);
                hist[t] = 0;
            }
        }
        if (MODE != COUNT) {
            __syncthreads();
#pragma unroll
            for (int r = 0; r < BIN_GPT; r++) {
                const EmitGeo &e = em[r];
                int bit = 0;
                for (int y = e.cy0; y < e.cy1; y++)
                    for (int x = e.cx0; x < e.cx1; x++, bit++) {
                        const bool h = bit < 64 ? ((e.hitmask >> bit) & 1ull) != 0ull
                                                : ellipse_hits_rect(e.x, e.y, e.A, e.B, e.C, e.iA, e.iC, e.tau,
                                                                    (float)(x * BX), (float)(x * BX + BX - 1),
                                                                    (float)(y * BY), (float)(y * BY + BY - 1));
                        if (!h) continue;
                        const int t = y * d.gx + x;
                        pairs[dest(t, hbase[t] + atomicAdd(&hist[t], 1))] = e.key;
                    }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(&misc[0], s_tot[0]);
        atomicAdd(&misc[1], s_tot[1]);
    }
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
constexpr int RS_THREADS = 512, RS_WAVES = RS_THREADS / 64, RS_CAP = 8192, RS_MAXR = RS_CAP / RS_THREADS;
constexpr int RS_LDS = RS_CAP * 8 + RS_WAVES * 256 * 4;

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// Lanes of the wavefront holding the same 8-bit digit as this lane (restricted to valid lanes).
__device__ __forceinline__ unsigned long long match8(unsigned dgt, bool valid) {
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
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
__device__ __forceinline__ int wave_incl_scan(int x, int lane) {
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
        const int y = __shfl_up(x, dd, 64);
        if (lane >= dd) x += y;
    }
    return x;
}

// One stable LSD pass over 8-bit digits (kr >> shift) & 255 of the per-wave chunks held in registers; writes
// the permuted (key, value) pairs to LDS sk/sv. All threads of the block must call it.
__device__ __forceinline__ void radix_pass(unsigned (&kr)[RS_MAXR], unsigned (&vr)[RS_MAXR], bool by_value,
                                          int shift, int n, int c0, int R, unsigned *sk, unsigned *sv, int *cnt,
                                          int *s_wsum) {
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    int *my = cnt + w * 256;
    for (int q = lane; q < 256; q += 64) my[q] = 0;
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        if (r < R) {
            const int e = c0 + r * 64 + lane;
            if (e < n) atomicAdd(&my[((by_value ? vr[r] : kr[r]) >> shift) & 255u], 1);
        }
    }
    __syncthreads();
    int run = 0, incl = 0;
    if (tid < 256) {
        for (int ww = 0; ww < RS_WAVES; ww++) {
            const int x = cnt[ww * 256 + tid];
            cnt[ww * 256 + tid] = run;
            run += x;
        }
        incl = wave_incl_scan(run, lane);
        if (lane == 63) s_wsum[w] = incl;
    }
    __syncthreads();
    if (tid < 256) {
        int off = incl - run;
        for (int ww = 0; ww < w; ww++) off += s_wsum[ww];
        for (int ww = 0; ww < RS_WAVES; ww++) cnt[ww * 256 + tid] += off;
    }
    __syncthreads();
    const unsigned long long lt = lanemask_lt(lane);
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        if (r < R) {
            const int e = c0 + r * 64 + lane;
            const bool valid = e < n;
            const unsigned dgt = ((by_value ? vr[r] : kr[r]) >> shift) & 255u;
            const unsigned long long peers = match8(dgt, valid);
            if (valid) {
                const int rank = __popcll(peers & lt);
                const int pos = my[dgt] + rank;
                if (rank == 0) my[dgt] += __popcll(peers);
                sk[pos] = kr[r];
                sv[pos] = vr[r];
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
// index >= n act as +inf) on the u64 composite keys in place: LDS blocks of RS_CAP for short distances, global
// memory for long ones. Rare (only huge central tiles); correct for any n.
__device__ void sort_oversized(unsigned long long *seg, int n, unsigned long long *sk) {
    const int C = RS_CAP;
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

// k_sort: grid (B*V*T), block RS_THREADS, dynamic LDS RS_LDS bytes.
__global__ __launch_bounds__(RS_THREADS) void k_sort(long long slot_stride, const int *__restrict__ tile_start,
                                                     const int *__restrict__ tile_count,
                                                     unsigned long long *__restrict__ pairs) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned *sk = reinterpret_cast<unsigned *>(smem);
    unsigned *sv = sk + RS_CAP;
    int *cnt = reinterpret_cast<int *>(sv + RS_CAP);
    __shared__ unsigned s_min, s_max;
    __shared__ int s_wsum[4], s_long;
    long long base;
    int n;
    tile_range(blockIdx.x, slot_stride, tile_start, tile_count, base, n);
    if (n <= 1) return;  // a single id already sits in place (low half of its key)
    unsigned long long *seg = pairs + base;
    if (n > RS_CAP) {
        sort_oversized(seg, n, reinterpret_cast<unsigned long long *>(smem));
        return;
    }
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int C = ((n + RS_THREADS - 1) / RS_THREADS) * 64;  // per-wave chunk, a multiple of 64
    const int R = C >> 6, c0 = w * C;
    unsigned kr[RS_MAXR], vr[RS_MAXR];
    unsigned lmin = 0xffffffffu, lmax = 0u, vmax = 0u;
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) {
        kr[r] = 0u;
        vr[r] = 0u;
        const int e = c0 + r * 64 + lane;
        if (r < R && e < n) {
            const unsigned long long x = seg[e];
            kr[r] = (unsigned)(x >> 32);
            vr[r] = (unsigned)x;
            lmin = min(lmin, kr[r]);
            lmax = max(lmax, kr[r]);
            vmax = max(vmax, vr[r]);
        }
    }
    if (tid == 0) { s_min = 0xffffffffu; s_max = 0u; s_long = 0; }
    __syncthreads();
    lmin = wave_min_u32(lmin);
    lmax = wave_max_u32(lmax);
    if (lane == 0) { atomicMin(&s_min, lmin); atomicMax(&s_max, lmax); }
    __syncthreads();
    const unsigned kmin = s_min, span = s_max - s_min;
    const int kpasses = span ? (32 - __clz(span) + 7) >> 3 : 0;
#pragma unroll
    for (int r = 0; r < RS_MAXR; r++) kr[r] -= kmin;
    for (int p = 0; p < kpasses; p++) {
        radix_pass(kr, vr, false, 8 * p, n, c0, R, sk, sv, cnt, s_wsum);
        if (p + 1 < kpasses) {
#pragma unroll
            for (int r = 0; r < RS_MAXR; r++) {
                if (r < R) {
                    const int e = c0 + r * 64 + lane;
                    if (e < n) { kr[r] = sk[e]; vr[r] = sv[e]; }
                }
            }
        }
    }
    if (kpasses == 0) {
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            if (r < R) {
                const int e = c0 + r * 64 + lane;
                if (e < n) { sk[e] = kr[r]; sv[e] = vr[r]; }
            }
        }
        __syncthreads();
    }
    // Ties (equal depth bits) must end in increasing id order, as upstream's stable sort leaves them.
    for (int q = tid + 32; q < n; q += RS_THREADS)
        if (sk[q] == sk[q - 32]) s_long = 1;
    __syncthreads();
    if (s_long) {
        // long runs of equal depth (e.g. a flat layer facing the camera): full LSD on (key, id): id digits first
        __syncthreads();
#pragma unroll
        for (int r = 0; r < RS_MAXR; r++) {
            if (r < R) {
                const int e = c0 + r * 64 + lane;
                if (e < n) { kr[r] = sk[e]; vr[r] = sv[e]; }
            }
        }
        __syncthreads();
        vmax = wave_max_u32(vmax);
        if (lane == 0) atomicMax(&s_max, 0u);  // keep s_max; vmax reduced below
        __shared__ unsigned s_vmax;
        if (tid == 0) s_vmax = 0u;
        __syncthreads();
        if (lane == 0) atomicMax(&s_vmax, vmax);
        __syncthreads();
        const int vpasses = s_vmax ? (32 - __clz(s_vmax) + 7) >> 3 : 0;
        const int total = vpasses + kpasses;
        for (int p = 0; p < total; p++) {
            const bool byv = p < vpasses;
            radix_pass(kr, vr, byv, 8 * (byv ? p : p - vpasses), n, c0, R, sk, sv, cnt, s_wsum);
            if (p + 1 < total) {
#pragma unroll
                for (int r = 0; r < RS_MAXR; r++) {
                    if (r < R) {
                        const int e = c0 + r * 64 + lane;
                        if (e < n) { kr[r] = sk[e]; vr[r] = sv[e]; }
                    }
                }
            }
        }
    } else {
        // short runs: insertion-sort each run by id (runs <= 32 long)
        for (int q = tid; q < n; q += RS_THREADS) {
            if (q + 1 < n && sk[q] == sk[q + 1] && (q == 0 || sk[q - 1] != sk[q])) {
                int e = q + 1;
                while (e < n && sk[e] == sk[q]) e++;
                for (int a = q + 1; a < e; a++) {
                    const unsigned v = sv[a];
                    int z = a - 1;
                    while (z >= q && sv[z] > v) { sv[z + 1] = sv[z]; z--; }
                    sv[z + 1] = v;
                }
            }
        }
        __syncthreads();
    }
    unsigned *ids = reinterpret_cast<unsigned *>(seg);
    for (int q = tid; q < n; q += RS_THREADS) ids[q] = sv[q];
}

}  // namespace

// ------------------------------------------------------------------------------------------------------------
int launch_binning(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                   char *ws, const Layout &L, int *radii_out, long long *stats_out, bool count_only,
                   hipStream_t st) {
    const size_t M = (size_t)d.BV * d.T;
    if (hipMemsetAsync(ws + L.tile_count, 0, M * 4, st) != hipSuccess ||
        hipMemsetAsync(ws + L.misc, 0, 64, st) != hipSuccess) {
        set_error("hipMemsetAsync failed");
        return LGM_E_HIP;
    }
    float4 *gA = (float4 *)(ws + L.gA), *gB = (float4 *)(ws + L.gB);
    float *gD = (float *)(ws + L.gD);
    uint2 *rects = (uint2 *)(ws + L.rects);
    int *tcount = (int *)(ws + L.tile_count), *tstart = (int *)(ws + L.tile_start);
    unsigned long long *pairs = (unsigned long long *)(ws + L.pairs), *misc = (unsigned long long *)(ws + L.misc);
    const size_t lds = d.T <= LDS_HIST_MAX ? 2 * (size_t)d.T * 4 : 0;
    dim3 grid((d.N + BIN_G - 1) / BIN_G, d.BV);
    if (d.N > 0) {
        if (count_only || !L.slot) {
            LGM_LAUNCH("k_bin_count", st, (k_bin<COUNT><<<grid, 256, lds, st>>>(d, gaussians, cam_view, cam_view_proj,
                       gA, gB, gD, rects, nullptr, tcount, tstart, pairs, 0, misc)));
        }
        if (!count_only) {
            if (L.slot) {
                LGM_LAUNCH("k_bin", st, (k_bin<EMIT_SLOT><<<grid, 256, lds, st>>>(d, gaussians, cam_view, cam_view_proj,
                           gA, gB, gD, rects, radii_out, tcount, tstart, pairs, (long long)d.N, misc)));
            } else {
                LGM_LAUNCH("k_scan", st, (k_scan<<<1, 1024, 0, st>>>(tcount, (int)M, tstart)));
                if (hipMemsetAsync(ws + L.tile_count, 0, M * 4, st) != hipSuccess ||
                    hipMemsetAsync(ws + L.misc, 0, 64, st) != hipSuccess) {
                    set_error("hipMemsetAsync failed");
                    return LGM_E_HIP;
                }
                LGM_LAUNCH("k_bin", st, (k_bin<EMIT_PACKED><<<grid, 256, lds, st>>>(d, gaussians, cam_view,
                           cam_view_proj, gA, gB, gD, rects, radii_out, tcount, tstart, pairs, 0, misc)));
            }
            LGM_LAUNCH("k_sort", st, (k_sort<<<(unsigned)M, RS_THREADS, RS_LDS, st>>>(
                                         L.slot ? (long long)d.N : -1LL, tstart, tcount, pairs)));
        }
    }
    if (stats_out && hipMemcpyAsync(stats_out, ws + L.misc, 16, hipMemcpyDeviceToDevice, st) != hipSuccess) {
        set_error("hipMemcpyAsync failed");
        return LGM_E_HIP;
    }
    return LGM_OK;
}

}  // namespace lgm
