// lgm_amd/csrc/render.hip -- MI355X (gfx950, CDNA4) Gaussian-splat render path: forward + backward.
//
// Replaces the per-(b, v) external rasterizer call of core/gs.py:58-85 (diff_gaussian_rasterization, EXT) with
// ONE stream-ordered launch sequence over all B x V views and no host synchronisation:
//
//   forward : k_preprocess  per (view, Gaussian): frustum cull, EWA projection, conic, radius, tile rect,
//                           per-tile pair counts (LDS histogram -> one global atomic per touched tile per WG)
//             k_scan        exclusive scan of the B*V*T tile counts -> global tile ranges (no D2H of K)
//             k_emit        per (view, Gaussian): scatter key (depth_bits << 32 | id) into its tiles' buckets
//             k_sort        per tile: LDS bitonic sort of the bucket by (depth, id) == upstream's stable LSD radix
//                           sort of (tile << 32 | depth) on index-ordered pairs; oversized buckets: LDS-chunk
//                           sort + global merge stages (same network)
//             k_render_fwd  per 16x16 tile: stage 256 Gaussians at a time in LDS, front-to-back compositing
//   backward: k_render_bwd  per tile, back to front from each pixel's last contributor; per-Gaussian partial
//                           gradients reduced across the wavefront with DPP, across waves with LDS float atomics,
//                           then one global atomic per (tile, Gaussian, value)
//             k_preproc_bwd per (scene, Gaussian): loops over the scene's views (deterministic sum over views),
//                           cov2D / projection / depth / cov3D backward -> dL/dgaussians [B,N,14]
//
// Numerics follow SURVEY.md §2.3 (the restated upstream algorithm, see oracle/raster_oracle.c):
// 0.3 dilation, 1.3 tanfov clamp, depth cull 0.2, alpha cap 0.99, alpha floor 1/255, T floor 1e-4 tested before
// accumulation, ndc2Pix in double, integer tile-rect math, full-precision expf.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "common.h"
#include "lgm_render.h"

namespace {

constexpr int BX = 16, BY = 16, TILE_PIX = BX * BY;  // 256 pixels per tile = 4 wavefronts
constexpr int SORT_THREADS = 512;
constexpr int SORT_CAP = 8192;       // keys sorted in LDS in one piece (64 KiB)
constexpr int LDS_HIST_MAX = 8192;   // tiles per view for the LDS-histogram binning path
constexpr int NACC = 10;             // per-(view, Gaussian) 2D gradient record

// ------------------------------------------------------------------------------------------------------------

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }

struct Layout {
    size_t gA, gB, rects, tile_count, tile_start, tile_cursor, keys, keys2, ids, final_T, n_contrib, accum, misc,
        total;
};

Layout make_layout(int B, int V, int N, int H, int W, long long cap) {
    const size_t BV = (size_t)B * V, T = (size_t)((W + BX - 1) / BX) * ((H + BY - 1) / BY), P = (size_t)H * W;
    Layout L;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    L.gA = take(BV * N * 16);
    L.gB = take(BV * N * 16);
    L.rects = take(BV * N * 8);
    L.tile_count = take(BV * T * 4);
    L.tile_start = take((BV * T + 1) * 4);
    L.tile_cursor = take(BV * T * 4);
    L.keys = take((size_t)cap * 8);
    L.keys2 = take((size_t)cap * 8);
    L.ids = take((size_t)cap * 4);
    L.final_T = take(BV * P * 4);
    L.n_contrib = take(BV * P * 4);
    L.accum = take(BV * N * NACC * 4);
    L.misc = take(64);
    L.total = o;
    return L;
}

long long worst_capacity(int B, int V, int N, int H, int W) {
    const long long T = (long long)((W + BX - 1) / BX) * ((H + BY - 1) / BY);
    return (long long)B * V * N * T;
}

// ------------------------------------------------------------------------------------------------------------
// Camera helpers: the 4x4 matrices are the row-major torch tensors of core/gs.py:54-55 read column-major.
__device__ __forceinline__ void xf43(const float *M, float x, float y, float z, float o[3]) {
    o[0] = M[0] * x + M[4] * y + M[8] * z + M[12];
    o[1] = M[1] * x + M[5] * y + M[9] * z + M[13];
    o[2] = M[2] * x + M[6] * y + M[10] * z + M[14];
}
__device__ __forceinline__ void xf44(const float *M, float x, float y, float z, float o[4]) {
    o[0] = M[0] * x + M[4] * y + M[8] * z + M[12];
    o[1] = M[1] * x + M[5] * y + M[9] * z + M[13];
    o[2] = M[2] * x + M[6] * y + M[10] * z + M[14];
    o[3] = M[3] * x + M[7] * y + M[11] * z + M[15];
}

// glm-convention rotation matrix Rg[col][row] from un-normalised quaternion (r,x,y,z) (upstream semantics).
__device__ __forceinline__ void quat_rot(const float q[4], float R[3][3]) {
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// Sigma = M^T M with M = S*R (glm): Sigma[c][r] = sum_k s_k^2 R[c][k] R[r][k]; stored (00,01,02,11,12,22).
__device__ __forceinline__ void cov3d(const float s[3], const float R[3][3], float c3[6]) {
    const float s0 = s[0] * s[0], s1 = s[1] * s[1], s2 = s[2] * s[2];
#define SIG(c, r) (s0 * R[c][0] * R[r][0] + s1 * R[c][1] * R[r][1] + s2 * R[c][2] * R[r][2])
    c3[0] = SIG(0, 0); c3[1] = SIG(0, 1); c3[2] = SIG(0, 2);
    c3[3] = SIG(1, 1); c3[4] = SIG(1, 2); c3[5] = SIG(2, 2);
#undef SIG
}

// The two non-zero glm columns of T = W*J (with the 1.3 tanfov clamp on t), SURVEY §2.3 row 1.
struct ProjCtx {
    float T0[3], T1[3];  // glm T[0][*], T[1][*]
    float t[3];          // clamped view-space mean
    float xmul, ymul;
};
__device__ __forceinline__ ProjCtx make_proj(const float *Vw, float mx, float my, float mz, float fx, float fy,
                                             float tanx, float tany) {
    ProjCtx P;
    xf43(Vw, mx, my, mz, P.t);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = P.t[0] / P.t[2], tytz = P.t[1] / P.t[2];
    P.t[0] = fminf(limx, fmaxf(-limx, txtz)) * P.t[2];
    P.t[1] = fminf(limy, fmaxf(-limy, tytz)) * P.t[2];
    P.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    P.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float tz = P.t[2];
    const float J00 = fx / tz, J02 = -(fx * P.t[0]) / (tz * tz);
    const float J11 = fy / tz, J12 = -(fy * P.t[1]) / (tz * tz);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        P.T0[r] = Vw[4 * r + 0] * J00 + Vw[4 * r + 2] * J02;
        P.T1[r] = Vw[4 * r + 1] * J11 + Vw[4 * r + 2] * J12;
    }
    return P;
}
__device__ __forceinline__ void cov2d(const ProjCtx &P, const float c3[6], float &a, float &b, float &c) {
    const float S[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float s0[3], s1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s0[k] = S[k][0] * P.T0[0] + S[k][1] * P.T0[1] + S[k][2] * P.T0[2];
        s1[k] = S[k][0] * P.T1[0] + S[k][1] * P.T1[1] + S[k][2] * P.T1[2];
    }
    a = P.T0[0] * s0[0] + P.T0[1] * s0[1] + P.T0[2] * s0[2] + 0.3f;
    b = P.T1[0] * s0[0] + P.T1[1] * s0[1] + P.T1[2] * s0[2];
    c = P.T1[0] * s1[0] + P.T1[1] * s1[1] + P.T1[2] * s1[2] + 0.3f;
}

__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

struct Geo {
    float x, y, depth, cx, cy, cz;
    int x0, y0, x1, y1, radius;
};

// Per-Gaussian forward preprocess. Returns false if culled.
__device__ __forceinline__ bool preprocess_one(const float *g, const float *Vw, const float *Pm, float tanx,
                                               float tany, float fx, float fy, float mod, int W, int H, int gx,
                                               int gy, Geo &o) {
    float hom[4], pv[3];
    xf44(Pm, g[0], g[1], g[2], hom);
    const float pw = 1.0f / (hom[3] + 0.0000001f);
    const float ppx = hom[0] * pw, ppy = hom[1] * pw;
    xf43(Vw, g[0], g[1], g[2], pv);
    if (pv[2] <= 0.2f) return false;
    float R[3][3];
    const float q[4] = {g[7], g[8], g[9], g[10]};
    quat_rot(q, R);
    const float s[3] = {mod * g[4], mod * g[5], mod * g[6]};
    float c3[6];
    cov3d(s, R, c3);
    const ProjCtx P = make_proj(Vw, g[0], g[1], g[2], fx, fy, tanx, tany);
    float a, b, c;
    cov2d(P, c3, a, b, c);
    const float det = a * c - b * b;
    if (det == 0.0f) return false;
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (a + c);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float px = ndc2pix(ppx, W), py = ndc2pix(ppy, H);
    const int r = (int)rad;
    const int x0 = min(gx, max(0, (int)((px - r) / BX)));
    const int y0 = min(gy, max(0, (int)((py - r) / BY)));
    const int x1 = min(gx, max(0, (int)((px + r + BX - 1) / BX)));
    const int y1 = min(gy, max(0, (int)((py + r + BY - 1) / BY)));
    if ((x1 - x0) * (y1 - y0) == 0) return false;
    o.x = px; o.y = py; o.depth = pv[2];
    o.cx = c * det_inv; o.cy = -b * det_inv; o.cz = a * det_inv;
    o.x0 = x0; o.y0 = y0; o.x1 = x1; o.y1 = y1; o.radius = r;
    return true;
}

__device__ __forceinline__ void load_gaussian(const float *__restrict__ src, float g[14]) {
    // rows are 56 B, always 8-B aligned: 7 x dwordx2
    const float2 *p = reinterpret_cast<const float2 *>(src);
#pragma unroll
    for (int k = 0; k < 7; k++) {
        const float2 v = p[k];
        g[2 * k] = v.x;
        g[2 * k + 1] = v.y;
    }
}

// ------------------------------------------------------------------------------------------------------------
// k_preprocess: grid (ceil(N/256), B*V), block 256.
template <bool LDS_HIST>
__global__ __launch_bounds__(256) void k_preprocess(int N, int V, int W, int H, int gx, int gy,
                                                    const float *__restrict__ gauss, const float *__restrict__ views,
                                                    const float *__restrict__ projs, float tanx, float tany,
                                                    float fx, float fy, float mod, float4 *__restrict__ gA,
                                                    float4 *__restrict__ gB, uint2 *__restrict__ rects,
                                                    int *__restrict__ tile_count, int *__restrict__ radii_out) {
    extern __shared__ int hist[];
    const int bv = blockIdx.y, b = bv / V, T = gx * gy;
    if (LDS_HIST) {
        for (int t = threadIdx.x; t < T; t += blockDim.x) hist[t] = 0;
        __syncthreads();
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    Geo o;
    bool vis = false;
    if (i < N) {
        float g[14];
        load_gaussian(gauss + ((size_t)b * N + i) * 14, g);
        vis = preprocess_one(g, views + 16 * bv, projs + 16 * bv, tanx, tany, fx, fy, mod, W, H, gx, gy, o);
        const size_t k = (size_t)bv * N + i;
        if (vis) {
            gA[k] = make_float4(o.x, o.y, o.cx, o.cy);
            gB[k] = make_float4(o.cz, g[3], o.depth, 0.f);
            rects[k] = make_uint2((unsigned)o.x0 | ((unsigned)o.y0 << 16), (unsigned)o.x1 | ((unsigned)o.y1 << 16));
        } else {
            gA[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            gB[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            rects[k] = make_uint2(0u, 0u);
        }
        if (radii_out) radii_out[k] = vis ? o.radius : 0;
    }
    if (vis) {
        for (int y = o.y0; y < o.y1; y++)
            for (int x = o.x0; x < o.x1; x++) {
                if (LDS_HIST) atomicAdd(&hist[y * gx + x], 1);
                else atomicAdd(&tile_count[(size_t)bv * T + y * gx + x], 1);
            }
    }
    if (LDS_HIST) {
        __syncthreads();
        for (int t = threadIdx.x; t < T; t += blockDim.x)
            if (hist[t]) atomicAdd(&tile_count[(size_t)bv * T + t], hist[t]);
    }
}

// k_scan: one workgroup of 1024 threads; exclusive scan of M tile counts -> tile_start[0..M], tile_cursor.
__global__ __launch_bounds__(1024) void k_scan(const int *__restrict__ count, int M, int *__restrict__ start,
                                               int *__restrict__ cursor, long long *__restrict__ misc,
                                               long long cap, long long *__restrict__ stats_out) {
    __shared__ long long wsum[16];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int per = (M + 1023) / 1024;
    const int lo = min(M, tid * per), hi = min(M, lo + per);
    long long s = 0;
    for (int i = lo; i < hi; i++) s += count[i];
    // inclusive wave scan
    long long x = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const long long y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (wid == 0) {
        long long w = lane < 16 ? wsum[lane] : 0;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const long long y = __shfl_up(w, d, 64);
            if (lane >= d) w += y;
        }
        if (lane < 16) wsum[lane] = w;
    }
    __syncthreads();
    long long run = x - s + (wid > 0 ? wsum[wid - 1] : 0);
    for (int i = lo; i < hi; i++) {
        start[i] = (int)run;
        cursor[i] = (int)run;
        run += count[i];
    }
    if (tid == 1023) {
        const long long total = wsum[15];
        start[M] = (int)min(total, cap);
        misc[0] = total;
        misc[1] = total > cap ? 1 : 0;
        if (stats_out) { stats_out[0] = total; stats_out[1] = total > cap ? 1 : 0; }
    }
}

// k_emit: grid (ceil(N/256), B*V). Scatter (depth_bits << 32 | id) into each touched tile's bucket.
template <bool LDS_HIST>
__global__ __launch_bounds__(256) void k_emit(int N, int gx, int gy, const uint2 *__restrict__ rects,
                                              const float4 *__restrict__ gB, int *__restrict__ tile_cursor,
                                              unsigned long long *__restrict__ keys, long long cap) {
    extern __shared__ int sh[];
    const int T = gx * gy;
    int *hist = sh;
    int *base = sh + (LDS_HIST ? T : 0);
    const int bv = blockIdx.y;
    if (LDS_HIST) {
        for (int t = threadIdx.x; t < T; t += blockDim.x) hist[t] = 0;
        __syncthreads();
    }
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    int x0 = 0, y0 = 0, x1 = 0, y1 = 0;
    unsigned long long key = 0;
    if (i < N) {
        const uint2 r = rects[(size_t)bv * N + i];
        x0 = r.x & 0xffff; y0 = r.x >> 16; x1 = r.y & 0xffff; y1 = r.y >> 16;
        key = ((unsigned long long)__float_as_uint(gB[(size_t)bv * N + i].z) << 32) | (unsigned)i;
    }
    int *cur = tile_cursor + (size_t)bv * T;
    if (LDS_HIST) {
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) atomicAdd(&hist[y * gx + x], 1);
        __syncthreads();
        for (int t = threadIdx.x; t < T; t += blockDim.x) {
            const int c = hist[t];
            if (c) base[t] = atomicAdd(&cur[t], c);
            hist[t] = 0;
        }
        __syncthreads();
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                const int t = y * gx + x;
                const long long pos = (long long)base[t] + atomicAdd(&hist[t], 1);
                if (pos < cap) keys[pos] = key;
            }
    } else {
        for (int y = y0; y < y1; y++)
            for (int x = x0; x < x1; x++) {
                const long long pos = atomicAdd(&cur[y * gx + x], 1);
                if (pos < cap) keys[pos] = key;
            }
    }
}

// ------------------------------------------------------------------------------------------------------------
// Bitonic sort, "flip + half-cleaner" form: every comparator is ascending, so entries at index >= n act as
// +infinity and every comparator touching them is a no-op -- no padding needed.
__device__ __forceinline__ void cas(unsigned long long *s, int lo, int hi) {
    const unsigned long long a = s[lo], b = s[hi];
    if (a > b) { s[lo] = b; s[hi] = a; }
}
// full sort of s[0..n) (n <= m = next pow2), all threads of the block participate
__device__ void bitonic_sort_lds(unsigned long long *s, int n, int m) {
    for (int k = 2; k <= m; k <<= 1) {
        for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {  // flip
            const int half = k >> 1;
            const int lo = (p / half) * k + (p % half);
            const int hi = lo ^ (k - 1);
            if (hi < n) cas(s, lo, hi);
        }
        __syncthreads();
        for (int j = k >> 2; j > 0; j >>= 1) {  // half-cleaners
            for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
                const int lo = 2 * p - (p & (j - 1));
                const int hi = lo + j;
                if (hi < n) cas(s, lo, hi);
            }
            __syncthreads();
        }
    }
}
// half-cleaners j = m/2 .. 1 on s[0..n) (the tail of a merge stage whose distances fit in one LDS block)
__device__ void bitonic_clean_lds(unsigned long long *s, int n, int m) {
    for (int j = m >> 1; j > 0; j >>= 1) {
        for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
            const int lo = 2 * p - (p & (j - 1));
            const int hi = lo + j;
            if (hi < n) cas(s, lo, hi);
        }
        __syncthreads();
    }
}

__device__ __forceinline__ int next_pow2(int n) {
    int m = 1;
    while (m < n) m <<= 1;
    return m;
}

// k_sort: grid (B*V*T), block SORT_THREADS, dynamic LDS SORT_CAP*8 bytes.
__global__ __launch_bounds__(SORT_THREADS) void k_sort(const int *__restrict__ tile_start,
                                                       unsigned long long *__restrict__ keys,
                                                       unsigned *__restrict__ ids) {
    extern __shared__ unsigned long long skeys[];
    const int tile = blockIdx.x;
    const int s0 = tile_start[tile], s1 = tile_start[tile + 1];
    const int n = s1 - s0;
    if (n <= 0) return;
    unsigned long long *seg = keys + s0;
    if (n <= SORT_CAP) {
        const int m = next_pow2(n);
        for (int i = threadIdx.x; i < n; i += blockDim.x) skeys[i] = seg[i];
        __syncthreads();
        bitonic_sort_lds(skeys, n, m);
        for (int i = threadIdx.x; i < n; i += blockDim.x) ids[s0 + i] = (unsigned)skeys[i];
        return;
    }
    // ---- oversized bucket: sort SORT_CAP-blocks in LDS, then global merge stages, LDS for distances < CAP.
    const int m = next_pow2(n);
    for (int c0 = 0; c0 < n; c0 += SORT_CAP) {
        const int nb = min(SORT_CAP, n - c0);
        for (int i = threadIdx.x; i < nb; i += blockDim.x) skeys[i] = seg[c0 + i];
        __syncthreads();
        bitonic_sort_lds(skeys, nb, SORT_CAP);
        for (int i = threadIdx.x; i < nb; i += blockDim.x) seg[c0 + i] = skeys[i];
        __syncthreads();
    }
    for (int k = 2 * SORT_CAP; k <= m; k <<= 1) {
        for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {  // global flip
            const int half = k >> 1;
            const int lo = (p / half) * k + (p % half);
            const int hi = lo ^ (k - 1);
            if (hi < n) cas(seg, lo, hi);
        }
        __syncthreads();
        for (int j = k >> 2; j >= SORT_CAP; j >>= 1) {  // global half-cleaners
            for (int p = threadIdx.x; p < (m >> 1); p += blockDim.x) {
                const int lo = 2 * p - (p & (j - 1));
                const int hi = lo + j;
                if (hi < n) cas(seg, lo, hi);
            }
            __syncthreads();
        }
        for (int c0 = 0; c0 < n; c0 += SORT_CAP) {  // LDS half-cleaners j < CAP
            const int nb = min(SORT_CAP, n - c0);
            for (int i = threadIdx.x; i < nb; i += blockDim.x) skeys[i] = seg[c0 + i];
            __syncthreads();
            bitonic_clean_lds(skeys, nb, SORT_CAP);
            for (int i = threadIdx.x; i < nb; i += blockDim.x) seg[c0 + i] = skeys[i];
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < n; i += blockDim.x) ids[s0 + i] = (unsigned)seg[i];
}

// ------------------------------------------------------------------------------------------------------------
// Pixel of thread t inside a 16x16 tile: each wavefront owns an 8x8 quadrant (compact footprint per wave).
__device__ __forceinline__ void tile_pixel(int t, int &lx, int &ly) {
    const int w = t >> 6, l = t & 63;
    lx = ((w & 1) << 3) + (l & 7);
    ly = ((w >> 1) << 3) + (l >> 3);
}

// k_render_fwd: grid (B*V*T), block 256.
__global__ __launch_bounds__(256) void k_render_fwd(int N, int V, int W, int H, int gx, int T,
                                                    const int *__restrict__ tile_start,
                                                    const unsigned *__restrict__ ids,
                                                    const float4 *__restrict__ gA, const float4 *__restrict__ gB,
                                                    const float *__restrict__ gauss, const float *__restrict__ bg,
                                                    float *__restrict__ out_img, float *__restrict__ out_depth,
                                                    float *__restrict__ out_alpha, float *__restrict__ final_T,
                                                    int *__restrict__ n_contrib) {
    __shared__ float4 sA[TILE_PIX], sB[TILE_PIX], sC[TILE_PIX];
    const int tile = blockIdx.x;
    const int bv = tile / T, t = tile - bv * T, b = bv / V;
    const int tx = t % gx, ty = t / gx;
    int lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const int px = tx * BX + lx, py = ty * BY + ly;
    const bool inside = px < W && py < H;
    const float pfx = (float)px, pfy = (float)py;
    const int s0 = tile_start[tile], s1 = tile_start[tile + 1];
    bool done = !inside;
    float Tr = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, D = 0.f;
    int contributor = 0, last = 0;
    const size_t gbase = (size_t)bv * N;
    for (int base = s0; base < s1; base += TILE_PIX) {
        if (__syncthreads_count(done) == TILE_PIX) break;
        const int k = base + threadIdx.x;
        if (k < s1) {
            const unsigned gid = ids[k];
            sA[threadIdx.x] = gA[gbase + gid];
            const float4 bb = gB[gbase + gid];
            sB[threadIdx.x] = bb;
            const float *c = gauss + ((size_t)b * N + gid) * 14 + 11;
            sC[threadIdx.x] = make_float4(c[0], c[1], c[2], bb.z);
        }
        __syncthreads();
        const int cnt = min(TILE_PIX, s1 - base);
        for (int j = 0; !done && j < cnt; j++) {
            contributor++;
            const float4 a = sA[j];
            const float4 bb = sB[j];
            const float dx = a.x - pfx, dy = a.y - pfy;
            const float power = -0.5f * (a.z * dx * dx + bb.x * dy * dy) - a.w * dx * dy;
            if (power > 0.0f) continue;
            const float alpha = fminf(0.99f, bb.y * expf(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = Tr * (1 - alpha);
            if (test_T < 0.0001f) { done = true; continue; }
            const float4 c = sC[j];
            C0 += c.x * alpha * Tr;
            C1 += c.y * alpha * Tr;
            C2 += c.z * alpha * Tr;
            D += c.w * alpha * Tr;
            Tr = test_T;
            last = contributor;
        }
    }
    if (inside) {
        const size_t P = (size_t)H * W;
        const size_t pid = (size_t)W * py + px;
        final_T[bv * P + pid] = Tr;
        n_contrib[bv * P + pid] = last;
        float *img = out_img + (size_t)bv * 3 * P;
        img[pid] = C0 + Tr * bg[0];
        img[P + pid] = C1 + Tr * bg[1];
        img[2 * P + pid] = C2 + Tr * bg[2];
        out_depth[bv * P + pid] = D;
        out_alpha[bv * P + pid] = 1 - Tr;
    }
}

// ------------------------------------------------------------------------------------------------------------
// Wavefront sum with DPP (gfx9 row_bcast): the total lands in lane 63.
#define DPP_ADD(v, ctrl, rmask)                                                                                \
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, rmask, 0xf, \
                                                               false))
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    DPP_ADD(v, 0xB1, 0xf);   // quad_perm [1,0,3,2]
    DPP_ADD(v, 0x4E, 0xf);   // quad_perm [2,3,0,1]
    DPP_ADD(v, 0x141, 0xf);  // row_half_mirror
    DPP_ADD(v, 0x140, 0xf);  // row_mirror
    DPP_ADD(v, 0x142, 0xa);  // row_bcast:15 -> rows 1, 3
    DPP_ADD(v, 0x143, 0xc);  // row_bcast:31 -> rows 2, 3
    return v;
}

// k_render_bwd: grid (B*V*T), block 256.
__global__ __launch_bounds__(256) void k_render_bwd(int N, int V, int W, int H, int gx, int T,
                                                    const int *__restrict__ tile_start,
                                                    const unsigned *__restrict__ ids,
                                                    const float4 *__restrict__ gA, const float4 *__restrict__ gB,
                                                    const float *__restrict__ gauss, const float *__restrict__ bg,
                                                    const float *__restrict__ final_T,
                                                    const int *__restrict__ n_contrib,
                                                    const float *__restrict__ d_img,
                                                    const float *__restrict__ d_depth,
                                                    const float *__restrict__ d_alpha, float *__restrict__ accum) {
    __shared__ float4 sA[TILE_PIX], sB[TILE_PIX], sC[TILE_PIX];
    __shared__ unsigned sId[TILE_PIX];
    __shared__ float sAcc[TILE_PIX * NACC];
    __shared__ int sMaxLast;
    const int tile = blockIdx.x;
    const int bv = tile / T, t = tile - bv * T, b = bv / V;
    const int tx = t % gx, ty = t / gx;
    int lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const int px = tx * BX + lx, py = ty * BY + ly;
    const bool inside = px < W && py < H;
    const float pfx = (float)px, pfy = (float)py;
    const int s0 = tile_start[tile];
    const size_t P = (size_t)H * W;
    const size_t pid = (size_t)W * (inside ? py : 0) + (inside ? px : 0);

    const float T_final = inside ? final_T[bv * P + pid] : 0.f;
    const int last = inside ? n_contrib[bv * P + pid] : 0;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f, dpd = 0.f, dpa = 0.f;
    if (inside) {
        const float *di = d_img + (size_t)bv * 3 * P;
        dp0 = di[pid]; dp1 = di[P + pid]; dp2 = di[2 * P + pid];
        if (d_depth) dpd = d_depth[bv * P + pid];
        if (d_alpha) dpa = d_alpha[bv * P + pid];
    }
    if (threadIdx.x == 0) sMaxLast = 0;
    __syncthreads();
    if (last > 0) atomicMax(&sMaxLast, last);
    __syncthreads();
    const int nlist = sMaxLast;  // entries beyond every pixel's last contributor are never visited
    if (nlist == 0) return;
    const float bg0 = bg[0], bg1 = bg[1], bg2 = bg[2];
    const float bg_dot = bg0 * dp0 + bg1 * dp1 + bg2 * dp2;
    const float ddelx_dx = 0.5f * W, ddely_dy = 0.5f * H;
    float Tr = T_final;
    float acc_r0 = 0, acc_r1 = 0, acc_r2 = 0, acc_d = 0, acc_a = 0;
    float last_alpha = 0, lc0 = 0, lc1 = 0, lc2 = 0, last_depth = 0;
    int contributor = nlist;
    const int lane = threadIdx.x & 63;
    const size_t gbase = (size_t)bv * N;

    for (int done_cnt = 0; done_cnt < nlist; done_cnt += TILE_PIX) {
        __syncthreads();
        const int k = done_cnt + threadIdx.x;  // position counted from the back
        if (k < nlist) {
            const unsigned gid = ids[s0 + nlist - 1 - k];
            sId[threadIdx.x] = gid;
            sA[threadIdx.x] = gA[gbase + gid];
            const float4 bb = gB[gbase + gid];
            sB[threadIdx.x] = bb;
            const float *c = gauss + ((size_t)b * N + gid) * 14 + 11;
            sC[threadIdx.x] = make_float4(c[0], c[1], c[2], bb.z);
        }
#pragma unroll
        for (int q = 0; q < NACC; q++) sAcc[threadIdx.x * NACC + q] = 0.f;
        __syncthreads();
        const int cnt = min(TILE_PIX, nlist - done_cnt);
        for (int j = 0; j < cnt; j++) {
            contributor--;
            float v[NACC];
#pragma unroll
            for (int q = 0; q < NACC; q++) v[q] = 0.f;
            bool valid = false;
            if (contributor < last) {
                const float4 a = sA[j];
                const float4 bb = sB[j];
                const float dx = a.x - pfx, dy = a.y - pfy;
                const float power = -0.5f * (a.z * dx * dx + bb.x * dy * dy) - a.w * dx * dy;
                if (power <= 0.0f) {
                    const float G = expf(power);
                    const float alpha = fminf(0.99f, bb.y * G);
                    if (alpha >= 1.0f / 255.0f) {
                        valid = true;
                        const float4 c = sC[j];
                        Tr = Tr / (1.f - alpha);
                        const float dchannel_dcolor = alpha * Tr;
                        float dL_dopa = 0.f;
                        acc_r0 = last_alpha * lc0 + (1.f - last_alpha) * acc_r0; lc0 = c.x;
                        dL_dopa += (c.x - acc_r0) * dp0;
                        acc_r1 = last_alpha * lc1 + (1.f - last_alpha) * acc_r1; lc1 = c.y;
                        dL_dopa += (c.y - acc_r1) * dp1;
                        acc_r2 = last_alpha * lc2 + (1.f - last_alpha) * acc_r2; lc2 = c.z;
                        dL_dopa += (c.z - acc_r2) * dp2;
                        v[6] = dchannel_dcolor * dp0;
                        v[7] = dchannel_dcolor * dp1;
                        v[8] = dchannel_dcolor * dp2;
                        acc_d = last_alpha * last_depth + (1.f - last_alpha) * acc_d;
                        last_depth = c.w;
                        dL_dopa += (c.w - acc_d) * dpd;
                        v[9] = dchannel_dcolor * dpd;
                        acc_a = last_alpha + (1.f - last_alpha) * acc_a;
                        dL_dopa += (1 - acc_a) * dpa;
                        dL_dopa *= Tr;
                        last_alpha = alpha;
                        dL_dopa += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = bb.y * dL_dopa;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * a.z - gdy * a.w;
                        const float dG_ddely = -gdy * bb.x - gdx * a.w;
                        v[0] = dL_dG * dG_ddelx * ddelx_dx;
                        v[1] = dL_dG * dG_ddely * ddely_dy;
                        v[2] = -0.5f * gdx * dx * dL_dG;
                        v[3] = -0.5f * gdx * dy * dL_dG;
                        v[4] = -0.5f * gdy * dy * dL_dG;
                        v[5] = G * dL_dopa;
                    }
                }
            }
            if (__ballot(valid)) {  // wave-uniform
                float tot[NACC];
#pragma unroll
                for (int q = 0; q < NACC; q++)
                    tot[q] = __builtin_bit_cast(
                        float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, wave_sum_to_lane63(v[q])), 63));
                float mine = 0.f;
#pragma unroll
                for (int q = 0; q < NACC; q++) mine = (lane == q) ? tot[q] : mine;
                if (lane < NACC) atomicAdd(&sAcc[j * NACC + lane], mine);
            }
        }
        __syncthreads();
        if (k < nlist) {
            const float *a = sAcc + threadIdx.x * NACC;
            float *dst = accum + (gbase + sId[threadIdx.x]) * NACC;
#pragma unroll
            for (int q = 0; q < NACC; q++)
                if (a[q] != 0.f) atomicAdd(dst + q, a[q]);
        }
    }
}

// ------------------------------------------------------------------------------------------------------------
// k_preproc_bwd: grid (ceil(N/256), B), block 256. Sums over the scene's views in order (deterministic).
__global__ __launch_bounds__(256) void k_preproc_bwd(int N, int V, int W, int H, const float *__restrict__ gauss,
                                                     const float *__restrict__ views,
                                                     const float *__restrict__ projs, float tanx, float tany,
                                                     float fx, float fy, float mod, const uint2 *__restrict__ rects,
                                                     const float *__restrict__ accum, float *__restrict__ d_gauss,
                                                     float *__restrict__ d_means2D) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    if (i >= N) return;
    float g[14];
    load_gaussian(gauss + ((size_t)b * N + i) * 14, g);
    float R[3][3];
    const float q4[4] = {g[7], g[8], g[9], g[10]};
    quat_rot(q4, R);
    const float s[3] = {mod * g[4], mod * g[5], mod * g[6]};
    float c3[6];
    cov3d(s, R, c3);
    const float Sg[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float dmean[3] = {0, 0, 0}, dcov[6] = {0, 0, 0, 0, 0, 0}, dop = 0, dcol[3] = {0, 0, 0};
    for (int v = 0; v < V; v++) {
        const int bv = b * V + v;
        const size_t k = (size_t)bv * N + i;
        const uint2 r = rects[k];
        const bool vis = (r.x & 0xffff) != (r.y & 0xffff);
        if (!vis) {
            if (d_means2D) { d_means2D[2 * k] = 0.f; d_means2D[2 * k + 1] = 0.f; }
            continue;
        }
        const float *acc = accum + k * NACC;
        const float dm2x = acc[0], dm2y = acc[1];
        const float dcx = acc[2], dcy = acc[3], dcz = acc[4];
        dop += acc[5];
        dcol[0] += acc[6]; dcol[1] += acc[7]; dcol[2] += acc[8];
        const float ddep = acc[9];
        if (d_means2D) { d_means2D[2 * k] = dm2x; d_means2D[2 * k + 1] = dm2y; }
        const float *Vw = views + 16 * bv;
        const float *Pm = projs + 16 * bv;
        // ---- cov2D backward
        const ProjCtx P = make_proj(Vw, g[0], g[1], g[2], fx, fy, tanx, tany);
        float a, bb, c;
        cov2d(P, c3, a, bb, c);
        const float denom = a * c - bb * bb;
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dcx + 2 * bb * c * dcy + (denom - a * c) * dcz);
            dL_dc = denom2inv * (-a * a * dcz + 2 * a * bb * dcy + (denom - a * c) * dcx);
            dL_db = denom2inv * 2 * (bb * c * dcx - (denom + 2 * bb * bb) * dcy + a * bb * dcz);
            const float *t0 = P.T0, *t1 = P.T1;
            dcov[0] += (t0[0] * t0[0] * dL_da + t0[0] * t1[0] * dL_db + t1[0] * t1[0] * dL_dc);
            dcov[3] += (t0[1] * t0[1] * dL_da + t0[1] * t1[1] * dL_db + t1[1] * t1[1] * dL_dc);
            dcov[5] += (t0[2] * t0[2] * dL_da + t0[2] * t1[2] * dL_db + t1[2] * t1[2] * dL_dc);
            dcov[1] += 2 * t0[0] * t0[1] * dL_da + (t0[0] * t1[1] + t0[1] * t1[0]) * dL_db + 2 * t1[0] * t1[1] * dL_dc;
            dcov[2] += 2 * t0[0] * t0[2] * dL_da + (t0[0] * t1[2] + t0[2] * t1[0]) * dL_db + 2 * t1[0] * t1[2] * dL_dc;
            dcov[4] += 2 * t0[2] * t0[1] * dL_da + (t0[1] * t1[2] + t0[2] * t1[1]) * dL_db + 2 * t1[1] * t1[2] * dL_dc;
        }
        float dT0[3], dT1[3];
#pragma unroll
        for (int kk = 0; kk < 3; kk++) {
            const float s0 = P.T0[0] * Sg[kk][0] + P.T0[1] * Sg[kk][1] + P.T0[2] * Sg[kk][2];
            const float s1 = P.T1[0] * Sg[kk][0] + P.T1[1] * Sg[kk][1] + P.T1[2] * Sg[kk][2];
            dT0[kk] = 2 * s0 * dL_da + s1 * dL_db;
            dT1[kk] = 2 * s1 * dL_dc + s0 * dL_db;
        }
        const float dJ00 = Vw[0] * dT0[0] + Vw[4] * dT0[1] + Vw[8] * dT0[2];
        const float dJ02 = Vw[2] * dT0[0] + Vw[6] * dT0[1] + Vw[10] * dT0[2];
        const float dJ11 = Vw[1] * dT1[0] + Vw[5] * dT1[1] + Vw[9] * dT1[2];
        const float dJ12 = Vw[2] * dT1[0] + Vw[6] * dT1[1] + Vw[10] * dT1[2];
        const float tz = 1.f / P.t[2], tz2 = tz * tz, tz3 = tz2 * tz;
        const float dtx = P.xmul * -fx * tz2 * dJ02;
        const float dty = P.ymul * -fy * tz2 * dJ12;
        const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2 * fx * P.t[0]) * tz3 * dJ02 +
                          (2 * fy * P.t[1]) * tz3 * dJ12;
        dmean[0] += Vw[0] * dtx + Vw[1] * dty + Vw[2] * dtz;
        dmean[1] += Vw[4] * dtx + Vw[5] * dty + Vw[6] * dtz;
        dmean[2] += Vw[8] * dtx + Vw[9] * dty + Vw[10] * dtz;
        // ---- perspective-divide backward
        float hom[4];
        xf44(Pm, g[0], g[1], g[2], hom);
        const float m_w = 1.0f / (hom[3] + 0.0000001f);
        const float mul1 = hom[0] * m_w * m_w;
        const float mul2 = hom[1] * m_w * m_w;
        dmean[0] += (Pm[0] * m_w - Pm[3] * mul1) * dm2x + (Pm[1] * m_w - Pm[3] * mul2) * dm2y;
        dmean[1] += (Pm[4] * m_w - Pm[7] * mul1) * dm2x + (Pm[5] * m_w - Pm[7] * mul2) * dm2y;
        dmean[2] += (Pm[8] * m_w - Pm[11] * mul1) * dm2x + (Pm[9] * m_w - Pm[11] * mul2) * dm2y;
        // ---- depth backward
        dmean[0] += Vw[2] * ddep;
        dmean[1] += Vw[6] * ddep;
        dmean[2] += Vw[10] * ddep;
    }
    // ---- cov3D backward, once on the view-summed dL/dcov3D (linear, so equal to the per-view sum)
    const float dS[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                            {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                            {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
    // dM[c][r] = 2 * s_r * sum_k R[k][r] * dS[c][k]   (glm M = S*R, M[k][r] = s_r R[k][r])
    float dM[3][3];
#pragma unroll
    for (int cc = 0; cc < 3; cc++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
            dM[cc][rr] = 2.0f * s[rr] * (R[0][rr] * dS[cc][0] + R[1][rr] * dS[cc][1] + R[2][rr] * dS[cc][2]);
    float dscale[3], d[3][3];
#pragma unroll
    for (int ii = 0; ii < 3; ii++) {
        dscale[ii] = (R[0][ii] * dM[0][ii] + R[1][ii] * dM[1][ii] + R[2][ii] * dM[2][ii]) * mod;
#pragma unroll
        for (int rr = 0; rr < 3; rr++) d[ii][rr] = dM[rr][ii] * s[ii];  // dL_dMt[ii][rr] * s_ii
    }
    const float r_ = g[7], x = g[8], y = g[9], z = g[10];
    float dq[4];
    dq[0] = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
    dq[1] = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r_ * (d[1][2] - d[2][1]) - 4 * x * (d[2][2] + d[1][1]);
    dq[2] = 2 * x * (d[1][0] + d[0][1]) + 2 * r_ * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) - 4 * y * (d[2][2] + d[0][0]);
    dq[3] = 2 * r_ * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) - 4 * z * (d[1][1] + d[0][0]);
    float *o = d_gauss + ((size_t)b * N + i) * 14;
    const float out[14] = {dmean[0], dmean[1], dmean[2], dop, dscale[0], dscale[1], dscale[2],
                           dq[0], dq[1], dq[2], dq[3], dcol[0], dcol[1], dcol[2]};
    float2 *o2 = reinterpret_cast<float2 *>(o);
#pragma unroll
    for (int kk = 0; kk < 7; kk++) o2[kk] = make_float2(out[2 * kk], out[2 * kk + 1]);
}


struct Dims {
    int B, V, N, H, W, gx, gy, T, BV;
    float fx, fy;
};

int check_common(int B, int V, int N, int H, int W, const void *g, const void *cv, const void *cvp, Dims &d) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0 || H > 16 * 65535 || W > 16 * 65535) {
        lgm::set_error("invalid sizes (B=%d V=%d N=%d H=%d W=%d)", B, V, N, H, W);
        return LGM_E_INVALID;
    }
    if ((N > 0 && !g) || !cv || !cvp) {
        lgm::set_error("null input pointer");
        return LGM_E_INVALID;
    }
    d.B = B; d.V = V; d.N = N; d.H = H; d.W = W;
    d.gx = (W + BX - 1) / BX; d.gy = (H + BY - 1) / BY; d.T = d.gx * d.gy; d.BV = B * V;
    return LGM_OK;
}

int run_preprocess_scan(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                        float tanx, float tany, float mod, char *ws, const Layout &L, long long cap,
                        int *radii_out, long long *stats_out, hipStream_t st) {
    const float fx = d.W / (2.0f * tanx), fy = d.H / (2.0f * tany);
    if (hipMemsetAsync(ws + L.tile_count, 0, (size_t)d.BV * d.T * 4, st) != hipSuccess) {
        lgm::set_error("memset failed");
        return LGM_E_HIP;
    }
    if (d.N > 0) {
        dim3 grid((d.N + 255) / 256, d.BV);
        if (d.T <= LDS_HIST_MAX)
            LGM_LAUNCH("k_preprocess", st, (k_preprocess<true><<<grid, 256, d.T * 4, st>>>(
                d.N, d.V, d.W, d.H, d.gx, d.gy, gaussians, cam_view, cam_view_proj, tanx, tany, fx, fy, mod,
                (float4 *)(ws + L.gA), (float4 *)(ws + L.gB), (uint2 *)(ws + L.rects), (int *)(ws + L.tile_count),
                radii_out)));
        else
            LGM_LAUNCH("k_preprocess", st, (k_preprocess<false><<<grid, 256, 0, st>>>(
                d.N, d.V, d.W, d.H, d.gx, d.gy, gaussians, cam_view, cam_view_proj, tanx, tany, fx, fy, mod,
                (float4 *)(ws + L.gA), (float4 *)(ws + L.gB), (uint2 *)(ws + L.rects), (int *)(ws + L.tile_count),
                radii_out)));
    }
    LGM_LAUNCH("k_scan", st, (k_scan<<<1, 1024, 0, st>>>((const int *)(ws + L.tile_count), d.BV * d.T, (int *)(ws + L.tile_start),
                               (int *)(ws + L.tile_cursor), (long long *)(ws + L.misc), cap, stats_out)));
    return LGM_OK;
}

}  // namespace

// ============================================================================================================
extern "C" {


size_t lgm_render_workspace_size(int B, int V, int N, int H, int W, long long pair_capacity) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0) return 0;
    const long long cap = pair_capacity > 0 ? pair_capacity : worst_capacity(B, V, N, H, W);
    return make_layout(B, V, N, H, W, cap).total;
}

int lgm_render_count_pairs(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                           const float *cam_view_proj, float tanfovx, float tanfovy, float scale_modifier,
                           void *workspace, size_t workspace_bytes, long long *pairs_out, void *stream) {
    lgm::clear_error();
    Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, d);
    if (rc) return rc;
    const Layout L = make_layout(B, V, N, H, W, 1);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small for counting");
        return LGM_E_WORKSPACE;
    }
    long long *stats = pairs_out;
    return run_preprocess_scan(d, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier,
                               (char *)workspace, L, (long long)1 << 62, nullptr, stats, (hipStream_t)stream);
}

int lgm_render_forward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                       const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                       float scale_modifier, float *image, float *depth, float *alpha, int *radii_out,
                       void *workspace, size_t workspace_bytes, long long pair_capacity, long long *stats_out,
                       void *stream) {
    lgm::clear_error();
    Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, d);
    if (rc) return rc;
    if (!bg || !image || !depth || !alpha) {
        lgm::set_error("null output pointer");
        return LGM_E_INVALID;
    }
    const long long cap = pair_capacity > 0 ? pair_capacity : worst_capacity(B, V, N, H, W);
    if (cap > 0x7fffffffLL) {
        lgm::set_error("pair capacity exceeds 2^31");
        return LGM_E_INVALID;
    }
    const Layout L = make_layout(B, V, N, H, W, cap);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small");
        return LGM_E_WORKSPACE;
    }
    char *ws = (char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    rc = run_preprocess_scan(d, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, ws, L, cap,
                             radii_out, stats_out, st);
    if (rc) return rc;
    if (N > 0) {
        dim3 grid((N + 255) / 256, d.BV);
        if (d.T <= LDS_HIST_MAX)
            LGM_LAUNCH("k_emit", st, (k_emit<true><<<grid, 256, 2 * d.T * 4, st>>>(N, d.gx, d.gy, (const uint2 *)(ws + L.rects),
                                                          (const float4 *)(ws + L.gB), (int *)(ws + L.tile_cursor),
                                                          (unsigned long long *)(ws + L.keys), cap)));
        else
            LGM_LAUNCH("k_emit", st, (k_emit<false><<<grid, 256, 0, st>>>(N, d.gx, d.gy, (const uint2 *)(ws + L.rects),
                                                (const float4 *)(ws + L.gB), (int *)(ws + L.tile_cursor),
                                                (unsigned long long *)(ws + L.keys), cap)));
        LGM_LAUNCH("k_sort", st, (k_sort<<<d.BV * d.T, SORT_THREADS, SORT_CAP * 8, st>>>((const int *)(ws + L.tile_start),
                                                                (unsigned long long *)(ws + L.keys),
                                                                (unsigned *)(ws + L.ids))));
    }
    LGM_LAUNCH("k_render_fwd", st, (k_render_fwd<<<d.BV * d.T, 256, 0, st>>>(N, V, W, H, d.gx, d.T, (const int *)(ws + L.tile_start),
                                             (const unsigned *)(ws + L.ids), (const float4 *)(ws + L.gA),
                                             (const float4 *)(ws + L.gB), gaussians, bg, image, depth, alpha,
                                             (float *)(ws + L.final_T), (int *)(ws + L.n_contrib))));
    return LGM_OK;
}

int lgm_render_backward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                        const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                        float scale_modifier, const float *d_image, const float *d_depth, const float *d_alpha,
                        float *d_gaussians, float *d_means2D, void *workspace, size_t workspace_bytes,
                        long long pair_capacity, void *stream) {
    lgm::clear_error();
    Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, d);
    if (rc) return rc;
    if (!bg || !d_image || (N > 0 && !d_gaussians)) {
        lgm::set_error("null pointer in backward");
        return LGM_E_INVALID;
    }
    const long long cap = pair_capacity > 0 ? pair_capacity : worst_capacity(B, V, N, H, W);
    const Layout L = make_layout(B, V, N, H, W, cap);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small");
        return LGM_E_WORKSPACE;
    }
    if (N == 0) return LGM_OK;
    char *ws = (char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(ws + L.accum, 0, (size_t)d.BV * N * NACC * 4, st) != hipSuccess) {
        lgm::set_error("memset failed");
        return LGM_E_HIP;
    }
    LGM_LAUNCH("k_render_bwd", st, (k_render_bwd<<<d.BV * d.T, 256, 0, st>>>(N, V, W, H, d.gx, d.T, (const int *)(ws + L.tile_start),
                                             (const unsigned *)(ws + L.ids), (const float4 *)(ws + L.gA),
                                             (const float4 *)(ws + L.gB), gaussians, bg,
                                             (const float *)(ws + L.final_T), (const int *)(ws + L.n_contrib),
                                             d_image, d_depth, d_alpha, (float *)(ws + L.accum))));
    const float fx = W / (2.0f * tanfovx), fy = H / (2.0f * tanfovy);
    dim3 grid((N + 255) / 256, B);
    LGM_LAUNCH("k_preproc_bwd", st, (k_preproc_bwd<<<grid, 256, 0, st>>>(N, V, W, H, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, fx, fy,
                                        scale_modifier, (const uint2 *)(ws + L.rects),
                                        (const float *)(ws + L.accum), d_gaussians, d_means2D)));
    return LGM_OK;
}

}  // extern "C"
