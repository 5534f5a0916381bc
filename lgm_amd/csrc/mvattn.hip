// lgm_amd/csrc/mvattn.hip -- the token layout changes around MVAttention's attention core (core/unet.py:35-49),
// fused with the GroupNorm before and the residual after:
//   k_mva_gn_reg (slab in registers; else k_mva_gn_tok with the slab in LDS, or for slabs beyond LDS k_mva_stats +
//   k_mva_norm)  GroupNorm(x) of [B*F, C, H, W]
//                (core/unet.py:40, fp32 statistics), written straight into the [B, F*H*W, C] token layout of :41-42
//                in the qkv Linear's input dtype (bf16 under autocast): one launch instead of torch's moments /
//                fused-params / normalise launches + the permute copy + the cast.
//   k_mva_out    the [B, F*H*W, C] -> [B*F, C, H, W] permute of :45-46 fused with (x + res) * skip_scale of :47-48.
// Both are HBM-bound layout kernels: 64x64 LDS-tiled transposes, so global reads and writes run along rows.
#include <hip/hip_bf16.h>
#include <initializer_list>
#include <hip/hip_fp16.h>

#include "common.h"
#include "lgm_attn.h"

namespace lgm {
namespace {

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(__hip_bfloat16 v) { return __bfloat162float(v); }
__device__ __forceinline__ float to_f(__half v) { return __half2float(v); }
template <class T> __device__ __forceinline__ T from_f(float v);
template <> __device__ __forceinline__ float from_f<float>(float v) { return v; }
template <> __device__ __forceinline__ __hip_bfloat16 from_f<__hip_bfloat16>(float v) { return __float2bfloat16(v); }
template <> __device__ __forceinline__ __half from_f<__half>(float v) { return __float2half(v); }

__device__ __forceinline__ float block_sum256(float v, float *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // red is reused between calls
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);  // fixed order: every thread gets the same value
}

// GroupNorm statistics in two launches, all deterministic:
// k_mva_stats  grid (S, G, B*F): chunk s of group g of sample bf (the group's Cg*HW elements are contiguous) ->
//              its mean and centred sum of squares (two passes over the chunk, which stays in L1/L2).
// k_mva_norm   grid (ceil(HW/64), ceil(C/64), B*F): merges the chunk statistics of the groups its 64 channels
//              belong to (Chan's parallel formula, fixed order), then normalises a 64-channel x 64-pixel tile
//              through LDS: reads along hw, writes token rows along c. y = x (rstd gamma) + (beta - mean rstd gamma),
//              torch's fused GroupNorm parameters.
constexpr int MVA_CHUNK = 4096;  // elements per statistics workgroup

__device__ __forceinline__ int mva_chunks(int n) { return (n + MVA_CHUNK - 1) / MVA_CHUNK; }

template <class TI>
__global__ __launch_bounds__(256) void k_mva_stats(int C, int HW, int G, const TI *__restrict__ x,
                                                   float2 *__restrict__ part) {
    __shared__ float red[4];
    const int s = blockIdx.x, g = blockIdx.y, bf = blockIdx.z, Cg = C / G, tid = threadIdx.x;
    const int n = Cg * HW, S = mva_chunks(n);
    const int i0 = s * MVA_CHUNK, i1 = min(n, i0 + MVA_CHUNK), m = i1 - i0;
    const TI *xg = x + ((size_t)bf * C + (size_t)g * Cg) * HW;
    float v[MVA_CHUNK / 256];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < MVA_CHUNK / 256; k++) {
        const int i = i0 + k * 256 + tid;
        const float t = to_f(xg[i < i1 ? i : i0]);  // unconditional loads (clamped index): all in flight at once
        v[k] = i < i1 ? t : 0.f;
        sum += v[k];
    }
    const float mean = block_sum256(sum, red) / (float)m;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < MVA_CHUNK / 256; k++) {
        const float d = i0 + k * 256 + tid < i1 ? v[k] - mean : 0.f;
        q = fmaf(d, d, q);
    }
    q = block_sum256(q, red);
    if (tid == 0) part[((size_t)bf * G + g) * S + s] = make_float2(mean, q);
}

template <class TI, class TO>
__global__ __launch_bounds__(256) void k_mva_norm(int F, int C, int HW, int G, float eps, const TI *__restrict__ x,
                                                  const float *__restrict__ gamma, const float *__restrict__ beta,
                                                  const float2 *__restrict__ part, TO *__restrict__ tok,
                                                  float *__restrict__ mean_out, float *__restrict__ rstd_out) {
    __shared__ float tile[64][65];  // [pixel][channel]
    __shared__ float sa[64], sb[64];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int Cg = C / G, n = Cg * HW, S = mva_chunks(n);
    if (tid < 64 && c0 + tid < C) {  // this channel's group statistics (Chan merge of the chunks, in order)
        const int c = c0 + tid, g = c / Cg;
        const float2 *pg = part + ((size_t)bf * G + g) * S;
        float mean = 0.f, M2 = 0.f;
        int cnt = 0;
        for (int s2 = 0; s2 < S; s2++) {
            const float2 p = pg[s2];
            const int m = min(n, (s2 + 1) * MVA_CHUNK) - s2 * MVA_CHUNK;
            const int tot = cnt + m;
            const float d = p.x - mean;
            mean = fmaf(d, (float)m / (float)tot, mean);
            M2 += p.y + d * d * ((float)cnt * (float)m / (float)tot);
            cnt = tot;
        }
        const float rstd = rsqrtf(fmaxf(M2 / (float)n, 0.f) + eps);  // biased variance, as torch
        const float a = rstd * (gamma ? gamma[c] : 1.f);
        sa[tid] = a;
        sb[tid] = (beta ? beta[c] : 0.f) - mean * a;
        if (blockIdx.x == 0 && c % Cg == 0) {  // one writer per (sample, group)
            mean_out[(size_t)bf * G + g] = mean;
            rstd_out[(size_t)bf * G + g] = rstd;
        }
    }
    __syncthreads();
    const TI *xb = x + (size_t)bf * C * HW;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // all 16 loads issued before the first use (clamped, unconditional addresses)
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
        const bool ok = hw0 + h < HW && c0 + r < C;
        v[k] = to_f(xb[ok ? (size_t)(c0 + r) * HW + hw0 + h : 0]);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;
        tile[h][r] = fmaf(v[k], sa[r], sb[r]);
    }
    __syncthreads();
    const int b = bf / F, f = bf - b * F;
    TO *tb = tok + ((size_t)b * F * HW + (size_t)f * HW) * C;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;  // token row r, channel c
        if (hw0 + r < HW && c0 + c < C) tb[(size_t)(hw0 + r) * C + c0 + c] = from_f<TO>(tile[r][c]);
    }
}

// k_mva_gn_tok  grid (G, B*F), block 512: the same GroupNorm -> tokens in ONE launch where a group's Cg x HW slab
//               fits in LDS (every LGM level: <= 100 KB): the slab is read once into LDS (float4 loads for fp32
//               input), its mean and centred sum of squares reduced in a fixed order (two passes over LDS), then
//               written normalised along the token rows (Cg / 8 x 16-B stores per token). Replaces the chunked
//               statistics launch + the tiled normalise launch (their fixed launch latency dominated LGM's small
//               levels: 600 and 2,400 tokens at C = 1024). cfg4's 16 blocks: GPU span per pass 2.43 -> 2.38 ms
//               (profiles/r05/ab_mva_gn_fused). The slab loads go 8 per thread at a time (the plain loop waited for
//               each before issuing the next): bench level 34.2 -> 32.2 us, cfg4 190.8 -> 182.9 us per pass
//               (profiles/r05/ab_mva_batch); the same for k_mva_gn_coef's tile partials (13.8 -> 11.5 us).
constexpr int GN_THREADS = 512;
constexpr size_t GN_LDS_MAX = 144 * 1024;  // bytes of dynamic LDS the fused form may take

__device__ __forceinline__ float block_sum512(float v, float *red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int w = threadIdx.x >> 6;
    __syncthreads();  // red is reused between calls
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + (red[2] + red[3])) + ((red[4] + red[5]) + (red[6] + red[7]));  // fixed order
}

template <class TI, class TO>
__global__ __launch_bounds__(GN_THREADS) void k_mva_gn_tok(int F, int C, int HW, int G, float eps,
                                                            const TI *__restrict__ x, const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, TO *__restrict__ tok,
                                                            float *__restrict__ mean_out, float *__restrict__ rstd_out) {
    extern __shared__ __attribute__((aligned(16))) float slab[];  // [Cg][HW], then a[Cg], b[Cg]
    __shared__ float red[8];
    const int g = blockIdx.x, bf = blockIdx.y, Cg = C / G, n = Cg * HW, tid = threadIdx.x;
    const TI *xg = x + ((size_t)bf * C + (size_t)g * Cg) * HW;
    float s = 0.f;
    if constexpr (sizeof(TI) == 4) {
        if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(xg) & 15) == 0) {
            const float4 *x4 = reinterpret_cast<const float4 *>(xg);
            int i = tid;
            // 8 loads in flight per thread, then their LDS stores and sums in the same order (the plain loop waited
            // for each load before issuing the next)
            for (; i + 7 * GN_THREADS < n / 4; i += 8 * GN_THREADS) {
                float4 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = x4[i + u * GN_THREADS];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    reinterpret_cast<float4 *>(slab)[i + u * GN_THREADS] = v[u];
                    s += (v[u].x + v[u].y) + (v[u].z + v[u].w);
                }
            }
            for (; i < n / 4; i += GN_THREADS) {
                const float4 v = x4[i];
                reinterpret_cast<float4 *>(slab)[i] = v;
                s += (v.x + v.y) + (v.z + v.w);
            }
        } else {
            for (int i = tid; i < n; i += GN_THREADS) { const float v = to_f(xg[i]); slab[i] = v; s += v; }
        }
    } else {
        int i = tid;
        for (; i + 7 * GN_THREADS < n; i += 8 * GN_THREADS) {  // (as above, 16-bit elements)
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; u++) v[u] = to_f(xg[i + u * GN_THREADS]);
#pragma unroll
            for (int u = 0; u < 8; u++) {
                slab[i + u * GN_THREADS] = v[u];
                s += v[u];
            }
        }
        for (; i < n; i += GN_THREADS) { const float v = to_f(xg[i]); slab[i] = v; s += v; }
    }
    const float mean = block_sum512(s, red) / (float)n;
    float q = 0.f;
    for (int i = tid; i < n; i += GN_THREADS) {
        const float d = slab[i] - mean;
        q = fmaf(d, d, q);
    }
    const float rstd = rsqrtf(block_sum512(q, red) / (float)n + eps);  // biased variance, as torch
    float *sa = slab + n, *sb = sa + Cg;
    for (int c = tid; c < Cg; c += GN_THREADS) {
        const float a = rstd * (gamma ? gamma[g * Cg + c] : 1.f);
        sa[c] = a;
        sb[c] = (beta ? beta[g * Cg + c] : 0.f) - mean * a;
    }
    if (tid == 0) {
        mean_out[(size_t)bf * G + g] = mean;
        rstd_out[(size_t)bf * G + g] = rstd;
    }
    __syncthreads();
    const int b = bf / F, f = bf - b * F;
    TO *tb = tok + ((size_t)b * F * HW + (size_t)f * HW) * C + (size_t)g * Cg;
    if ((Cg & 7) == 0) {  // 8 channels per thread: one 16-B (bf16) / 32-B (fp32) store
        const int c8n = Cg / 8;
        for (int p = tid; p < HW * c8n; p += GN_THREADS) {
            const int hw = p / c8n, c0 = (p - hw * c8n) * 8;
            TO o[8];
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = from_f<TO>(fmaf(slab[(c0 + j) * HW + hw], sa[c0 + j], sb[c0 + j]));
            TO *dst = tb + (size_t)hw * C + c0;
            if constexpr (sizeof(TO) == 2) {
                *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(o);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++) dst[j] = o[j];
            }
        }
    } else {
        for (int p = tid; p < HW * Cg; p += GN_THREADS) {
            const int hw = p / Cg, c = p - hw * Cg;
            tb[(size_t)hw * C + c] = from_f<TO>(fmaf(slab[c * HW + hw], sa[c], sb[c]));
        }
    }
}

// k_mva_gn_reg  grid (G, B*F), block 512: the one-launch GroupNorm -> tokens with the group's slab in REGISTERS
//               instead of LDS, for Cg % 8 == 0 channels, HW % 4 == 0 and <= GNR_K * 512 items (every LGM level). An
//               item is 8 channel rows x 4 pixels: thread t holds items t + 512 k (channel block fastest, so the lanes
//               of one pixel quad write adjacent 16 B of each token row), loaded as one 4-pixel vector per channel row,
//               all in flight at once; the statistics are
//               reduced in a fixed order (two passes over the registers); each pixel of an item is written as one
//               token-row store of 8 channels. No LDS slab, so LDS does not cap the launch at two workgroups per CU.
//               Against k_mva_gn_tok: bench level 31.8 -> 29.5 us, cfg4 184.4 -> 153.3 us per pass (its C = 512 level
//               has 192 workgroups: all loads in flight at once matters most there; profiles/r05/ab_mva_gn_reg).
constexpr int GNR_K = 2;  // items per thread (64 registers of slab)
template <class TI>
__device__ __forceinline__ void load4(const TI *p, float (&o)[4]) {
    if constexpr (sizeof(TI) == 4) {
        const float4 t = *reinterpret_cast<const float4 *>(p);
        o[0] = t.x; o[1] = t.y; o[2] = t.z; o[3] = t.w;
    } else {
        const uint2 t = *reinterpret_cast<const uint2 *>(p);
        TI e[4];
        *reinterpret_cast<uint2 *>(e) = t;
#pragma unroll
        for (int j = 0; j < 4; j++) o[j] = to_f(e[j]);
    }
}
template <class TI, class TO>
__global__ __launch_bounds__(GN_THREADS) void k_mva_gn_reg(int F, int C, int HW, int G, float eps,
                                                            const TI *__restrict__ x, const float *__restrict__ gamma,
                                                            const float *__restrict__ beta, TO *__restrict__ tok,
                                                            float *__restrict__ mean_out, float *__restrict__ rstd_out) {
    __shared__ float red[8];
    __shared__ float sab[2][256];  // per channel of the group: a = rstd gamma, b = beta - mean a (Cg <= 256)
    const int g = blockIdx.x, bf = blockIdx.y, Cg = C / G, tid = threadIdx.x;
    const int nCB = Cg / 8, nit = nCB * (HW / 4);  // items (channel block fastest: lane pairs share a pixel quad)
    const TI *xg = x + ((size_t)bf * C + (size_t)g * Cg) * HW;
    float v[GNR_K][8][4];
#pragma unroll
    for (int k = 0; k < GNR_K; k++) {
        const int it = tid + GN_THREADS * k;
        const int p4 = it / nCB, cb = it - p4 * nCB;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            if (it < nit) load4<TI>(xg + (size_t)(8 * cb + j) * HW + 4 * p4, v[k][j]);
            else v[k][j][0] = v[k][j][1] = v[k][j][2] = v[k][j][3] = 0.f;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < GNR_K; k++)
#pragma unroll
        for (int j = 0; j < 8; j++) s += (v[k][j][0] + v[k][j][1]) + (v[k][j][2] + v[k][j][3]);  // (past nit: 0)
    const float n = (float)Cg * (float)HW;
    const float mean = block_sum512(s, red) / n;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < GNR_K; k++) {
        if (tid + GN_THREADS * k < nit) {
#pragma unroll
            for (int j = 0; j < 8; j++)
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    const float d = v[k][j][e] - mean;
                    q = fmaf(d, d, q);
                }
        }
    }
    const float rstd = rsqrtf(block_sum512(q, red) / n + eps);  // biased variance, as torch
    for (int c = tid; c < Cg; c += GN_THREADS) {
        const float a = rstd * (gamma ? gamma[g * Cg + c] : 1.f);
        sab[0][c] = a;
        sab[1][c] = (beta ? beta[g * Cg + c] : 0.f) - mean * a;
    }
    if (tid == 0) {
        mean_out[(size_t)bf * G + g] = mean;
        rstd_out[(size_t)bf * G + g] = rstd;
    }
    __syncthreads();
    const int b = bf / F, f = bf - b * F;
    TO *tb = tok + ((size_t)b * F * HW + (size_t)f * HW) * C + (size_t)g * Cg;
#pragma unroll
    for (int k = 0; k < GNR_K; k++) {
        const int it = tid + GN_THREADS * k;
        if (it < nit) {
            const int p4 = it / nCB, cb = it - p4 * nCB;
            float a8[8], b8[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                a8[j] = sab[0][8 * cb + j];
                b8[j] = sab[1][8 * cb + j];
            }
#pragma unroll
            for (int e = 0; e < 4; e++) {
                TO o[8];
#pragma unroll
                for (int j = 0; j < 8; j++) o[j] = from_f<TO>(fmaf(v[k][j][e], a8[j], b8[j]));
                TO *dst = tb + (size_t)(4 * p4 + e) * C + 8 * cb;
                if constexpr (sizeof(TO) == 2) {
                    *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(o);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; j++) dst[j] = o[j];
                }
            }
        }
    }
}

// grid (ceil(HW/64), ceil(C/64), B*F), block 256: out[bf][c][hw] = (y[b][f HW + hw][c] + res[bf][c][hw]) * skip
// through a 64 x 64 LDS tile (reads along c, writes along hw). In a lower-precision output the sum is rounded
// before the scale, as torch's two ops do.
template <class TY, class TR, class TO>
__global__ __launch_bounds__(256) void k_mva_out(int F, int C, int HW, const TY *__restrict__ y,
                                                 const TR *__restrict__ res, float skip, TO *__restrict__ out) {
    __shared__ float tile[64][65];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int b = bf / F, f = bf - b * F;
    const TY *yb = y + ((size_t)b * F * HW + (size_t)f * HW) * C;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // all loads in flight before the first use (clamped, unconditional addresses)
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;  // token row r, channel c
        const bool ok = hw0 + r < HW && c0 + c < C;
        v[k] = to_f(yb[ok ? (size_t)(hw0 + r) * C + c0 + c : 0]);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;
        tile[c][r] = v[k];
    }
    float rv[16];
    if (res) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
            const bool ok = hw0 + h < HW && c0 + r < C;
            rv[k] = to_f(res[ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + h : 0]);
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
        if (hw0 + h < HW && c0 + r < C) {
            const size_t o = ((size_t)bf * C + c0 + r) * HW + hw0 + h;
            float t = tile[r][h];
            if (res) {
                t += rv[k];
                t = to_f(from_f<TO>(t));  // (exact for an fp32 output)
                t *= skip;
            }
            out[o] = from_f<TO>(t);
        }
    }
}

template <class T>
__device__ __forceinline__ void load8(const T *p, float (&o)[8]) {
    if constexpr (sizeof(T) == 4) {
        const float4 a = reinterpret_cast<const float4 *>(p)[0], b = reinterpret_cast<const float4 *>(p)[1];
        o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
    } else {
        T e[8];
        *reinterpret_cast<uint4 *>(e) = *reinterpret_cast<const uint4 *>(p);
#pragma unroll
        for (int j = 0; j < 8; j++) o[j] = to_f(e[j]);
    }
}
template <class T>
__device__ __forceinline__ void store4(T *p, const float (&v)[4]) {
    if constexpr (sizeof(T) == 4) {
        *reinterpret_cast<float4 *>(p) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
        T e[4];
#pragma unroll
        for (int j = 0; j < 4; j++) e[j] = from_f<T>(v[j]);
        *reinterpret_cast<uint2 *>(p) = *reinterpret_cast<const uint2 *>(e);
    }
}
// k_mva_out with vector accesses (C % 8 == 0, HW % 4 == 0, 16-B aligned tensors): the tokens read 8 channels per
// lane (16 B at 16 bits), the residual read and the output written 4 pixels per lane; the residual's loads go out
// with the tokens' (one round trip). Same arithmetic, bitwise equal. Against k_mva_out: bench level 37.0 -> 31.2 us,
// cfg4 171.6 -> 141.0 us per pass (profiles/r05/ab_mva_vec).
template <class TY, class TR, class TO>
__global__ __launch_bounds__(256) void k_mva_out_v(int F, int C, int HW, const TY *__restrict__ y,
                                                   const TR *__restrict__ res, float skip, TO *__restrict__ out) {
    __shared__ float tile[64][65];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int b = bf / F, f = bf - b * F;
    const TY *yb = y + ((size_t)b * F * HW + (size_t)f * HW) * C;
    float v[2][8], rv[4][4];
    // every load unconditional, out-of-range lanes on a clamped in-range address (their values are never used), so
    // all six go out before the first wait
#pragma unroll
    for (int k = 0; k < 2; k++) {  // token row r, channels 8 q .. 8 q + 7
        const int i = tid + 256 * k, r = i >> 3, q = i & 7;
        const bool ok = hw0 + r < HW && c0 + 8 * q < C;
        load8<TY>(yb + (ok ? (size_t)(hw0 + r) * C + c0 + 8 * q : 0), v[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {  // channel row r, pixels 4 p .. 4 p + 3
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        const bool ok = c0 + r < C && hw0 + 4 * p < HW;
        if (res) {
            const TR *src = res + (ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p : 0);
            if constexpr (sizeof(TR) == 4) {
                const float4 a = *reinterpret_cast<const float4 *>(src);
                rv[k][0] = a.x; rv[k][1] = a.y; rv[k][2] = a.z; rv[k][3] = a.w;
            } else {
                TR e[4];
                *reinterpret_cast<uint2 *>(e) = *reinterpret_cast<const uint2 *>(src);
#pragma unroll
                for (int j = 0; j < 4; j++) rv[k][j] = to_f(e[j]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int i = tid + 256 * k, r = i >> 3, q = i & 7;
#pragma unroll
        for (int j = 0; j < 8; j++) tile[8 * q + j][r] = v[k][j];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        if (c0 + r < C && hw0 + 4 * p < HW) {
            float o4[4];
#pragma unroll
            for (int e = 0; e < 4; e++) {
                float t = tile[r][4 * p + e];
                if (res) {
                    t += rv[k][e];
                    t = to_f(from_f<TO>(t));  // (exact for an fp32 output)
                    t *= skip;
                }
                o4[e] = t;
            }
            store4<TO>(out + ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p, o4);
        }
    }
}

// ---- backward (core/unet.py:40-48 backward), the mirror of the two passes above:
// k_mva_out_bwd   grid (ceil(HW/64), ceil(C/64), B*F): g = dL/dout * scale (rounded to out's dtype, as torch's
//                 `d_out * skip`), written to d_res [B*F, C, H, W] along hw and, through the 64 x 64 LDS tile, to the
//                 tokens' gradient d_y [B, F*H*W, C] along c.
// k_mva_gn_part   grid (ceil(HW/64), ceil(C/64), B*F): per (sample, channel, 64-pixel tile) partial sums of
//                 dy * x and dy (dy = the token gradient read back through the LDS tile) -> part2
// k_mva_gn_coef   grid (G): per (sample, channel) ds = sum dy x, db = sum dy (fixed order over the tiles), then per
//                 (sample, group) torch's fused backward parameters c2, c3 and per channel dgamma, dbeta (fixed
//                 order over the samples): deterministic
// k_mva_gn_dx     grid (ceil(HW/64), ceil(C/64), B*F): dx = rstd gamma dy + c2 x + c3 (+ d_res), one rounding to
//                 x's dtype: the GroupNorm backward and autograd's sum with the residual's gradient in one pass.
template <class TD, class TY, class TR>
__global__ __launch_bounds__(256) void k_mva_out_bwd(int F, int C, int HW, const TD *__restrict__ dout, float scale,
                                                     TY *__restrict__ dy, TR *__restrict__ dres) {
    __shared__ float tile[64][65];  // [channel][pixel]
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // all loads in flight before the first use (clamped, unconditional addresses)
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
        const bool ok = hw0 + h < HW && c0 + r < C;
        v[k] = to_f(dout[ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + h : 0]);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;
        const float g = to_f(from_f<TD>(v[k] * scale));  // (exact: scale 1 and an fp32 gradient)
        tile[r][h] = g;
        if (dres && hw0 + h < HW && c0 + r < C) dres[((size_t)bf * C + c0 + r) * HW + hw0 + h] = from_f<TR>(g);
    }
    __syncthreads();
    const int b = bf / F, f = bf - b * F;
    TY *yb = dy + ((size_t)b * F * HW + (size_t)f * HW) * C;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;  // token row r, channel c
        if (hw0 + r < HW && c0 + c < C) yb[(size_t)(hw0 + r) * C + c0 + c] = from_f<TY>(tile[c][r]);
    }
}

// the token gradient of a 64-channel x 64-pixel tile into LDS as [pixel][channel] (reads along c), zero outside
template <class TT>
__device__ __forceinline__ void load_tok_tile(float (&tile)[64][65], const TT *__restrict__ tok, int F, int C, int HW,
                                              int bf, int hw0, int c0) {
    const int b = bf / F, f = bf - b * F, tid = threadIdx.x;
    const TT *tb = tok + ((size_t)b * F * HW + (size_t)f * HW) * C;
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;  // token row r, channel c
        const bool ok = hw0 + r < HW && c0 + c < C;
        v[k] = to_f(tb[ok ? (size_t)(hw0 + r) * C + c0 + c : 0]);
        v[k] = ok ? v[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, c = i & 63;
        tile[r][c] = v[k];
    }
}

template <class TI, class TT>
__global__ __launch_bounds__(256) void k_mva_gn_part(int F, int C, int HW, const TI *__restrict__ x,
                                                     const TT *__restrict__ dtok, float2 *__restrict__ part) {
    __shared__ float tile[64][65];  // dy [pixel][channel]
    __shared__ float xs[64][65];    // x [channel][pixel]
    __shared__ float2 red[4][64];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int nT = gridDim.x;
    {
        float xv[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {  // x along hw (zero outside), issued before the token tile's loads
            const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
            const bool ok = hw0 + h < HW && c0 + r < C;
            xv[k] = to_f(x[ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + h : 0]);
            xv[k] = ok ? xv[k] : 0.f;
        }
        load_tok_tile(tile, dtok, F, C, HW, bf, hw0, c0);
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int i = tid + 256 * k, r = i >> 6, h = i & 63;
            xs[r][h] = xv[k];
        }
    }
    __syncthreads();
    // thread: channel c = tid & 63, pixels 16 q .. 16 q + 15 (q = the wave); the four quarters summed in order
    const int c = tid & 63, q = tid >> 6;
    float sdx = 0.f, sd = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int h = 16 * q + k;
        const float g = tile[h][c];
        sd += g;
        sdx = fmaf(g, xs[c][h], sdx);
    }
    red[q][c] = make_float2(sdx, sd);
    __syncthreads();
    if (tid < 64 && c0 + tid < C) {
        const float2 a = red[0][tid], b2 = red[1][tid], c2 = red[2][tid], d2 = red[3][tid];
        part[((size_t)bf * C + c0 + tid) * nT + blockIdx.x] =
            make_float2((a.x + b2.x) + (c2.x + d2.x), (a.y + b2.y) + (c2.y + d2.y));
    }
}

constexpr int GN_NMAX = 2048;  // (sample, channel) pairs of one group held in LDS at a time
constexpr int GN_CPT = GN_NMAX / 256;  // channels per thread of k_mva_gn_coef (any Cg <= GN_NMAX)
__global__ __launch_bounds__(256) void k_mva_gn_coef(int BF, int C, int HW, int G, int nT,
                                                     const float2 *__restrict__ part, const float *__restrict__ gamma,
                                                     const float *__restrict__ mean, const float *__restrict__ rstd,
                                                     float2 *__restrict__ coef, float *__restrict__ dgamma,
                                                     float *__restrict__ dbeta) {
    __shared__ float2 sdb[GN_NMAX];  // (ds, db) of the chunk's (sample, channel) pairs
    const int g = blockIdx.x, Cg = C / G, tid = threadIdx.x;
    const float s = 1.f / ((float)Cg * (float)HW);
    const int nchunk = max(1, GN_NMAX / Cg);  // samples per LDS chunk
    // this thread's channels tid + 256 k (k < GN_CPT, Cg <= GN_NMAX), each summed over the samples in order
    float dg[GN_CPT], dbt[GN_CPT];
#pragma unroll
    for (int k = 0; k < GN_CPT; k++) dg[k] = dbt[k] = 0.f;
    for (int n0 = 0; n0 < BF; n0 += nchunk) {
        const int n1 = min(BF, n0 + nchunk), items = (n1 - n0) * Cg;
        for (int it = tid; it < items; it += 256) {
            const int n = n0 + it / Cg, c = g * Cg + it % Cg;
            const float2 *pp = part + ((size_t)n * C + c) * nT;
            float a = 0.f, b = 0.f;
            int t = 0;
            for (; t + 8 <= nT; t += 8) {  // 8 loads in flight, then the sums in the same fixed order
                float2 p[8];
#pragma unroll
                for (int u = 0; u < 8; u++) p[u] = pp[t + u];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    a += p[u].x;
                    b += p[u].y;
                }
            }
            for (; t < nT; t++) {  // fixed order over the pixel tiles
                const float2 p = pp[t];
                a += p.x;
                b += p.y;
            }
            sdb[it] = make_float2(a, b);
        }
        __syncthreads();
        for (int n = n0 + tid; n < n1; n += 256) {  // per sample: torch's fused backward parameters
            float sum1 = 0.f, sum2 = 0.f;
            for (int cc = 0; cc < Cg; cc++) {
                const float ga = gamma ? gamma[g * Cg + cc] : 1.f;
                const float2 v = sdb[(n - n0) * Cg + cc];
                sum1 = fmaf(v.x, ga, sum1);
                sum2 = fmaf(v.y, ga, sum2);
            }
            const float mu = mean[(size_t)n * G + g], rs = rstd[(size_t)n * G + g];
            const float c2 = (sum2 * mu - sum1) * rs * rs * rs * s;
            const float c3 = -c2 * mu - sum2 * rs * s;
            coef[(size_t)n * G + g] = make_float2(c2, c3);
        }
#pragma unroll
        for (int k = 0; k < GN_CPT; k++) {  // per channel: dgamma, dbeta over this chunk's samples, in order
            const int c = tid + 256 * k;
            if (c < Cg) {
                for (int n = n0; n < n1; n++) {
                    const float2 v = sdb[(n - n0) * Cg + c];
                    const float mu = mean[(size_t)n * G + g], rs = rstd[(size_t)n * G + g];
                    dg[k] = fmaf(v.x - v.y * mu, rs, dg[k]);
                    dbt[k] += v.y;
                }
            }
        }
        __syncthreads();  // (sdb is rewritten by the next chunk)
    }
#pragma unroll
    for (int k = 0; k < GN_CPT; k++) {
        const int c = tid + 256 * k;
        if (c < Cg) {
            if (dgamma) dgamma[g * Cg + c] = dg[k];
            if (dbeta) dbeta[g * Cg + c] = dbt[k];
        }
    }
}

template <class TI, class TT, class TR>
__global__ __launch_bounds__(256) void k_mva_gn_dx(int F, int C, int HW, int G, const TI *__restrict__ x,
                                                   const TT *__restrict__ dtok, const TR *__restrict__ dres,
                                                   const float *__restrict__ gamma, const float *__restrict__ rstd,
                                                   const float2 *__restrict__ coef, TI *__restrict__ dx) {
    __shared__ float tile[64][65];  // [pixel][channel]
    __shared__ float sa[64], sb[64], sc[64];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int Cg = C / G;
    if (tid < 64 && c0 + tid < C) {
        const int c = c0 + tid, g = c / Cg;
        const float2 k = coef[(size_t)bf * G + g];
        sa[tid] = rstd[(size_t)bf * G + g] * (gamma ? gamma[c] : 1.f);
        sb[tid] = k.x;
        sc[tid] = k.y;
    }
    load_tok_tile(tile, dtok, F, C, HW, bf, hw0, c0);
    float xv[16], rv[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {  // x and the residual's gradient along hw, all in flight before the barrier
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;  // channel r, pixel h
        const bool ok = hw0 + h < HW && c0 + r < C;
        const size_t o = ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + h : 0;
        xv[k] = to_f(x[o]);
        rv[k] = dres ? to_f(dres[o]) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int i = tid + 256 * k, r = i >> 6, h = i & 63;
        if (hw0 + h < HW && c0 + r < C) {
            const float v = fmaf(sa[r], tile[h][r], fmaf(sb[r], xv[k], sc[r])) + rv[k];
            dx[((size_t)bf * C + c0 + r) * HW + hw0 + h] = from_f<TI>(v);
        }
    }
}

// ---- vector-access forms of the three backward layout kernels (C % 8 == 0, HW % 4 == 0, 16-B aligned tensors):
// channel rows read / written 4 pixels per lane, token rows 8 channels per lane, every load in flight before the
// first wait; the same arithmetic and summation order as the scalar forms (bitwise equal). Bench level (C = 512,
// 32 x 32, 32 samples): k_mva_out_bwd 36.0 -> 31.8 us, k_mva_gn_part 25.3 -> 23.3 us, k_mva_gn_dx 40.8 -> 40.2 us
// (profiles/r05/ab_mva_vecb).
template <class T>
__device__ __forceinline__ void store8(T *p, const float (&v)[8]) {
    if constexpr (sizeof(T) == 4) {
        reinterpret_cast<float4 *>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4 *>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
    } else {
        T e[8];
#pragma unroll
        for (int j = 0; j < 8; j++) e[j] = from_f<T>(v[j]);
        *reinterpret_cast<uint4 *>(p) = *reinterpret_cast<const uint4 *>(e);
    }
}
template <class TD, class TY, class TR>
__global__ __launch_bounds__(256) void k_mva_out_bwd_v(int F, int C, int HW, const TD *__restrict__ dout, float scale,
                                                       TY *__restrict__ dy, TR *__restrict__ dres) {
    __shared__ float tile[64][65];  // [channel][pixel]
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    float v[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // channel row r, pixels 4 p .. 4 p + 3
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        const bool ok = c0 + r < C && hw0 + 4 * p < HW;
        load4<TD>(dout + (ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p : 0), v[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        float g[4];
#pragma unroll
        for (int e = 0; e < 4; e++) {
            g[e] = to_f(from_f<TD>(v[k][e] * scale));  // (exact: scale 1 and an fp32 gradient)
            tile[r][4 * p + e] = g[e];
        }
        if (dres && c0 + r < C && hw0 + 4 * p < HW) store4<TR>(dres + ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p, g);
    }
    __syncthreads();
    const int b = bf / F, f = bf - b * F;
    TY *yb = dy + ((size_t)b * F * HW + (size_t)f * HW) * C;
#pragma unroll
    for (int k = 0; k < 2; k++) {  // token row r, channels 8 q .. 8 q + 7
        const int i = tid + 256 * k, r = i >> 3, q = i & 7;
        if (hw0 + r < HW && c0 + 8 * q < C) {
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = tile[8 * q + j][r];
            store8<TY>(yb + (size_t)(hw0 + r) * C + c0 + 8 * q, o);
        }
    }
}
// the token gradient tile into LDS as [pixel][channel], zero outside (the loads only issued here; the caller's
// other loads can go out before the stores to LDS)
template <class TT>
struct TokTileV {
    float v[2][8];
    __device__ __forceinline__ void load(const TT *__restrict__ tok, int F, int C, int HW, int bf, int hw0, int c0) {
        const int b = bf / F, f = bf - b * F, tid = threadIdx.x;
        const TT *tb = tok + ((size_t)b * F * HW + (size_t)f * HW) * C;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int i = tid + 256 * k, r = i >> 3, q = i & 7;
            const bool ok = hw0 + r < HW && c0 + 8 * q < C;
            load8<TT>(tb + (ok ? (size_t)(hw0 + r) * C + c0 + 8 * q : 0), v[k]);
        }
    }
    __device__ __forceinline__ void store(float (&tile)[64][65], int C, int HW, int hw0, int c0) const {
        const int tid = threadIdx.x;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int i = tid + 256 * k, r = i >> 3, q = i & 7;
            const bool ok = hw0 + r < HW && c0 + 8 * q < C;  // (masked here, not at the load: no wait per load)
#pragma unroll
            for (int j = 0; j < 8; j++) tile[r][8 * q + j] = ok ? v[k][j] : 0.f;
        }
    }
};
template <class TI, class TT>
__global__ __launch_bounds__(256) void k_mva_gn_part_v(int F, int C, int HW, const TI *__restrict__ x,
                                                       const TT *__restrict__ dtok, float2 *__restrict__ part) {
    __shared__ float tile[64][65];  // dy [pixel][channel]
    __shared__ float xs[64][65];    // x [channel][pixel]
    __shared__ float2 red[4][64];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int nT = gridDim.x;
    {
        float xv[4][4];
#pragma unroll
        for (int k = 0; k < 4; k++) {  // x along hw (zero outside)
            const int i = tid + 256 * k, r = i >> 4, p = i & 15;
            const bool ok = c0 + r < C && hw0 + 4 * p < HW;
            load4<TI>(x + (ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p : 0), xv[k]);
        }
        TokTileV<TT> tt;
        tt.load(dtok, F, C, HW, bf, hw0, c0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int i = tid + 256 * k, r = i >> 4, p = i & 15;
            const bool ok = c0 + r < C && hw0 + 4 * p < HW;
#pragma unroll
            for (int e = 0; e < 4; e++) xs[r][4 * p + e] = ok ? xv[k][e] : 0.f;
        }
        tt.store(tile, C, HW, hw0, c0);
    }
    __syncthreads();
    const int c = tid & 63, q = tid >> 6;  // as k_mva_gn_part
    float sdx = 0.f, sd = 0.f;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int h = 16 * q + k;
        const float g = tile[h][c];
        sd += g;
        sdx = fmaf(g, xs[c][h], sdx);
    }
    red[q][c] = make_float2(sdx, sd);
    __syncthreads();
    if (tid < 64 && c0 + tid < C) {
        const float2 a = red[0][tid], b2 = red[1][tid], c2 = red[2][tid], d2 = red[3][tid];
        part[((size_t)bf * C + c0 + tid) * nT + blockIdx.x] =
            make_float2((a.x + b2.x) + (c2.x + d2.x), (a.y + b2.y) + (c2.y + d2.y));
    }
}
template <class TI, class TT, class TR>
__global__ __launch_bounds__(256) void k_mva_gn_dx_v(int F, int C, int HW, int G, const TI *__restrict__ x,
                                                     const TT *__restrict__ dtok, const TR *__restrict__ dres,
                                                     const float *__restrict__ gamma, const float *__restrict__ rstd,
                                                     const float2 *__restrict__ coef, TI *__restrict__ dx) {
    __shared__ float tile[64][65];  // [pixel][channel]
    __shared__ float sa[64], sb[64], sc[64];
    const int hw0 = blockIdx.x * 64, c0 = blockIdx.y * 64, bf = blockIdx.z, tid = threadIdx.x;
    const int Cg = C / G;
    TokTileV<TT> tt;
    tt.load(dtok, F, C, HW, bf, hw0, c0);
    float xv[4][4], rv[4][4];
#pragma unroll
    for (int k = 0; k < 4; k++) {  // x and the residual's gradient along hw
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        const bool ok = c0 + r < C && hw0 + 4 * p < HW;
        const size_t o = ok ? ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p : 0;
        load4<TI>(x + o, xv[k]);
        if (dres) load4<TR>(dres + o, rv[k]);
        else
#pragma unroll
            for (int e = 0; e < 4; e++) rv[k][e] = 0.f;
    }
    if (tid < 64 && c0 + tid < C) {
        const int c = c0 + tid, g = c / Cg;
        const float2 kk = coef[(size_t)bf * G + g];
        sa[tid] = rstd[(size_t)bf * G + g] * (gamma ? gamma[c] : 1.f);
        sb[tid] = kk.x;
        sc[tid] = kk.y;
    }
    tt.store(tile, C, HW, hw0, c0);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int i = tid + 256 * k, r = i >> 4, p = i & 15;
        if (c0 + r < C && hw0 + 4 * p < HW) {
            float o[4];
#pragma unroll
            for (int e = 0; e < 4; e++)
                o[e] = fmaf(sa[r], tile[4 * p + e][r], fmaf(sb[r], xv[k][e], sc[r])) + rv[k][e];
            store4<TI>(dx + ((size_t)bf * C + c0 + r) * HW + hw0 + 4 * p, o);
        }
    }
}
__host__ __forceinline__ bool mva_vec_ok(int C, int HW, std::initializer_list<const void *> ps) {
    if (C % 8 || HW % 4) return false;
    for (const void *p : ps)
        if (reinterpret_cast<uintptr_t>(p) & 15) return false;
    return true;
}

template <class TI, class TO>
int launch_norm(int B, int F, int C, int HW, int G, float eps, const void *x, const float *gamma, const float *beta,
                void *tok, float *mean, float *rstd, float2 *part, hipStream_t st) {
    const int Cg = C / G;
    if (Cg % 8 == 0 && Cg <= 256 && HW % 4 == 0 &&
        (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (long long)(Cg / 8) * (HW / 4) <= (long long)GNR_K * GN_THREADS) {
        LGM_LAUNCH("k_mva_gn_reg", st, (k_mva_gn_reg<TI, TO><<<dim3(G, B * F), GN_THREADS, 0, st>>>(
                                           F, C, HW, G, eps, (const TI *)x, gamma, beta, (TO *)tok, mean, rstd)));
        return LGM_OK;
    }
    const size_t lds = ((size_t)(C / G) * HW + 2 * (C / G)) * sizeof(float);
    if (lds <= GN_LDS_MAX) {  // one launch: the group's slab in LDS
        // the kernel's dynamic LDS limit is raised on every launch of this path: the attribute belongs to the current
        // device, and a process-wide "already set" flag would skip it on a second device (and race between threads);
        // the call is a host-side table update, no device work (include/lgm_attn.h, threading note)
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(&k_mva_gn_tok<TI, TO>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)GN_LDS_MAX) != hipSuccess) {
            set_error("hipFuncSetAttribute(k_mva_gn_tok) failed");
            return LGM_E_HIP;
        }
        LGM_LAUNCH("k_mva_gn_tok", st, (k_mva_gn_tok<TI, TO><<<dim3(G, B * F), GN_THREADS, lds, st>>>(
                                           F, C, HW, G, eps, (const TI *)x, gamma, beta, (TO *)tok, mean, rstd)));
        return LGM_OK;
    }
    const int S = (C / G * HW + MVA_CHUNK - 1) / MVA_CHUNK;  // larger slabs: chunked statistics + tiled normalise
    LGM_LAUNCH("k_mva_stats", st,
               (k_mva_stats<TI><<<dim3(S, G, B * F), 256, 0, st>>>(C, HW, G, (const TI *)x, part)));
    const dim3 grid((HW + 63) / 64, (C + 63) / 64, B * F);
    LGM_LAUNCH("k_mva_norm", st, (k_mva_norm<TI, TO><<<grid, 256, 0, st>>>(F, C, HW, G, eps, (const TI *)x, gamma,
                                                                            beta, part, (TO *)tok, mean, rstd)));
    return LGM_OK;
}

template <class TY, class TR, class TO>
int launch_out(int B, int F, int C, int HW, const void *y, const void *res, float skip, void *out, hipStream_t st) {
    const dim3 grid((HW + 63) / 64, (C + 63) / 64, B * F);
    const bool vec = C % 8 == 0 && HW % 4 == 0 && ((reinterpret_cast<uintptr_t>(y) |
                     reinterpret_cast<uintptr_t>(res) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    if (vec) {
        LGM_LAUNCH("k_mva_out", st, (k_mva_out_v<TY, TR, TO><<<grid, 256, 0, st>>>(F, C, HW, (const TY *)y,
                                                                                  (const TR *)res, skip, (TO *)out)));
        return LGM_OK;
    }
    LGM_LAUNCH("k_mva_out", st,
               (k_mva_out<TY, TR, TO><<<grid, 256, 0, st>>>(F, C, HW, (const TY *)y, (const TR *)res, skip, (TO *)out)));
    return LGM_OK;
}

template <class TI>
int norm_by_out(int dto, int B, int F, int C, int HW, int G, float eps, const void *x, const float *gamma,
                const float *beta, void *tok, float *mean, float *rstd, float2 *part, hipStream_t st) {
    switch (dto) {
        case LGM_ATTN_F32: return launch_norm<TI, float>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, part, st);
        case LGM_ATTN_BF16: return launch_norm<TI, __hip_bfloat16>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, part, st);
        case LGM_ATTN_F16: return launch_norm<TI, __half>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, part, st);
    }
    set_error("lgm_mva_norm_tokens: bad output dtype %d", dto);
    return LGM_E_INVALID;
}

template <class TY, class TR>
int out_by_o(int dto, int B, int F, int C, int HW, const void *y, const void *res, float skip, void *out,
             hipStream_t st) {
    switch (dto) {
        case LGM_ATTN_F32: return launch_out<TY, TR, float>(B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_BF16: return launch_out<TY, TR, __hip_bfloat16>(B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_F16: return launch_out<TY, TR, __half>(B, F, C, HW, y, res, skip, out, st);
    }
    set_error("lgm_mva_tokens_out: bad output dtype %d", dto);
    return LGM_E_INVALID;
}

template <class TY>
int out_by_r(int dtr, int dto, int B, int F, int C, int HW, const void *y, const void *res, float skip, void *out,
             hipStream_t st) {
    switch (dtr) {
        case LGM_ATTN_F32: return out_by_o<TY, float>(dto, B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_BF16: return out_by_o<TY, __hip_bfloat16>(dto, B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_F16: return out_by_o<TY, __half>(dto, B, F, C, HW, y, res, skip, out, st);
    }
    set_error("lgm_mva_tokens_out: bad residual dtype %d", dtr);
    return LGM_E_INVALID;
}

// backward launchers: the dtype switches (LGM_ATTN_F32 / BF16 / F16 codes -> types)
template <class Fn>
int with_type(int code, Fn &&fn) {
    switch (code) {
        case LGM_ATTN_F32: return fn(float{});
        case LGM_ATTN_BF16: return fn(__hip_bfloat16{});
        case LGM_ATTN_F16: return fn(__half{});
    }
    set_error("lgm_mva backward: bad dtype %d", code);
    return LGM_E_INVALID;
}

size_t gn_part_bytes(int BF, int C, int HW) { return (((size_t)BF * C * ((HW + 63) / 64) * sizeof(float2)) + 255) & ~(size_t)255; }

}  // namespace
}  // namespace lgm

extern "C" size_t lgm_mva_backward_workspace_size(int B, int F, int C, int HW, int groups) {
    if (B <= 0 || F <= 0 || C <= 0 || HW <= 0 || groups <= 0 || C % groups) return 0;
    return lgm::gn_part_bytes(B * F, C, HW) + (size_t)B * F * groups * sizeof(float2);
}

extern "C" int lgm_mva_tokens_out_backward(int dtype_dout, int dtype_dy, int dtype_dres, int B, int F, int C, int HW,
                                           const void *d_out, float scale, void *d_y, void *d_res, void *stream,
                                           const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    if (B < 0 || F <= 0 || C <= 0 || HW < 0) {
        lgm::set_error("lgm_mva_tokens_out_backward: bad shape B=%d F=%d C=%d HW=%d", B, F, C, HW);
        return LGM_E_INVALID;
    }
    if (B == 0 || HW == 0) return LGM_OK;
    if (!d_out || !d_y) {
        lgm::set_error("lgm_mva_tokens_out_backward: null pointer");
        return LGM_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    const dim3 grid((HW + 63) / 64, (C + 63) / 64, B * F);
    return lgm::with_type(dtype_dout, [&](auto td) {
        using TD = decltype(td);
        return lgm::with_type(dtype_dy, [&](auto ty) {
            using TY = decltype(ty);
            return lgm::with_type(d_res ? dtype_dres : LGM_ATTN_F32, [&](auto tr) {
                using TR = decltype(tr);
                if (lgm::mva_vec_ok(C, HW, {d_out, d_y, d_res})) {
                    LGM_LAUNCH("k_mva_out_bwd", st, (lgm::k_mva_out_bwd_v<TD, TY, TR><<<grid, 256, 0, st>>>(
                                                         F, C, HW, (const TD *)d_out, scale, (TY *)d_y, (TR *)d_res)));
                    return LGM_OK;
                }
                LGM_LAUNCH("k_mva_out_bwd", st, (lgm::k_mva_out_bwd<TD, TY, TR><<<grid, 256, 0, st>>>(
                                                     F, C, HW, (const TD *)d_out, scale, (TY *)d_y, (TR *)d_res)));
                return LGM_OK;
            });
        });
    });
}

extern "C" int lgm_mva_norm_tokens_backward(int dtype_x, int dtype_tok, int B, int F, int C, int HW, int groups,
                                            const void *x, const float *gamma, const float *mean, const float *rstd,
                                            const void *d_tokens, const void *d_res, void *dx, float *dgamma,
                                            float *dbeta, void *workspace, size_t workspace_bytes, void *stream,
                                            const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    if (B < 0 || F <= 0 || C <= 0 || HW < 0 || groups <= 0 || C % groups || C / groups > lgm::GN_NMAX) {
        lgm::set_error("lgm_mva_norm_tokens_backward: bad shape B=%d F=%d C=%d HW=%d groups=%d (channels per group "
                       "<= %d)", B, F, C, HW, groups, lgm::GN_NMAX);
        return LGM_E_INVALID;
    }
    if (B == 0 || HW == 0) return LGM_OK;
    if (!x || !mean || !rstd || !d_tokens || !workspace) {
        lgm::set_error("lgm_mva_norm_tokens_backward: null pointer");
        return LGM_E_INVALID;
    }
    if (workspace_bytes < lgm_mva_backward_workspace_size(B, F, C, HW, groups)) {
        lgm::set_error("lgm_mva_norm_tokens_backward: workspace too small");
        return LGM_E_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    const int BF = B * F, nT = (HW + 63) / 64;
    float2 *part = (float2 *)workspace;
    float2 *coef = (float2 *)((char *)workspace + lgm::gn_part_bytes(BF, C, HW));
    const dim3 grid(nT, (C + 63) / 64, BF);
    return lgm::with_type(dtype_x, [&](auto tx) {
        using TI = decltype(tx);
        return lgm::with_type(dtype_tok, [&](auto tt) {
            using TT = decltype(tt);
            const bool vec = lgm::mva_vec_ok(C, HW, {x, d_tokens, d_res, dx});
            if (vec)
                LGM_LAUNCH("k_mva_gn_part", st, (lgm::k_mva_gn_part_v<TI, TT><<<grid, 256, 0, st>>>(
                                                     F, C, HW, (const TI *)x, (const TT *)d_tokens, part)));
            else
                LGM_LAUNCH("k_mva_gn_part", st, (lgm::k_mva_gn_part<TI, TT><<<grid, 256, 0, st>>>(
                                                     F, C, HW, (const TI *)x, (const TT *)d_tokens, part)));
            LGM_LAUNCH("k_mva_gn_coef", st, (lgm::k_mva_gn_coef<<<groups, 256, 0, st>>>(
                                                 BF, C, HW, groups, nT, part, gamma, mean, rstd, coef, dgamma, dbeta)));
            if (dx && vec)
                LGM_LAUNCH("k_mva_gn_dx", st, (lgm::k_mva_gn_dx_v<TI, TT, TI><<<grid, 256, 0, st>>>(
                                                   F, C, HW, groups, (const TI *)x, (const TT *)d_tokens,
                                                   (const TI *)d_res, gamma, rstd, coef, (TI *)dx)));
            else if (dx)
                LGM_LAUNCH("k_mva_gn_dx", st, (lgm::k_mva_gn_dx<TI, TT, TI><<<grid, 256, 0, st>>>(
                                                   F, C, HW, groups, (const TI *)x, (const TT *)d_tokens,
                                                   (const TI *)d_res, gamma, rstd, coef, (TI *)dx)));
            return LGM_OK;
        });
    });
}

extern "C" size_t lgm_mva_workspace_size(int B, int F, int C, int HW, int groups) {
    if (B <= 0 || F <= 0 || C <= 0 || HW <= 0 || groups <= 0 || C % groups) return 0;
    const size_t S = ((size_t)(C / groups) * HW + lgm::MVA_CHUNK - 1) / lgm::MVA_CHUNK;
    return (size_t)B * F * groups * S * sizeof(float2);
}

extern "C" int lgm_mva_norm_tokens(int dtype_x, int dtype_tok, int B, int F, int C, int HW, int groups, float eps,
                                   const void *x, const float *gamma, const float *beta, void *tokens, float *mean,
                                   float *rstd, void *workspace, size_t workspace_bytes, void *stream,
                                   const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    if (B < 0 || F <= 0 || C <= 0 || HW < 0 || groups <= 0 || C % groups) {
        lgm::set_error("lgm_mva_norm_tokens: bad shape B=%d F=%d C=%d HW=%d groups=%d", B, F, C, HW, groups);
        return LGM_E_INVALID;
    }
    if (B == 0 || HW == 0) return LGM_OK;
    if (!x || !tokens || !mean || !rstd || !workspace) {
        lgm::set_error("lgm_mva_norm_tokens: null pointer");
        return LGM_E_INVALID;
    }
    if (workspace_bytes < lgm_mva_workspace_size(B, F, C, HW, groups)) {
        lgm::set_error("lgm_mva_norm_tokens: workspace too small");
        return LGM_E_WORKSPACE;
    }
    float2 *part = (float2 *)workspace;
    hipStream_t st = (hipStream_t)stream;
    switch (dtype_x) {
        case LGM_ATTN_F32:
            return lgm::norm_by_out<float>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean, rstd, part, st);
        case LGM_ATTN_BF16:
            return lgm::norm_by_out<__hip_bfloat16>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean,
                                                    rstd, part, st);
        case LGM_ATTN_F16:
            return lgm::norm_by_out<__half>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean, rstd, part, st);
    }
    lgm::set_error("lgm_mva_norm_tokens: bad input dtype %d", dtype_x);
    return LGM_E_INVALID;
}

extern "C" int lgm_mva_tokens_out(int dtype_y, int dtype_res, int dtype_out, int B, int F, int C, int HW,
                                  const void *y, const void *res, float skip, void *out, void *stream,
                                  const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    if (B < 0 || F <= 0 || C <= 0 || HW < 0) {
        lgm::set_error("lgm_mva_tokens_out: bad shape B=%d F=%d C=%d HW=%d", B, F, C, HW);
        return LGM_E_INVALID;
    }
    if (B == 0 || HW == 0) return LGM_OK;
    if (!y || !out) {
        lgm::set_error("lgm_mva_tokens_out: null pointer");
        return LGM_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    const int dr = res ? dtype_res : LGM_ATTN_F32;  // (no residual: the type is not used)
    switch (dtype_y) {
        case LGM_ATTN_F32: return lgm::out_by_r<float>(dr, dtype_out, B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_BF16: return lgm::out_by_r<__hip_bfloat16>(dr, dtype_out, B, F, C, HW, y, res, skip, out, st);
        case LGM_ATTN_F16: return lgm::out_by_r<__half>(dr, dtype_out, B, F, C, HW, y, res, skip, out, st);
    }
    lgm::set_error("lgm_mva_tokens_out: bad y dtype %d", dtype_y);
    return LGM_E_INVALID;
}
