// lgm_amd/csrc/attention.hip -- MFMA flash attention (forward + backward) for LGM's multi-view self-attention.
//
// Replaces xformers.ops.memory_efficient_attention as called by core/attention.py:74-84 (MemEffAttention, used by
// core/unet.py:35-49 MVAttention), and its pure-torch fallback core/attention.py:51-64:
//     out = softmax(scale * q k^T) v,  q, k, v in xformers layout [B, L, H, D], scale = D^-1/2, no bias, p = 0.
// q/k/v are read in place from the packed qkv Linear output [B, L, 3, H, D] (row stride ld = 3 H D elements), so
// the reshape/unbind of core/attention.py:75-77 costs nothing; dq/dk/dv are written back packed the same way.
//
// Design (CDNA4, wave64, 16x16 MFMA tiles; fp32 accumulation):
//   * scores are computed TRANSPOSED, S^T = K Q^T, so every lane owns one query column (q = lane & 15) and holds
//     4 keys of each 16-key sub-tile: the online-softmax row state (m, l) and the O^T accumulator live in the
//     same lane, and the P tile feeds the P V product from registers (its key order permuted to match the
//     accumulator layout; the matching V^T operand is read with the same permutation from LDS);
//   * bf16 / fp16 use v_mfma_f32_16x16x32_{bf16,f16}; fp32 uses the exact-f32 v_mfma_f32_16x16x4_f32, so fp32
//     inputs keep the fp32 accuracy of the reference's fallback;
//   * the softmax runs in base 2 (exp2 with a log2(e) prescale); LSE is stored in natural log for the backward;
//   * backward = delta = rowsum(dO * O), then a dQ kernel (per query block, loops over key blocks) and a dK/dV
//     kernel (per key block, loops over query blocks): no atomics, deterministic.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "common.h"
#include "lgm_attn.h"

namespace lgm {
namespace attn {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr int BQ = 64, BK = 64, NT = 256;  // 4 wavefronts x 16 rows

template <int DT> struct Ty;
template <> struct Ty<LGM_ATTN_F32> { using T = float; static constexpr int PAD = 2; };
template <> struct Ty<LGM_ATTN_BF16> { using T = __bf16; using V8 = bf16x8; static constexpr int PAD = 8; };
template <> struct Ty<LGM_ATTN_F16> { using T = _Float16; using V8 = f16x8; static constexpr int PAD = 8; };
constexpr int PADT = 4;  // transposed bf16/fp16 tiles: [D][64 + 4]

template <typename T> __device__ __forceinline__ float to_f(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x) { return (T)x; }

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

template <int DT> __device__ __forceinline__ f32x4 mfma32(typename Ty<DT>::V8 a, typename Ty<DT>::V8 b, f32x4 c) {
    if constexpr (DT == LGM_ATTN_BF16) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// Register fragment of a 16-row operand Y[row = lane & 15][0..D): fp32 -> D/4 values Y[r][4s + g];
// 16-bit -> D/32 vectors Y[r][32c + 8g + 0..7].
template <int DT, int D> struct YFrag;
template <int D> struct YFrag<LGM_ATTN_F32, D> { float v[D / 4]; };
template <int D> struct YFrag<LGM_ATTN_BF16, D> { bf16x8 v[D / 32]; };
template <int D> struct YFrag<LGM_ATTN_F16, D> { f16x8 v[D / 32]; };

template <int DT, int D>
__device__ __forceinline__ void load_yfrag(YFrag<DT, D> &f, const typename Ty<DT>::T *row, bool valid, int g) {
    using T = typename Ty<DT>::T;
    if constexpr (DT == LGM_ATTN_F32) {
#pragma unroll
        for (int s = 0; s < D / 4; s++) f.v[s] = valid ? row[4 * s + g] : 0.f;
    } else {
        using V8 = typename Ty<DT>::V8;
#pragma unroll
        for (int c = 0; c < D / 32; c++) {
            if (valid) f.v[c] = *reinterpret_cast<const V8 *>(row + 32 * c + 8 * g);
            else
#pragma unroll
                for (int j = 0; j < 8; j++) f.v[c][j] = (T)0.f;
        }
    }
}

// acc[i] += (X Y^T)[rb + 4g + i][lane & 15]: X rows from an LDS row-major tile (stride ldx), Y = register frag.
template <int DT, int D>
__device__ __forceinline__ void s_like(f32x4 &acc, const typename Ty<DT>::T *X, int ldx, int rb,
                                       const YFrag<DT, D> &y, int g, int r16) {
    const typename Ty<DT>::T *xr = X + (rb + r16) * ldx;
    if constexpr (DT == LGM_ATTN_F32) {
#pragma unroll
        for (int s = 0; s < D / 4; s++) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[4 * s + g], y.v[s], acc, 0, 0, 0);
    } else {
        using V8 = typename Ty<DT>::V8;
#pragma unroll
        for (int c = 0; c < D / 32; c++)
            acc = mfma32<DT>(*reinterpret_cast<const V8 *>(xr + 32 * c + 8 * g), y.v[c], acc);
    }
}

// acc[dt][i] += (Z^T P)[d = 16 dt + 4g + i][col = lane & 15] over the 64 keys of a block, where P is held by the
// lanes as own[sub][i] = P[key = 16 sub + 4g + i][col]. fp32: Z is the row-major LDS tile [key][d] (stride ldz);
// 16-bit: Zt is the TRANSPOSED LDS tile [d][key] (stride ldzt), read with the key permutation of the operand.
template <int DT, int D>
__device__ __forceinline__ void pv_like(f32x4 (&acc)[D / 16], const typename Ty<DT>::T *Z, int ldz,
                                        const float (&own)[4][4], int g, int r16) {
    if constexpr (DT == LGM_ATTN_F32) {
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
            for (int sub = 0; sub < 4; sub++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    acc[dt] = __builtin_amdgcn_mfma_f32_16x16x4f32(Z[(16 * sub + 4 * g + i) * ldz + 16 * dt + r16],
                                                                    own[sub][i], acc[dt], 0, 0, 0);
    } else {
        using T = typename Ty<DT>::T;
        using V8 = typename Ty<DT>::V8;
#pragma unroll
        for (int t = 0; t < 2; t++) {
            V8 b;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                b[i] = (T)own[2 * t][i];
                b[4 + i] = (T)own[2 * t + 1][i];
            }
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++) {
                const T *zr = Z + (16 * dt + r16) * ldz + 32 * t + 4 * g;
                const uint2 lo = *reinterpret_cast<const uint2 *>(zr);
                const uint2 hi = *reinterpret_cast<const uint2 *>(zr + 16);
                V8 a;
                const uint4 packed = make_uint4(lo.x, lo.y, hi.x, hi.y);
                a = *reinterpret_cast<const V8 *>(&packed);
                acc[dt] = mfma32<DT>(a, b, acc[dt]);
            }
        }
    }
}

// Cooperative loads of a 64-row block (rows r0.., tokens >= L zero-filled) from a [tokens][ld] tensor.
template <typename T, int D, int PAD>
__device__ __forceinline__ void load_rows(T *dst, const T *src, long long ld, int r0, int L) {
    constexpr int VEC = 16 / sizeof(T), CPR = D / VEC;
    for (int c = threadIdx.x; c < 64 * CPR; c += NT) {
        const int r = c / CPR, col = (c - r * CPR) * VEC;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (r0 + r < L) v = *reinterpret_cast<const uint4 *>(src + (long long)(r0 + r) * ld + col);
        if constexpr (PAD % VEC == 0) {
            *reinterpret_cast<uint4 *>(dst + r * (D + PAD) + col) = v;
        } else {
            const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
            for (int j = 0; j < VEC; j++) dst[r * (D + PAD) + col + j] = pv[j];
        }
    }
}
template <typename T, int D>
__device__ __forceinline__ void load_rows_T(T *dst, const T *src, long long ld, int r0, int L) {
    constexpr int VEC = 16 / sizeof(T), CPR = D / VEC;
    for (int c = threadIdx.x; c < 64 * CPR; c += NT) {
        const int r = c / CPR, col = (c - r * CPR) * VEC;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (r0 + r < L) v = *reinterpret_cast<const uint4 *>(src + (long long)(r0 + r) * ld + col);
        const T *pv = reinterpret_cast<const T *>(&v);
#pragma unroll
        for (int j = 0; j < VEC; j++) dst[(col + j) * (64 + PADT) + r] = pv[j];
    }
}

__device__ __forceinline__ float xmax4(float v) {
    v = fmaxf(v, __shfl_xor(v, 16, 64));
    return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float xsum4(float v) {
    v += __shfl_xor(v, 16, 64);
    return v + __shfl_xor(v, 32, 64);
}

// ------------------------------------------------------------------------------------------------------------
// forward: grid (ceil(L/64), B*H), block 256.
template <int DT, int D>
__global__ __launch_bounds__(NT) void k_attn_fwd(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ q,
                                                 const typename Ty<DT>::T *__restrict__ k,
                                                 const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                 typename Ty<DT>::T *__restrict__ o, float *__restrict__ lse) {
    using T = typename Ty<DT>::T;
    constexpr int PAD = Ty<DT>::PAD;
    constexpr bool F32 = DT == LGM_ATTN_F32;
    __shared__ __attribute__((aligned(16))) T Ks[64 * (D + PAD)];
    __shared__ __attribute__((aligned(16))) T Vs[F32 ? 64 * (D + PAD) : D * (64 + PADT)];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int qrow = blockIdx.x * BQ + w * 16 + r16;
    const bool qvalid = qrow < L;
    const float c = scale * LOG2E;
    YFrag<DT, D> qf;
    load_yfrag<DT, D>(qf, q + base + (long long)qrow * ld, qvalid, g);
    f32x4 oacc[D / 16];
#pragma unroll
    for (int dt = 0; dt < D / 16; dt++) oacc[dt] = zero4();
    float m = -INFINITY, lsum = 0.f;
    for (int kb = 0; kb < L; kb += BK) {
        __syncthreads();
        load_rows<T, D, PAD>(Ks, k + base, ld, kb, L);
        if constexpr (F32) load_rows<T, D, PAD>(Vs, v + base, ld, kb, L);
        else load_rows_T<T, D>(Vs, v + base, ld, kb, L);
        __syncthreads();
        float p[4][4];
        float mloc = -INFINITY;
#pragma unroll
        for (int sub = 0; sub < 4; sub++) {
            f32x4 s = zero4();
            s_like<DT, D>(s, Ks, D + PAD, 16 * sub, qf, g, r16);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float x = (kb + 16 * sub + 4 * g + i < L) ? s[i] * c : -INFINITY;
                p[sub][i] = x;
                mloc = fmaxf(mloc, x);
            }
        }
        mloc = xmax4(mloc);
        const float mnew = fmaxf(m, mloc);
        const float alpha = (mnew == -INFINITY) ? 1.f : exp2f(m - mnew);
        float ls = 0.f;
#pragma unroll
        for (int sub = 0; sub < 4; sub++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float e = (mnew == -INFINITY) ? 0.f : exp2f(p[sub][i] - mnew);
                p[sub][i] = e;
                ls += e;
            }
        lsum = lsum * alpha + xsum4(ls);
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++) oacc[dt] *= alpha;
        pv_like<DT, D>(oacc, Vs, F32 ? D + PAD : 64 + PADT, p, g, r16);
        m = mnew;
    }
    if (qvalid) {
        const float inv = 1.f / lsum;
        T *orow = o + ((long long)b * L + qrow) * ((long long)H * D) + (long long)h * D;
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
            for (int i = 0; i < 4; i++) orow[16 * dt + 4 * g + i] = from_f<T>(oacc[dt][i] * inv);
        if (g == 0) lse[(long long)bh * L + qrow] = (m + log2f(lsum)) * LN2;
    }
}

// delta[bh][q] = sum_d dO[q][d] * O[q][d]  (fp32); grid ceil(B*L*H / 256).
template <int DT, int D>
__global__ __launch_bounds__(256) void k_attn_delta(int B, int L, int H, const typename Ty<DT>::T *__restrict__ o,
                                                    const typename Ty<DT>::T *__restrict__ dout,
                                                    float *__restrict__ delta) {
    // thread -> (b, h, q), q fastest: the delta row is written coalesced (with h fastest every wave scattered its 64
    // floats over 16 rows of L: 25 -> ? us at 8 x 16 x 4096 rows); each thread still reads its own contiguous D-vector
    const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
    if (idx >= (long long)B * L * H) return;
    const long long bh = idx / L;
    const int qrow = (int)(idx - bh * L);
    const int b = (int)(bh / H), h = (int)(bh - (long long)b * H);
    const long long off = (((long long)b * L + qrow) * H + h) * D;
    float s = 0.f;
#pragma unroll 8
    for (int d = 0; d < D; d++) s += to_f(o[off + d]) * to_f(dout[off + d]);
    delta[idx] = s;
}

// dQ: grid (ceil(L/64), B*H). dQ = scale * sum_k dS K with dS = P o (dP - delta), P = exp(scale S - lse).
template <int DT, int D>
__global__ __launch_bounds__(NT) void k_attn_dq(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ q,
                                                const typename Ty<DT>::T *__restrict__ k,
                                                const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                const typename Ty<DT>::T *__restrict__ dout,
                                                const float *__restrict__ lse, const float *__restrict__ delta,
                                                typename Ty<DT>::T *__restrict__ dq, long long ldd) {
    using T = typename Ty<DT>::T;
    constexpr int PAD = Ty<DT>::PAD;
    constexpr bool F32 = DT == LGM_ATTN_F32;
    __shared__ __attribute__((aligned(16))) T Ks[64 * (D + PAD)];
    __shared__ __attribute__((aligned(16))) T Vs[64 * (D + PAD)];
    __shared__ __attribute__((aligned(16))) T Kt[F32 ? 1 : D * (64 + PADT)];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const long long obase = (long long)b * L * H * D + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int qrow = blockIdx.x * BQ + w * 16 + r16;
    const bool qvalid = qrow < L;
    const float c = scale * LOG2E;
    YFrag<DT, D> qf, dof;
    load_yfrag<DT, D>(qf, q + base + (long long)qrow * ld, qvalid, g);
    load_yfrag<DT, D>(dof, dout + obase + (long long)qrow * H * D, qvalid, g);
    const float lse2 = qvalid ? lse[(long long)bh * L + qrow] * LOG2E : 0.f;
    const float dlt = qvalid ? delta[(long long)bh * L + qrow] : 0.f;
    f32x4 acc[D / 16];
#pragma unroll
    for (int dt = 0; dt < D / 16; dt++) acc[dt] = zero4();
    for (int kb = 0; kb < L; kb += BK) {
        __syncthreads();
        load_rows<T, D, PAD>(Ks, k + base, ld, kb, L);
        load_rows<T, D, PAD>(Vs, v + base, ld, kb, L);
        if constexpr (!F32) load_rows_T<T, D>(Kt, k + base, ld, kb, L);
        __syncthreads();
        float ds[4][4];
#pragma unroll
        for (int sub = 0; sub < 4; sub++) {
            f32x4 s = zero4(), dp = zero4();
            s_like<DT, D>(s, Ks, D + PAD, 16 * sub, qf, g, r16);
            s_like<DT, D>(dp, Vs, D + PAD, 16 * sub, dof, g, r16);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const bool kv = kb + 16 * sub + 4 * g + i < L;
                const float p = (kv && qvalid) ? exp2f(s[i] * c - lse2) : 0.f;
                ds[sub][i] = p * (dp[i] - dlt);
            }
        }
        pv_like<DT, D>(acc, F32 ? Ks : Kt, F32 ? D + PAD : 64 + PADT, ds, g, r16);
    }
    if (qvalid) {
        T *row = dq + (long long)b * L * ldd + (long long)qrow * ldd + (long long)h * D;
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
            for (int i = 0; i < 4; i++) row[16 * dt + 4 * g + i] = from_f<T>(acc[dt][i] * scale);
    }
}

// dK, dV: grid (ceil(L/64), B*H); each wavefront owns 16 keys, loops over all query blocks.
template <int DT, int D>
__global__ __launch_bounds__(NT) void k_attn_dkdv(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ q,
                                                  const typename Ty<DT>::T *__restrict__ k,
                                                  const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                  const typename Ty<DT>::T *__restrict__ dout,
                                                  const float *__restrict__ lse, const float *__restrict__ delta,
                                                  typename Ty<DT>::T *__restrict__ dk, typename Ty<DT>::T *__restrict__ dv,
                                                  long long ldd) {
    using T = typename Ty<DT>::T;
    constexpr int PAD = Ty<DT>::PAD;
    constexpr bool F32 = DT == LGM_ATTN_F32;
    __shared__ __attribute__((aligned(16))) T Qs[64 * (D + PAD)];
    __shared__ __attribute__((aligned(16))) T Os[64 * (D + PAD)];  // dO rows
    __shared__ __attribute__((aligned(16))) T Qt[F32 ? 1 : D * (64 + PADT)];
    __shared__ __attribute__((aligned(16))) T Ot[F32 ? 1 : D * (64 + PADT)];
    __shared__ float sl[64], sd[64];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const long long obase = (long long)b * L * H * D + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int key = blockIdx.x * BK + w * 16 + r16;
    const bool kvalid = key < L;
    const float c = scale * LOG2E;
    YFrag<DT, D> kf, vf;
    load_yfrag<DT, D>(kf, k + base + (long long)key * ld, kvalid, g);
    load_yfrag<DT, D>(vf, v + base + (long long)key * ld, kvalid, g);
    f32x4 dka[D / 16], dva[D / 16];
#pragma unroll
    for (int dt = 0; dt < D / 16; dt++) { dka[dt] = zero4(); dva[dt] = zero4(); }
    for (int qb = 0; qb < L; qb += BQ) {
        __syncthreads();
        load_rows<T, D, PAD>(Qs, q + base, ld, qb, L);
        load_rows<T, D, PAD>(Os, dout + obase, (long long)H * D, qb, L);
        if constexpr (!F32) {
            load_rows_T<T, D>(Qt, q + base, ld, qb, L);
            load_rows_T<T, D>(Ot, dout + obase, (long long)H * D, qb, L);
        }
        if (tid < 64) {
            const bool qv = qb + tid < L;
            sl[tid] = qv ? lse[(long long)bh * L + qb + tid] * LOG2E : INFINITY;  // invalid rows: P = 0
            sd[tid] = qv ? delta[(long long)bh * L + qb + tid] : 0.f;
        }
        __syncthreads();
        float p[4][4], ds[4][4];
#pragma unroll
        for (int sub = 0; sub < 4; sub++) {
            f32x4 s = zero4(), dp = zero4();
            s_like<DT, D>(s, Qs, D + PAD, 16 * sub, kf, g, r16);   // S[q = 16 sub + 4g + i][key]
            s_like<DT, D>(dp, Os, D + PAD, 16 * sub, vf, g, r16);  // dP[q][key]
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int qi = 16 * sub + 4 * g + i;
                const float e = exp2f(s[i] * c - sl[qi]);
                p[sub][i] = e;
                ds[sub][i] = e * (dp[i] - sd[qi]);
            }
        }
        pv_like<DT, D>(dva, F32 ? Os : Ot, F32 ? D + PAD : 64 + PADT, p, g, r16);   // dV^T += dO^T P
        pv_like<DT, D>(dka, F32 ? Qs : Qt, F32 ? D + PAD : 64 + PADT, ds, g, r16);  // dK^T += Q^T dS
    }
    if (kvalid) {
        T *krow = dk + (long long)b * L * ldd + (long long)key * ldd + (long long)h * D;
        T *vrow = dv + (long long)b * L * ldd + (long long)key * ldd + (long long)h * D;
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                krow[16 * dt + 4 * g + i] = from_f<T>(dka[dt][i] * scale);
                vrow[16 * dt + 4 * g + i] = from_f<T>(dva[dt][i]);
            }
    }
}

// ------------------------------------------------------------------------------------------------------------
// forward, 16-bit inputs (v2): grid (ceil(L / (64 QS)), B*H), block 256; wavefront w owns 16 QS query rows.
//   * S^T = K Q^T per 16-key sub-tile: the K fragment (ds_read_b128 from the row-major tile) is read once and used
//     for all QS query sub-tiles held in registers;
//   * P V as O^T += V^T P: the V^T operand comes straight from the row-major V tile via ds_read_b64_tr_b16 (the
//     hardware transpose read), again shared by the QS sub-tiles;
//   * row sums on the MFMA (ones^T P, on the same bf16/f16 P as the numerator), row max by max3 trees and the
//     permlane16/32 swaps; masking only on the tail tile; the O rescale skipped while no row max grows;
//   * K/V tiles double-buffered: the next tile's global loads are in flight during the current tile's MFMAs (at
//     D = 32 as LDS DMA straight into the other buffer, no staging registers: kv_swz).
template <typename T, typename V4>
__device__ __forceinline__ V4 tr_read(const T *p) {
    typedef __attribute__((ext_vector_type(4))) T TV4;
    return __builtin_bit_cast(V4, *reinterpret_cast<const TV4 *>(p));
}

__device__ __forceinline__ float xmax_groups(float v) {  // max over the 4 lane groups (lanes l, l^16, l^32, l^48)
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r2[0]), __uint_as_float(r2[1]));
}

template <int DT>
__device__ __forceinline__ typename Ty<DT>::V8 tr_frag(const typename Ty<DT>::T *tile, int ld, int k0, int d0,
                                                      int lane) {
    // rows k0 + 4g + (i>>2) and k0 + 16 + 4g + (i>>2), columns d0 + 4 (i&3): lane i of group g receives column
    // d0 + i of 4 consecutive keys -> the 16x16x32 A operand of V^T with the key order of the P operand
    using T = typename Ty<DT>::T;
    using V8 = typename Ty<DT>::V8;
    const int g = lane >> 4, i = lane & 15;
    const T *p0 = tile + (k0 + 4 * g + (i >> 2)) * ld + d0 + 4 * (i & 3);
    typedef short s4v __attribute__((__vector_size__(8)));
    // the transposing read moves 16-bit elements regardless of type: the i16 form serves bf16 and f16
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p0));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p0 + 16 * ld));
    typedef __attribute__((ext_vector_type(8))) short s8v;
    const s8v r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(V8, r);
}

// K/V tiles staged by LDS DMA (global_load_lds_dwordx4: lane i's 16 B land at M0 + 16 i, no VGPR staging) at
// D = 32 and 64: unpadded rows (64 / 128 B) whose 16-B chunks are XOR-permuted by row bits (logical chunk c of row r
// sits at physical chunk c ^ kv_swz<D>(r)). The permutation lives in each lane's SOURCE address (the DMA writes
// 1 KiB contiguously); reads apply the same XOR. Row reads (ds_read_b128, lanes = rows 0..15 of one chunk) and the
// transposed reads (ds_read_b64_tr_b16, 8 rows x 32 B per 32-lane half) are both conflict-free on it by the bank
// rule of MI355X_MICROARCH §LDS (checked exhaustively for both widths). Against register staging into padded rows
// (D = 128 keeps that): bench level fwd / dQ / dK,dV -2.5 / -2.2 / -1.8 % at D = 32, outputs bitwise equal
// (profiles/r05/ab_attn_dma; held at 5 waves per SIMD the forward gained nothing more); at D = 64 (LGM's C = 1024
// levels) fwd / dQ / dK,dV -2…-10 / -5…-7 / -3…-6 % (profiles/r05/ab_attn_d64).
template <int D>
__device__ __forceinline__ int kv_swz(int r) {
    if constexpr (D == 32) return ((r >> 2) & 1) << 1;       // rows r, r + 4 of a transposed read: other 32 B
    else return (((r >> 1) & 3) << 1) | ((r >> 2) & 1);       // D = 64: two rows per 256-B bank line
}
__device__ __forceinline__ unsigned lds_addr32(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
// Issued from inline asm so that the compiler's waitcnt pass does not tie later LDS reads to the pending copy;
// completion is ordered by vm_wait() + a barrier. M0 is saved and restored (the compiler owns it).
__device__ __forceinline__ void lds_dma16(const void *src, unsigned lds_base) {
    const unsigned m = __builtin_amdgcn_readfirstlane(lds_base);
    unsigned saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(m), "v"(src)
                 : "memory");
}
__device__ __forceinline__ void vm_wait() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)
// The 4-byte form: lane i's dword lands at M0 + 4 i (64 consecutive floats per wave-instruction).
__device__ __forceinline__ void lds_dma4(const void *src, unsigned lds_base) {
    const unsigned m = __builtin_amdgcn_readfirstlane(lds_base);
    unsigned saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(m), "v"(src)
                 : "memory");
}
// Per-row constants the dK,dV pass needs, written by k_attn_dq2 (16-bit paths): -lse * log2(e) and -delta of every
// query row, [B*H][Lp] each (Lp = L rounded up to 64; rows >= L hold -inf and 0, so P = 0 there), DMA'd with each
// query tile instead of loaded, negated and stored by one wave.
__host__ __device__ __forceinline__ int row_pitch(int L) { return (L + 63) & ~63; }

// One 64-row tile of each of two [tokens][ld] tensors into their swizzled LDS images by DMA: wave w copies rows
// 16 w .. 16 w + 15 (D / 32 pieces of 1 KiB per tensor); rows >= L read row L - 1 (finite; every consumer masks
// those rows: scores -> -inf, P = 0). Asynchronous: valid after vm_wait() in every wave and a barrier.
template <int D, typename T>
__device__ __forceinline__ void dma_tiles(const T *pa, long long lda, const T *pb, long long ldb, int r0, int L, T *ta,
                                          T *tb) {
    constexpr int CPR = D / 8;  // 16-B chunks per row
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < D / 32; j++) {
        const int slot = w * 16 * CPR + j * 64 + lane;  // 16-B slot of the image this lane fills
        const int r = slot / CPR, c = (slot % CPR) ^ kv_swz<D>(r);
        const long long row = min(r0 + r, L - 1);
        lds_dma16(pa + row * lda + 8 * c, lds_addr32(ta) + 1024u * (w * (D / 32) + j));
        lds_dma16(pb + row * ldb + 8 * c, lds_addr32(tb) + 1024u * (w * (D / 32) + j));
    }
}
// dma_tiles for a tile loop: this lane's source offsets inside tile 0 are computed once; a full tile adds the
// (uniform) tile offset to them, only a tile reaching past L recomputes with the row clamp.
template <int D, typename T>
struct DmaStream {
    const T *pa, *pb;
    long long lda, ldb;
    int oa, ob;  // this lane's element offsets in tile 0 (its row and swizzled chunk)
    __device__ __forceinline__ DmaStream(const T *a, long long la, const T *b, long long lb)
        : pa(a), pb(b), lda(la), ldb(lb) {
        constexpr int CPR = D / 8;
        const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
        const int slot = w * 16 * CPR + lane, r = slot / CPR, c = (slot % CPR) ^ kv_swz<D>(r);
        oa = (int)(r * la) + 8 * c;
        ob = (int)(r * lb) + 8 * c;
    }
    __device__ __forceinline__ void issue(int r0, int L, T *ta, T *tb) const {
        if (r0 + 64 <= L) {  // workgroup-uniform
            const int w = threadIdx.x >> 6;
            constexpr int RPP = 512 / D;  // rows per 1-KiB piece
#pragma unroll
            for (int j = 0; j < D / 32; j++) {
                lds_dma16(pa + (r0 + j * RPP) * lda + oa, lds_addr32(ta) + 1024u * (w * (D / 32) + j));
                lds_dma16(pb + (r0 + j * RPP) * ldb + ob, lds_addr32(tb) + 1024u * (w * (D / 32) + j));
            }
        } else {
            dma_tiles<D>(pa, lda, pb, ldb, r0, L, ta, tb);
        }
    }
};
// The 16x16x32 row operand (row `row`, logical 16-B chunk `ch`) from a swizzled image.
template <int DT, int D>
__device__ __forceinline__ typename Ty<DT>::V8 row_frag_swz(const typename Ty<DT>::T *tile, int row, int ch) {
    return *reinterpret_cast<const typename Ty<DT>::V8 *>(tile + row * D + 8 * (ch ^ kv_swz<D>(row)));
}
// tr_frag on a swizzled image; k0 a multiple of 32.
template <int DT, int D>
__device__ __forceinline__ typename Ty<DT>::V8 tr_frag_swz(const typename Ty<DT>::T *tile, int k0, int d0, int lane) {
    using T = typename Ty<DT>::T;
    using V8 = typename Ty<DT>::V8;
    const int g = lane >> 4, i = lane & 15;
    const int row = k0 + 4 * g + (i >> 2), ch = (d0 >> 3) + ((i & 3) >> 1);
    const T *p0 = tile + row * D + 8 * (ch ^ kv_swz<D>(row)) + 4 * (i & 1);
    typedef short s4v __attribute__((__vector_size__(8)));
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p0));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p0 + 16 * D));
    typedef __attribute__((ext_vector_type(8))) short s8v;
    const s8v r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(V8, r);
}

// Waves per SIMD the compiler is held to (register cap 512 / n) for D <= 64; D = 128 stays at the compiler's
// choice. Measured r02 (profiles/r02/ab_attn_wpe), cfg4 L=9600 C=512: forward 0.41 -> 0.34 ms at 3 (4 spills the
// D=64 two-sub-tile forward), dQ 0.51 -> 0.45 and dK/dV 0.64 -> 0.50 ms at 2 (4 puts dK/dV in scratch: 1.43 ms).
// LDS row stride of the 16-bit K/V/Q/dO tiles: D + 16 elements (row stride 24 / 40 / 72 dwords for D = 32 / 64 /
// 128, i.e. 24, 40 or 8 mod 64) puts the 16 lanes of every ds_read_b128 group on 16 distinct 4-bank slots and the 8
// rows of each ds_read_b64_tr_b16 half on disjoint 8-bank ranges: conflict-free. D + 8 (20 / 36 / 68 dwords) was
// 2-way on both (SQ_LDS_BANK_CONFLICT = half of the forward's LDS cycles, profiles/r02/pmc_attn). Measured
// (profiles/r02/ab_attn_pad): D = 64 fwd / dQ / dK,dV -5 / -8 / -10 %; D = 32 unchanged.
constexpr int LDK_PAD = 16, FWD_WPE = 3, BWD_WPE = 2;
// dK,dV at D = 32 with its tile in two 32-query halves (half the score registers live) held at 4 waves per SIMD (128
// VGPRs; 3 at the compiler's own 136): bench level k_attn_dkdv 636 -> 625 us (profiles/r04/ab_session_f; the
// forward split the same way ran 412 -> 435 us and stays whole)
constexpr int DKDV_WPE32 = 4;
// The two-sub-tile forward at D = 32 (grids of 512 .. 1,535 workgroups, e.g. cfg4's L = 9,600 level at 1,200) held
// at 5 waves per SIMD (96 VGPRs, spills outside the key loop only): 1,280 workgroup slots hold the whole grid in one
// round (4 waves: 1,024 slots, 1.17 rounds): cfg4 L = 9,600 k_attn_fwd 268.4 -> 264.2 us (profiles/r05/ab_attn_q2w5)
constexpr int FWD_WPE_Q2 = 5;
// The softmax's affine parts ride on the MFMAs: Q is pre-scaled by scale * log2(e) (rounded to the 16-bit type once;
// in registers in the forward and dQ kernels, as a second LDS image in dK/dV -- all three recompute P from the same
// rounded operands), so S comes out in log2 units, and the S / dP
// accumulators start at -m (-lse') and -delta of their rows, so exp2's argument and dS's (dP - delta) factor leave
// the MFMA ready: no per-score fma or subtract (profiles/r04: D = 32 fwd / dQ / dK,dV measured in DESIGN.md §4).
constexpr float ATT_THR = 8.0f;  // forward: the row reference m is raised only when a score exceeds it by more than
                                 // this (log2 units): P <= 2^8, exact either way
template <int DT, int N>
__device__ __forceinline__ void prescale(typename Ty<DT>::V8 (&v)[N], float c) {  // v *= c, rounded to the type
#pragma unroll
    for (int a = 0; a < N; a++)
#pragma unroll
        for (int j = 0; j < 8; j++) v[a][j] = (typename Ty<DT>::T)((float)v[a][j] * c);
}
constexpr long long QS_MIN_GRID = 512;  // two query sub-tiles per wave once the grid has this many workgroups
// The key-tile loop of the forward and dQ kernels: step(kb, tail, buffer) over the 64-key tiles, full tiles first,
// the buffer index alternating from 0 as a compile-time constant (the two buffers' bodies run in turn).
template <class Step>
__device__ __forceinline__ void tile_loop(int L, Step &&step) {
    using F = std::false_type;
    using Tr = std::true_type;
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    const int kfull = L & ~63;
    int kb = 0;
    for (; kb + 128 <= kfull; kb += 128) {
        step(kb, F{}, B0{});
        step(kb + 64, F{}, B1{});
    }
    if (kb < kfull) {  // one more full tile (buffer 0), then the tail in buffer 1
        step(kb, F{}, B0{});
        if (kfull < L) step(kfull, Tr{}, B1{});
    } else if (kfull < L) {
        step(kfull, Tr{}, B0{});
    }
}
template <int DT, int D, int QS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(D == 32 && QS == 2 ? FWD_WPE_Q2 : D <= 64 ? FWD_WPE : 1))) void k_attn_fwd2(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ q,
                                                  const typename Ty<DT>::T *__restrict__ k,
                                                  const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                  typename Ty<DT>::T *__restrict__ o, float *__restrict__ lse) {
    using T = typename Ty<DT>::T;
    using V8 = typename Ty<DT>::V8;
    constexpr bool DMA = D == 32 || D == 64;                      // LDS-DMA staging on the swizzled image (kv_swz)
    constexpr int LDK = DMA ? D : D + LDK_PAD;         // padded rows (see LDK_PAD)
    constexpr int CH = DMA ? 1 : 64 * D * 2 / 16 / NT;  // 16-B chunks per thread per tile (K or V)
    static_assert(CH >= 1, "tile too small for the loader");
    __shared__ __attribute__((aligned(16))) T Ks[2][64 * LDK];
    __shared__ __attribute__((aligned(16))) T Vs[2][64 * LDK];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int q0 = blockIdx.x * (64 * QS) + w * (16 * QS);
    const DmaStream<D, T> dsrc(k + base, ld, v + base, ld);
    auto dma_tile = [&](int kb, int buf) { dsrc.issue(kb, L, Ks[buf], Vs[buf]); };
    const float c = scale * LOG2E;
    YFrag<DT, D> qf[QS];
#pragma unroll
    for (int s = 0; s < QS; s++) {
        const int qr = q0 + 16 * s + r16;
        load_yfrag<DT, D>(qf[s], q + base + (long long)qr * ld, qr < L, g);
        prescale<DT, D / 32>(qf[s].v, c);  // scores come out in log2 units
    }
    f32x4 oacc[QS][D / 16], lacc[QS];
    float m[QS];
#pragma unroll
    for (int s = 0; s < QS; s++) {
        lacc[s] = zero4();
        m[s] = 0.f;
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++) oacc[s][dt] = zero4();
    }
    V8 ones;
#pragma unroll
    for (int j = 0; j < 8; j++) ones[j] = (T)1.0f;
    // tile loader (register staging)
    uint4 kr[CH], vr[CH];
    auto load_regs = [&](int kb) {
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            const int ci = tid + cc * NT, r = ci / (D / 8), col = (ci - r * (D / 8)) * 8;
            const bool ok = kb + r < L;
            const long long off = base + (long long)(kb + r) * ld + col;
            kr[cc] = ok ? *reinterpret_cast<const uint4 *>(k + off) : make_uint4(0u, 0u, 0u, 0u);
            vr[cc] = ok ? *reinterpret_cast<const uint4 *>(v + off) : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    auto store_regs = [&](int buf) {
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            const int ci = tid + cc * NT, r = ci / (D / 8), col = (ci - r * (D / 8)) * 8;
            *reinterpret_cast<uint4 *>(&Ks[buf][r * LDK + col]) = kr[cc];
            *reinterpret_cast<uint4 *>(&Vs[buf][r * LDK + col]) = vr[cc];
        }
    };
    if constexpr (DMA) {
        dma_tile(0, 0);
        vm_wait();
    } else {
        load_regs(0);
        store_regs(0);
    }
    __syncthreads();
    // one 64-key tile read from buffer CUR; TAIL: the last, partial tile (keys >= L masked): full tiles run a body
    // without the masking code. (An unconditional rescale instead of the branch below measured the same:
    // profiles/r02/ab_attn_pad.) CUR is a compile-time index (tile_loop runs the two buffers' bodies in turn), so
    // every LDS address is a per-lane base plus an immediate.
    auto step = [&](int kb, auto tail, auto cur_tag) {
        constexpr bool TAIL = decltype(tail)::value;
        constexpr int cur = decltype(cur_tag)::value;
        const bool more = kb + 64 < L;
        if (more) {  // in flight during this tile's compute
            if constexpr (DMA) dma_tile(kb + 64, cur ^ 1);  // (buffer cur^1 was last read before the previous barrier)
            else load_regs(kb + 64);
        }
        const T *Kt = Ks[cur], *Vt = Vs[cur];
        // ---- S^T sub-tiles (keys 16 sub + 4g + i, query r16 of sub-tile s)
        f32x4 sacc[QS][4];
#pragma unroll
        for (int sub = 0; sub < 4; sub++) {
            V8 kf[D / 32];
#pragma unroll
            for (int cc = 0; cc < D / 32; cc++)
                kf[cc] = DMA ? row_frag_swz<DT, D>(Kt, 16 * sub + r16, 4 * cc + g)
                             : *reinterpret_cast<const V8 *>(Kt + (16 * sub + r16) * LDK + 32 * cc + 8 * g);
#pragma unroll
            for (int s = 0; s < QS; s++) {
                f32x4 a = {-m[s], -m[s], -m[s], -m[s]};  // the MFMA leaves exp2's argument itself
#pragma unroll
                for (int cc = 0; cc < D / 32; cc++) a = mfma32<DT>(kf[cc], qf[s].v[cc], a);
                sacc[s][sub] = a;
            }
        }
        if (TAIL) {  // tail tile: keys >= L
#pragma unroll
            for (int sub = 0; sub < 4; sub++)
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (kb + 16 * sub + 4 * g + i >= L)
#pragma unroll
                        for (int s = 0; s < QS; s++) sacc[s][sub][i] = -INFINITY;
        }
        // ---- online softmax per query sub-tile; P as the B operand (key order of tr_frag)
        V8 pb[QS][2];
        // x = score - m (log2 units) straight from the MFMA. The reference m is raised (and O, l rescaled, x
        // shifted) only on the first tile or where some x exceeds ATT_THR: P = 2^x <= 2^ATT_THR, so no per-tile row
        // max and no per-score fma
#pragma unroll
        for (int s = 0; s < QS; s++) {
            float mxl = fmaxf(fmaxf(sacc[s][0][0], sacc[s][0][1]), fmaxf(sacc[s][0][2], sacc[s][0][3]));
#pragma unroll
            for (int sub = 1; sub < 4; sub++)
                mxl = fmaxf(fmaxf(mxl, sacc[s][sub][0]), fmaxf(fmaxf(sacc[s][sub][1], sacc[s][sub][2]), sacc[s][sub][3]));
            if (__ballot(kb == 0 || mxl > ATT_THR)) {  // wave-uniform, rare: kept a branch (not if-converted)
                asm volatile("" ::: "memory");
                const float mx = xmax_groups(mxl);
                const float dlt = kb == 0 ? mx : fmaxf(mx, 0.f);
                if (kb != 0) {
                    const float alpha = __builtin_amdgcn_exp2f(-dlt);
#pragma unroll
                    for (int dt = 0; dt < D / 16; dt++) oacc[s][dt] *= alpha;
                    lacc[s] *= alpha;
                }
                m[s] += dlt;
#pragma unroll
                for (int sub = 0; sub < 4; sub++) sacc[s][sub] -= dlt;
            }
#pragma unroll
            for (int t = 0; t < 2; t++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    pb[s][t][i] = (T)__builtin_amdgcn_exp2f(sacc[s][2 * t][i]);
                    pb[s][t][4 + i] = (T)__builtin_amdgcn_exp2f(sacc[s][2 * t + 1][i]);
                }
#pragma unroll
            for (int t = 0; t < 2; t++) lacc[s] = mfma32<DT>(ones, pb[s][t], lacc[s]);
        }
        // ---- O^T += V^T P
#pragma unroll
        for (int t = 0; t < 2; t++)
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++) {
                const V8 vf = DMA ? tr_frag_swz<DT, D>(Vt, 32 * t, 16 * dt, lane) : tr_frag<DT>(Vt, LDK, 32 * t, 16 * dt, lane);
#pragma unroll
                for (int s = 0; s < QS; s++) oacc[s][dt] = mfma32<DT>(vf, pb[s][t], oacc[s][dt]);
            }
        if (more) {
            if constexpr (DMA) vm_wait();  // this wave's copy landed (the barrier publishes every wave's)
            else store_regs(cur ^ 1);     // buffer cur^1 was last read before the previous barrier
        }
        __syncthreads();
    };
    tile_loop(L, step);
#pragma unroll
    for (int s = 0; s < QS; s++) {
        const int qr = q0 + 16 * s + r16;
        if (qr < L) {
            const float l = lacc[s][0];
            const float inv = 1.f / l;
            T *orow = o + ((long long)b * L + qr) * ((long long)H * D) + (long long)h * D;
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
                for (int i = 0; i < 4; i++) orow[16 * dt + 4 * g + i] = from_f<T>(oacc[s][dt][i] * inv);
            if (g == 0) lse[(long long)bh * L + qr] = (m[s] + log2f(l)) * LN2;
        }
    }
}

// ------------------------------------------------------------------------------------------------------------
// backward, 16-bit inputs (v2). Both kernels read their tiles row-major from LDS only: the row reads feed the
// S / dP products, the transposed operands (Q^T, dO^T, K^T) come from the same images via ds_read_b64_tr_b16.
// Tiles are double-buffered like the forward's (LDS DMA at D = 32, register staging otherwise).
template <typename T, int D>
struct TileLoader {  // one 64-row tile of up to two [tokens][ld] tensors, CH 16-B chunks per thread each
    static constexpr int CH = 64 * D * 2 / 16 / NT;
    uint4 a[CH], b[CH];
    __device__ __forceinline__ void load(const T *pa, long long lda, const T *pb, long long ldb, int r0, int L) {
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            const int ci = threadIdx.x + cc * NT, r = ci / (D / 8), col = (ci - r * (D / 8)) * 8;
            const bool ok = r0 + r < L;
            a[cc] = ok ? *reinterpret_cast<const uint4 *>(pa + (long long)(r0 + r) * lda + col) : make_uint4(0u, 0u, 0u, 0u);
            b[cc] = ok ? *reinterpret_cast<const uint4 *>(pb + (long long)(r0 + r) * ldb + col) : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    __device__ __forceinline__ void store(T *ta, T *tb, int ldt) {
#pragma unroll
        for (int cc = 0; cc < CH; cc++) {
            const int ci = threadIdx.x + cc * NT, r = ci / (D / 8), col = (ci - r * (D / 8)) * 8;
            *reinterpret_cast<uint4 *>(ta + r * ldt + col) = a[cc];
            *reinterpret_cast<uint4 *>(tb + r * ldt + col) = b[cc];
        }
    }
};

// dK, dV: grid (ceil(L / (64 KS)), B*H); wavefront w owns keys k0 + 16 s + (lane & 15), s < KS.
template <int DT, int D, int KS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(D <= 32 ? DKDV_WPE32 : D <= 64 ? BWD_WPE : 1))) void k_attn_dkdv2(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ qc,
                                                   const typename Ty<DT>::T *__restrict__ k,
                                                   const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                   const typename Ty<DT>::T *__restrict__ dout,
                                                   const float *__restrict__ nrow,
                                                   typename Ty<DT>::T *__restrict__ dk,
                                                   typename Ty<DT>::T *__restrict__ dv, long long ldd) {
    using T = typename Ty<DT>::T;
    using V8 = typename Ty<DT>::V8;
    constexpr bool DMA = D == 32 || D == 64;  // LDS-DMA staging on the swizzled image (kv_swz)
    constexpr int LDK = DMA ? D : D + LDK_PAD;
    __shared__ __attribute__((aligned(16))) T Qs[2][64 * LDK];  // Q * scale * log2(e), rounded (k_attn_dq2's qc)
    __shared__ __attribute__((aligned(16))) T Os[2][64 * LDK];
    __shared__ float sl[2][64], sd[2][64];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const long long obase = (long long)b * L * H * D + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int k0 = blockIdx.x * (64 * KS) + w * (16 * KS);
    const float dk_scale = 1.0f / LOG2E;  // scale / c: dK = scale sum dS^T Q = (scale / c) sum dS^T (Q c)
    YFrag<DT, D> kf[KS], vf[KS];
#pragma unroll
    for (int s = 0; s < KS; s++) {
        const int kr = k0 + 16 * s + r16;
        load_yfrag<DT, D>(kf[s], k + base + (long long)kr * ld, kr < L, g);
        load_yfrag<DT, D>(vf[s], v + base + (long long)kr * ld, kr < L, g);
    }
    f32x4 dka[KS][D / 16], dva[KS][D / 16];
#pragma unroll
    for (int s = 0; s < KS; s++)
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++) { dka[s][dt] = zero4(); dva[s][dt] = zero4(); }
    TileLoader<T, D> ld_;
    const DmaStream<D, T> dsrc(qc + (long long)bh * L * D, D, dout + obase, (long long)H * D);
    const int Lp = row_pitch(L);
    const float *nl2 = nrow + (long long)bh * Lp + lane, *nd = nl2 + (long long)gridDim.y * Lp;
    auto load_rows2 = [&](int qb, int buf) {
        if constexpr (DMA)
            dsrc.issue(qb, L, Qs[buf], Os[buf]);
        else
            ld_.load(qc + (long long)bh * L * D, D, dout + obase, (long long)H * D, qb, L);
        if (w == 0) {  // the tile's -lse' and -delta rows, straight into their LDS slots (workgroup-uniform by wave)
            lds_dma4(nl2 + qb, lds_addr32(&sl[buf][0]));
            lds_dma4(nd + qb, lds_addr32(&sd[buf][0]));
        }
    };
    auto store_rows2 = [&](int buf) {
        // S from the same rounded operand as k_attn_fwd2 / k_attn_dq2 (Q * c, which k_attn_dq2 wrote; K unscaled),
        // so the P recomputed here is the P whose row sums gave lse (with K * c instead, dK / dV were 1.8x further from
        // fp64: 7.2e-3 vs 4.0e-3 rel L2, bf16 at L 4096; profiles/r05/attn_prescale). dK's product reads the same
        // image and is rescaled by scale / c at the end (a second, unscaled Q image cost +15 % dK,dV time; scaling
        // the staged tile here +8.5 %)
        if constexpr (!DMA) ld_.store(Qs[buf], Os[buf], LDK);
        vm_wait();  // this wave's copies landed (the barrier publishes every wave's)
    };
    load_rows2(0, 0);
    store_rows2(0);
    __syncthreads();
    // one 64-query tile read from buffer CUR (a compile-time index: the loop below runs the two buffers' bodies in
    // turn, so every LDS address is a per-lane base plus an immediate)
    auto tile = [&](int qb, auto cur_tag) {
        constexpr int cur = decltype(cur_tag)::value;
        const bool more = qb + 64 < L;
        if (more) load_rows2(qb + 64, cur ^ 1);
        const T *Qt = Qs[cur], *Ot = Os[cur];  // (dK from Q * c: rescaled below)
        // the tile's two 32-query halves one after the other (S / dP of subs 2t, 2t + 1, then their dV / dK
        // products): half the score registers live at once (dK,dV at D = 32 fits 4 waves per SIMD instead of 3)
#pragma unroll
        for (int t = 0; t < 2; t++) {
            f32x4 sacc[KS][2], dpa[KS][2];
#pragma unroll
            for (int h2 = 0; h2 < 2; h2++) {
                const int sub = 2 * t + h2;
                V8 qr[D / 32], orr[D / 32];
#pragma unroll
                for (int cc = 0; cc < D / 32; cc++) {
                    if constexpr (DMA) {
                        qr[cc] = row_frag_swz<DT, D>(Qt, 16 * sub + r16, 4 * cc + g);
                        orr[cc] = row_frag_swz<DT, D>(Ot, 16 * sub + r16, 4 * cc + g);
                    } else {
                        qr[cc] = *reinterpret_cast<const V8 *>(Qt + (16 * sub + r16) * LDK + 32 * cc + 8 * g);
                        orr[cc] = *reinterpret_cast<const V8 *>(Ot + (16 * sub + r16) * LDK + 32 * cc + 8 * g);
                    }
                }
                // (the accumulators start at -lse' / -delta of their rows q = 16 sub + 4 g + i, read as stored)
                f32x4 ainit, dinit;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    ainit[i] = sl[cur][16 * sub + 4 * g + i];  // -lse' (negated when stored: no per-tile negations)
                    dinit[i] = sd[cur][16 * sub + 4 * g + i];  // -delta
                }
#pragma unroll
                for (int s = 0; s < KS; s++) {
                    f32x4 a = ainit, dp = dinit;
#pragma unroll
                    for (int cc = 0; cc < D / 32; cc++) {
                        a = mfma32<DT>(qr[cc], kf[s].v[cc], a);     // S[q = 16 sub + 4g + i][key]
                        dp = mfma32<DT>(orr[cc], vf[s].v[cc], dp);  // dP[q][key]
                    }
                    sacc[s][h2] = a;
                    dpa[s][h2] = dp;
                }
            }
            V8 pb[KS], db[KS];
#pragma unroll
            for (int h2 = 0; h2 < 2; h2++)
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int s = 0; s < KS; s++) {
                        const float p = __builtin_amdgcn_exp2f(sacc[s][h2][i]);
                        pb[s][4 * h2 + i] = (T)p;
                        db[s][4 * h2 + i] = (T)(p * dpa[s][h2][i]);
                    }
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++) {
                const V8 oT = DMA ? tr_frag_swz<DT, D>(Ot, 32 * t, 16 * dt, lane) : tr_frag<DT>(Ot, LDK, 32 * t, 16 * dt, lane);  // dO^T
                const V8 qT = DMA ? tr_frag_swz<DT, D>(Qt, 32 * t, 16 * dt, lane) : tr_frag<DT>(Qt, LDK, 32 * t, 16 * dt, lane);  // Q^T
#pragma unroll
                for (int s = 0; s < KS; s++) {
                    dva[s][dt] = mfma32<DT>(oT, pb[s], dva[s][dt]);
                    dka[s][dt] = mfma32<DT>(qT, db[s], dka[s][dt]);
                }
            }
        }
        if (more) store_rows2(cur ^ 1);
        __syncthreads();
    };
    for (int qb = 0; qb < L; qb += 128) {
        tile(qb, std::integral_constant<int, 0>{});
        if (qb + 64 < L) tile(qb + 64, std::integral_constant<int, 1>{});
    }
#pragma unroll
    for (int s = 0; s < KS; s++) {
        const int key = k0 + 16 * s + r16;
        if (key < L) {
            T *krow = dk + (long long)b * L * ldd + (long long)key * ldd + (long long)h * D;
            T *vrow = dv + (long long)b * L * ldd + (long long)key * ldd + (long long)h * D;
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    krow[16 * dt + 4 * g + i] = from_f<T>(dka[s][dt][i] * dk_scale);
                    vrow[16 * dt + 4 * g + i] = from_f<T>(dva[s][dt][i]);
                }
        }
    }
}

// dQ: grid (ceil(L / (64 QS)), B*H); wavefront w owns query rows q0 + 16 s + (lane & 15), s < QS.
template <int DT, int D, int QS>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(D <= 64 ? BWD_WPE : 1))) void k_attn_dq2(int L, int H, float scale, const typename Ty<DT>::T *__restrict__ q,
                                                 const typename Ty<DT>::T *__restrict__ k,
                                                 const typename Ty<DT>::T *__restrict__ v, long long ld,
                                                 const typename Ty<DT>::T *__restrict__ dout,
                                                 const float *__restrict__ lse, float *__restrict__ nrow,
                                                 typename Ty<DT>::T *__restrict__ dq, long long ldd,
                                                 const typename Ty<DT>::T *__restrict__ o,
                                                 typename Ty<DT>::T *__restrict__ qc) {
    using T = typename Ty<DT>::T;
    using V8 = typename Ty<DT>::V8;
    constexpr bool DMA = D == 32 || D == 64;  // LDS-DMA staging on the swizzled image (kv_swz)
    constexpr int LDK = DMA ? D : D + LDK_PAD;
    __shared__ __attribute__((aligned(16))) T Ks[2][64 * LDK];
    __shared__ __attribute__((aligned(16))) T Vs[2][64 * LDK];
    const int bh = blockIdx.y, b = bh / H, h = bh - b * H;
    const long long base = (long long)b * L * ld + (long long)h * D;
    const long long obase = (long long)b * L * H * D + (long long)h * D;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane >> 4, r16 = lane & 15;
    const int q0 = blockIdx.x * (64 * QS) + w * (16 * QS);
    const float c = scale * LOG2E;
    YFrag<DT, D> qf[QS], of[QS];
    float l2[QS], dl[QS];
#pragma unroll
    for (int s = 0; s < QS; s++) {
        const int qr = q0 + 16 * s + r16;
        const bool qv = qr < L;
        load_yfrag<DT, D>(qf[s], q + base + (long long)qr * ld, qv, g);
        load_yfrag<DT, D>(of[s], dout + obase + (long long)qr * H * D, qv, g);
        l2[s] = qv ? lse[(long long)bh * L + qr] * LOG2E : INFINITY;
        // delta = rowsum(dO o O) of this lane's row, here instead of a separate pass: each of the row's four lanes
        // (g) holds D / 4 of its elements; their partial sums meet by two lane exchanges, and lane g = 0 stores the
        // row's -delta and -lse' for k_attn_dkdv2 (launched after this kernel; row_pitch)
        {
            YFrag<DT, D> ofr;
            load_yfrag<DT, D>(ofr, o + obase + (long long)qr * H * D, qv, g);
            float part = 0.f;
#pragma unroll
            for (int cc = 0; cc < D / 32; cc++)
#pragma unroll
                for (int j = 0; j < 8; j++) part = fmaf((float)ofr.v[cc][j], (float)of[s].v[cc][j], part);
            part += __shfl_xor(part, 16, 64);
            part += __shfl_xor(part, 32, 64);
            dl[s] = qv ? part : 0.f;
            const int Lp = row_pitch(L);
            if (g == 0 && qr < Lp) {  // (the grid covers every row below Lp: 64 QS rows per workgroup)
                nrow[(long long)bh * Lp + qr] = qv ? -l2[s] : -INFINITY;
                nrow[(long long)gridDim.y * Lp + (long long)bh * Lp + qr] = qv ? -part : 0.f;
            }
        }
        prescale<DT, D / 32>(qf[s].v, c);  // S in log2 units
        if (qv) {  // the rounded Q * c rows for k_attn_dkdv2 ([B*H][L][D]), so it recomputes this P exactly
            T *dst = qc + ((long long)bh * L + qr) * D;
#pragma unroll
            for (int cc = 0; cc < D / 32; cc++) *reinterpret_cast<V8 *>(dst + 32 * cc + 8 * g) = qf[s].v[cc];
        }
    }
    f32x4 dqa[QS][D / 16];
#pragma unroll
    for (int s = 0; s < QS; s++)
#pragma unroll
        for (int dt = 0; dt < D / 16; dt++) dqa[s][dt] = zero4();
    TileLoader<T, D> ld_;
    if constexpr (DMA) {
        dma_tiles<D>(k + base, ld, v + base, ld, 0, L, Ks[0], Vs[0]);
        vm_wait();
    } else {
        ld_.load(k + base, ld, v + base, ld, 0, L);
        ld_.store(Ks[0], Vs[0], LDK);
    }
    __syncthreads();
    const DmaStream<D, T> dsrc(k + base, ld, v + base, ld);
    // one 64-key tile read from buffer CUR (compile-time: tile_loop); TAIL: the last, partial tile (keys >= L masked)
    // -- full tiles run a body without the masking (a runtime tail flag left ~70 compare / select VALU per tile in
    // the main loop)
    auto step = [&](int kb, auto tail_tag, auto cur_tag) {
        constexpr bool TAIL = decltype(tail_tag)::value;
        constexpr int cur = decltype(cur_tag)::value;
        const bool more = kb + 64 < L;
        if (more) {
            if constexpr (DMA) dsrc.issue(kb + 64, L, Ks[cur ^ 1], Vs[cur ^ 1]);
            else ld_.load(k + base, ld, v + base, ld, kb + 64, L);
        }
        const T *Kt = Ks[cur], *Vt = Vs[cur];
        // the tile's two 32-key halves one after the other (half the score registers live at once)
#pragma unroll
        for (int t = 0; t < 2; t++) {
            f32x4 sacc[QS][2], dpa[QS][2];
#pragma unroll
            for (int h2 = 0; h2 < 2; h2++) {
                const int sub = 2 * t + h2;
                V8 kr[D / 32], vr[D / 32];
#pragma unroll
                for (int cc = 0; cc < D / 32; cc++) {
                    if constexpr (DMA) {
                        kr[cc] = row_frag_swz<DT, D>(Kt, 16 * sub + r16, 4 * cc + g);
                        vr[cc] = row_frag_swz<DT, D>(Vt, 16 * sub + r16, 4 * cc + g);
                    } else {
                        kr[cc] = *reinterpret_cast<const V8 *>(Kt + (16 * sub + r16) * LDK + 32 * cc + 8 * g);
                        vr[cc] = *reinterpret_cast<const V8 *>(Vt + (16 * sub + r16) * LDK + 32 * cc + 8 * g);
                    }
                }
#pragma unroll
                for (int s = 0; s < QS; s++) {
                    // (the accumulators start at -lse' / -delta of the lane's query)
                    f32x4 a = {-l2[s], -l2[s], -l2[s], -l2[s]};
                    f32x4 dp = {-dl[s], -dl[s], -dl[s], -dl[s]};
#pragma unroll
                    for (int cc = 0; cc < D / 32; cc++) {
                        a = mfma32<DT>(kr[cc], qf[s].v[cc], a);    // S^T[key = 16 sub + 4g + i][q]
                        dp = mfma32<DT>(vr[cc], of[s].v[cc], dp);  // dP^T[key][q]
                    }
                    sacc[s][h2] = a;
                    dpa[s][h2] = dp;
                }
            }
            V8 db[QS];
#pragma unroll
            for (int h2 = 0; h2 < 2; h2++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const bool kv = !TAIL || kb + 32 * t + 16 * h2 + 4 * g + i < L;
#pragma unroll
                    for (int s = 0; s < QS; s++) {
                        const float p = kv ? __builtin_amdgcn_exp2f(sacc[s][h2][i]) : 0.f;
                        db[s][4 * h2 + i] = (T)(p * dpa[s][h2][i]);
                    }
                }
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++) {
                const V8 kT = DMA ? tr_frag_swz<DT, D>(Kt, 32 * t, 16 * dt, lane) : tr_frag<DT>(Kt, LDK, 32 * t, 16 * dt, lane);  // K^T
#pragma unroll
                for (int s = 0; s < QS; s++) dqa[s][dt] = mfma32<DT>(kT, db[s], dqa[s][dt]);
            }
        }
        if (more) {
            if constexpr (DMA) vm_wait();  // this wave's copies landed (the barrier publishes every wave's)
            else ld_.store(Ks[cur ^ 1], Vs[cur ^ 1], LDK);
        }
        __syncthreads();
    };
    tile_loop(L, step);
#pragma unroll
    for (int s = 0; s < QS; s++) {
        const int qr = q0 + 16 * s + r16;
        if (qr < L) {
            T *row = dq + (long long)b * L * ldd + (long long)qr * ldd + (long long)h * D;
#pragma unroll
            for (int dt = 0; dt < D / 16; dt++)
#pragma unroll
                for (int i = 0; i < 4; i++) row[16 * dt + 4 * g + i] = from_f<T>(dqa[s][dt][i] * scale);
        }
    }
}

template <int DT, int D>
int fwd_impl(int B, int L, int H, float scale, const void *q, const void *k, const void *v, long long ld, void *o,
             float *lse, hipStream_t st) {
    using T = typename Ty<DT>::T;
    if constexpr (DT != LGM_ATTN_F32) {
        // two query sub-tiles per wavefront when the grid stays large enough to fill the chip; at D = 32 four (64
        // queries per wave, 3 waves per SIMD at 168 VGPRs: each K fragment and V^T fragment read from LDS feeds four
        // MFMAs) once the grid covers two rounds of the 768 workgroup slots: bench level (2,048 workgroups)
        // k_attn_fwd -5 % against two, but cfg4's L = 9,600 (608 workgroups, a fifth of the slots idle) +10 %
        // (profiles/r05/ab_attn_qs; three sub-tiles measured slower, and the same widening of dQ / dK,dV gained nothing)
        constexpr int QS4 = D == 32 ? 4 : 0;
        constexpr int QS2 = D <= 64 ? 2 : 1;
        constexpr long long QS4_MIN_GRID = 1536;
        if (QS4 && (long long)((L + 255) / 256) * B * H >= QS4_MIN_GRID) {
            dim3 grid((L + 255) / 256, B * H);
            LGM_LAUNCH("k_attn_fwd", st, (k_attn_fwd2<DT, D, (QS4 ? QS4 : 1)><<<grid, NT, 0, st>>>(
                                              L, H, scale, (const T *)q, (const T *)k, (const T *)v, ld, (T *)o, lse)));
        } else if (QS2 == 2 && (long long)((L + 127) / 128) * B * H >= QS_MIN_GRID) {
            dim3 grid((L + 127) / 128, B * H);
            LGM_LAUNCH("k_attn_fwd", st, (k_attn_fwd2<DT, D, QS2><<<grid, NT, 0, st>>>(
                                              L, H, scale, (const T *)q, (const T *)k, (const T *)v, ld, (T *)o, lse)));
        } else {
            dim3 grid((L + 63) / 64, B * H);
            LGM_LAUNCH("k_attn_fwd", st, (k_attn_fwd2<DT, D, 1><<<grid, NT, 0, st>>>(
                                              L, H, scale, (const T *)q, (const T *)k, (const T *)v, ld, (T *)o, lse)));
        }
        return LGM_OK;
    }
    dim3 grid((L + BQ - 1) / BQ, B * H);
    LGM_LAUNCH("k_attn_fwd", st, (k_attn_fwd<DT, D><<<grid, NT, 0, st>>>(L, H, scale, (const T *)q, (const T *)k,
                                                                       (const T *)v, ld, (T *)o, lse)));
    return LGM_OK;
}

// backward workspace. fp32: delta [B*H][L]. 16-bit: -lse' and -delta [2][B*H][row_pitch(L)] fp32, then
// Q * scale * log2(e) [B*H][L][D] in the input type.
size_t qc_offset(int B, int L, int H) {
    return (2 * (size_t)B * H * row_pitch(L) * sizeof(float) + 255) & ~(size_t)255;
}

template <int DT, int D>
int bwd_impl(int B, int L, int H, float scale, const void *q, const void *k, const void *v, long long ld,
             const void *o, const float *lse, const void *dout, void *dq, void *dk, void *dv, long long ldd,
             float *delta, hipStream_t st) {
    using T = typename Ty<DT>::T;
    const long long rows = (long long)B * L * H;
    T *qc = reinterpret_cast<T *>(reinterpret_cast<char *>(delta) + qc_offset(B, L, H));  // (16-bit paths)
    if constexpr (DT != LGM_ATTN_F32) {  // (delta computed by k_attn_dq2 itself)
        constexpr int S2 = D <= 32 ? 2 : 1;  // two 16-row sub-tiles per wavefront where registers allow
        const bool two = S2 == 2 && (long long)((L + 127) / 128) * B * H >= 512;
        dim3 g2((L + (two ? 127 : 63)) / (two ? 128 : 64), B * H);
        if (two) {
            LGM_LAUNCH("k_attn_dq", st, (k_attn_dq2<DT, D, S2><<<g2, NT, 0, st>>>(L, H, scale, (const T *)q,
                       (const T *)k, (const T *)v, ld, (const T *)dout, lse, delta, (T *)dq, ldd, (const T *)o, qc)));
            LGM_LAUNCH("k_attn_dkdv", st, (k_attn_dkdv2<DT, D, S2><<<g2, NT, 0, st>>>(L, H, scale, (const T *)qc,
                       (const T *)k, (const T *)v, ld, (const T *)dout, delta, (T *)dk, (T *)dv, ldd)));
        } else {
            LGM_LAUNCH("k_attn_dq", st, (k_attn_dq2<DT, D, 1><<<g2, NT, 0, st>>>(L, H, scale, (const T *)q,
                       (const T *)k, (const T *)v, ld, (const T *)dout, lse, delta, (T *)dq, ldd, (const T *)o, qc)));
            LGM_LAUNCH("k_attn_dkdv", st, (k_attn_dkdv2<DT, D, 1><<<g2, NT, 0, st>>>(L, H, scale, (const T *)qc,
                       (const T *)k, (const T *)v, ld, (const T *)dout, delta, (T *)dk, (T *)dv, ldd)));
        }
        return LGM_OK;
    }
    LGM_LAUNCH("k_attn_delta", st, (k_attn_delta<DT, D><<<(unsigned)((rows + 255) / 256), 256, 0, st>>>(
                                       B, L, H, (const T *)o, (const T *)dout, delta)));
    dim3 grid((L + 63) / 64, B * H);
    LGM_LAUNCH("k_attn_dq", st, (k_attn_dq<DT, D><<<grid, NT, 0, st>>>(L, H, scale, (const T *)q, (const T *)k,
                                                                     (const T *)v, ld, (const T *)dout, lse, delta,
                                                                     (T *)dq, ldd)));
    LGM_LAUNCH("k_attn_dkdv", st, (k_attn_dkdv<DT, D><<<grid, NT, 0, st>>>(L, H, scale, (const T *)q, (const T *)k,
                                                                         (const T *)v, ld, (const T *)dout, lse,
                                                                         delta, (T *)dk, (T *)dv, ldd)));
    return LGM_OK;
}

int check(int dtype, int B, int L, int H, int D) {
    if (dtype < 0 || dtype > 2 || B <= 0 || L <= 0 || H <= 0 || !(D == 32 || D == 64 || D == 128)) {
        set_error("unsupported attention shape/dtype (dtype=%d B=%d L=%d H=%d D=%d; D must be 32, 64 or 128)", dtype,
                  B, L, H, D);
        return LGM_E_INVALID;
    }
    return LGM_OK;
}

}  // namespace attn
}  // namespace lgm

#define LGM_ATTN_DISPATCH(FN, ...)                                                                             \
    switch (dtype * 1000 + D) {                                                                                \
        case LGM_ATTN_F32 * 1000 + 32: return lgm::attn::FN<LGM_ATTN_F32, 32>(__VA_ARGS__);                   \
        case LGM_ATTN_F32 * 1000 + 64: return lgm::attn::FN<LGM_ATTN_F32, 64>(__VA_ARGS__);                   \
        case LGM_ATTN_F32 * 1000 + 128: return lgm::attn::FN<LGM_ATTN_F32, 128>(__VA_ARGS__);                 \
        case LGM_ATTN_BF16 * 1000 + 32: return lgm::attn::FN<LGM_ATTN_BF16, 32>(__VA_ARGS__);                 \
        case LGM_ATTN_BF16 * 1000 + 64: return lgm::attn::FN<LGM_ATTN_BF16, 64>(__VA_ARGS__);                 \
        case LGM_ATTN_BF16 * 1000 + 128: return lgm::attn::FN<LGM_ATTN_BF16, 128>(__VA_ARGS__);               \
        case LGM_ATTN_F16 * 1000 + 32: return lgm::attn::FN<LGM_ATTN_F16, 32>(__VA_ARGS__);                   \
        case LGM_ATTN_F16 * 1000 + 64: return lgm::attn::FN<LGM_ATTN_F16, 64>(__VA_ARGS__);                   \
        case LGM_ATTN_F16 * 1000 + 128: return lgm::attn::FN<LGM_ATTN_F16, 128>(__VA_ARGS__);                 \
        default: return LGM_E_INVALID;                                                                         \
    }

extern "C" {

size_t lgm_attn_workspace_size(int dtype, int B, int L, int H, int D) {
    if (B <= 0 || L <= 0 || H <= 0 || D <= 0) return 0;
    if (dtype == LGM_ATTN_F32) return (size_t)B * L * H * sizeof(float);  // delta
    return lgm::attn::qc_offset(B, L, H) + (size_t)B * L * H * D * 2;      // row constants, Q * c
}

int lgm_attn_forward(int dtype, int B, int L, int H, int D, float scale, const void *q, const void *k,
                     const void *v, long long ld_qkv, void *o, float *lse, void *stream, const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    int rc = lgm::attn::check(dtype, B, L, H, D);
    if (rc) return rc;
    if (!q || !k || !v || !o || !lse) {
        lgm::set_error("null pointer");
        return LGM_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    LGM_ATTN_DISPATCH(fwd_impl, B, L, H, scale, q, k, v, ld_qkv, o, lse, st)
}

int lgm_attn_backward(int dtype, int B, int L, int H, int D, float scale, const void *q, const void *k,
                      const void *v, long long ld_qkv, const void *o, const float *lse, const void *d_o, void *dq,
                      void *dk, void *dv, long long ld_dqkv, void *workspace, size_t workspace_bytes, void *stream,
                      const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    int rc = lgm::attn::check(dtype, B, L, H, D);
    if (rc) return rc;
    if (!q || !k || !v || !o || !lse || !d_o || !dq || !dk || !dv) {
        lgm::set_error("null pointer");
        return LGM_E_INVALID;
    }
    if (!workspace || workspace_bytes < lgm_attn_workspace_size(dtype, B, L, H, D)) {
        lgm::set_error("attention workspace too small");
        return LGM_E_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    LGM_ATTN_DISPATCH(bwd_impl, B, L, H, scale, q, k, v, ld_qkv, o, lse, d_o, dq, dk, dv, ld_dqkv,
                      (float *)workspace, st)
}

}  // extern "C"
