// lgm_amd/csrc/mvattn.hip -- the token layout changes around MVAttention's attention core (core/unet.py:35-49),
// fused with the GroupNorm before and the residual after:
//   k_mva_norm   GroupNorm(x) of [B*F, C, H, W] (core/unet.py:40, fp32 statistics), written straight into the
//                [B, F*H*W, C] token layout of :41-42 in the qkv Linear's input dtype (bf16 under autocast): one
//                kernel instead of torch's moments / fused-params / normalise launches + the permute copy + the cast.
//   k_mva_out    the [B, F*H*W, C] -> [B*F, C, H, W] permute of :45-46 fused with (x + res) * skip_scale of :47-48.
// Both are HBM-bound layout kernels: 64x64 LDS-tiled transposes (k_mva_out) or per-thread channel runs stored as
// 16-B vectors (k_mva_norm), so every global access is a full 64-B+ segment.
#include <hip/hip_bf16.h>
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

// grid (G, B*F), block 256: one (sample, group). Two passes over the group for mean and (centred) variance -- the
// group's Cg*HW elements are contiguous and stay in L2 -- then y = x * (rstd gamma) + (beta - mean rstd gamma)
// (torch's fused GroupNorm parameters) written to token rows: thread hw stores its Cg channels as 16-B vectors.
template <class TI, class TO>
__global__ __launch_bounds__(256) void k_mva_norm(int F, int C, int HW, int G, float eps, const TI *__restrict__ x,
                                                  const float *__restrict__ gamma, const float *__restrict__ beta,
                                                  TO *__restrict__ tok, float *__restrict__ mean_out,
                                                  float *__restrict__ rstd_out) {
    __shared__ float red[4];
    __shared__ float sa[256], sb[256];  // per-channel scale / shift (Cg <= 256)
    const int g = blockIdx.x, bf = blockIdx.y, Cg = C / G, tid = threadIdx.x;
    const int n = Cg * HW;
    const TI *xg = x + ((size_t)bf * C + (size_t)g * Cg) * HW;
    float s = 0.f;
    for (int i = tid; i < n; i += 256) s += to_f(xg[i]);
    const float mean = block_sum256(s, red) / (float)n;
    float v = 0.f;
    for (int i = tid; i < n; i += 256) {
        const float d = to_f(xg[i]) - mean;
        v = fmaf(d, d, v);
    }
    const float var = block_sum256(v, red) / (float)n;  // biased, as torch
    const float rstd = rsqrtf(fmaxf(var, 0.f) + eps);
    for (int c = tid; c < Cg; c += 256) {
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
    constexpr int VEC = 16 / sizeof(TO);  // channels per 16-B store
    const bool vec = (Cg % VEC) == 0 && (C % VEC) == 0;
    for (int hw = tid; hw < HW; hw += 256) {
        TO *row = tok + ((size_t)b * F * HW + (size_t)f * HW + hw) * C + (size_t)g * Cg;
        if (vec) {
            for (int c0 = 0; c0 < Cg; c0 += VEC) {
                union { uint4 u; TO e[VEC]; } pk;
#pragma unroll
                for (int k = 0; k < VEC; k++) {
                    const int c = c0 + k;
                    pk.e[k] = from_f<TO>(fmaf(to_f(xg[(size_t)c * HW + hw]), sa[c], sb[c]));
                }
                *reinterpret_cast<uint4 *>(row + c0) = pk.u;
            }
        } else {
            for (int c = 0; c < Cg; c++) row[c] = from_f<TO>(fmaf(to_f(xg[(size_t)c * HW + hw]), sa[c], sb[c]));
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
    for (int i = tid; i < 64 * 64; i += 256) {
        const int r = i >> 6, c = i & 63;  // token row r, channel c
        if (hw0 + r < HW && c0 + c < C) tile[c][r] = to_f(yb[(size_t)(hw0 + r) * C + c0 + c]);
    }
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
        const int r = i >> 6, h = i & 63;  // channel r, pixel h
        if (hw0 + h < HW && c0 + r < C) {
            const size_t o = ((size_t)bf * C + c0 + r) * HW + hw0 + h;
            float v = tile[r][h];
            if (res) {
                v += to_f(res[o]);
                v = to_f(from_f<TO>(v));  // (exact for an fp32 output)
                v *= skip;
            }
            out[o] = from_f<TO>(v);
        }
    }
}

template <class TI, class TO>
int launch_norm(int B, int F, int C, int HW, int G, float eps, const void *x, const float *gamma, const float *beta,
                void *tok, float *mean, float *rstd, hipStream_t st) {
    LGM_LAUNCH("k_mva_norm", st, (k_mva_norm<TI, TO><<<dim3(G, B * F), 256, 0, st>>>(
                                      F, C, HW, G, eps, (const TI *)x, gamma, beta, (TO *)tok, mean, rstd)));
    return LGM_OK;
}

template <class TY, class TR, class TO>
int launch_out(int B, int F, int C, int HW, const void *y, const void *res, float skip, void *out, hipStream_t st) {
    const dim3 grid((HW + 63) / 64, (C + 63) / 64, B * F);
    LGM_LAUNCH("k_mva_out", st,
               (k_mva_out<TY, TR, TO><<<grid, 256, 0, st>>>(F, C, HW, (const TY *)y, (const TR *)res, skip, (TO *)out)));
    return LGM_OK;
}

template <class TI>
int norm_by_out(int dto, int B, int F, int C, int HW, int G, float eps, const void *x, const float *gamma,
                const float *beta, void *tok, float *mean, float *rstd, hipStream_t st) {
    switch (dto) {
        case LGM_ATTN_F32: return launch_norm<TI, float>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, st);
        case LGM_ATTN_BF16: return launch_norm<TI, __hip_bfloat16>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, st);
        case LGM_ATTN_F16: return launch_norm<TI, __half>(B, F, C, HW, G, eps, x, gamma, beta, tok, mean, rstd, st);
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

}  // namespace
}  // namespace lgm

extern "C" int lgm_mva_norm_tokens(int dtype_x, int dtype_tok, int B, int F, int C, int HW, int groups, float eps,
                                   const void *x, const float *gamma, const float *beta, void *tokens, float *mean,
                                   float *rstd, void *stream) {
    lgm::clear_error();
    if (B < 0 || F <= 0 || C <= 0 || HW < 0 || groups <= 0 || C % groups || C / groups > 256) {
        lgm::set_error("lgm_mva_norm_tokens: bad shape B=%d F=%d C=%d HW=%d groups=%d", B, F, C, HW, groups);
        return LGM_E_INVALID;
    }
    if (B == 0 || HW == 0) return LGM_OK;
    if (!x || !tokens || !mean || !rstd) {
        lgm::set_error("lgm_mva_norm_tokens: null pointer");
        return LGM_E_INVALID;
    }
    hipStream_t st = (hipStream_t)stream;
    switch (dtype_x) {
        case LGM_ATTN_F32:
            return lgm::norm_by_out<float>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean, rstd, st);
        case LGM_ATTN_BF16:
            return lgm::norm_by_out<__hip_bfloat16>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean,
                                                    rstd, st);
        case LGM_ATTN_F16:
            return lgm::norm_by_out<__half>(dtype_tok, B, F, C, HW, groups, eps, x, gamma, beta, tokens, mean, rstd, st);
    }
    lgm::set_error("lgm_mva_norm_tokens: bad input dtype %d", dtype_x);
    return LGM_E_INVALID;
}

extern "C" int lgm_mva_tokens_out(int dtype_y, int dtype_res, int dtype_out, int B, int F, int C, int HW,
                                  const void *y, const void *res, float skip, void *out, void *stream) {
    lgm::clear_error();
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
