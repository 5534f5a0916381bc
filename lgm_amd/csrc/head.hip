// lgm_amd/csrc/head.hip -- the fused Gaussian head (include/lgm_head.h): LGM.forward_gaussians' epilogue after
// the UNet (core/models.py:95-117): 1x1 conv 14 -> 14, the [B*V,14,h,w] -> [B,N,14] permute (N = V*h*w) and the
// five activations (core/models.py:40-44), and the mirror backward.
//
// The rotation activation is the reference's `F.normalize` with its DEFAULT dim=1 applied to the [B, N, 4] slice
// (core/models.py:43,112): each quaternion component is normalised over the N Gaussians of its object, not over
// the 4 components. That is a reduction over all points, so the forward is two kernels: k_head_fwd (conv, the
// other activations, the raw rotation channels and per-workgroup sums of their squares) and k_head_rot (the
// per-object norms, reduced in a fixed order by every workgroup, and the rotation columns divided in place).
// The backward likewise: k_head_rotdot (per-workgroup sums of r . dL/dr per object and component), then k_head_bwd
// (dL/dy for all channels, dL/dx = W^T dL/dy, per-workgroup dL/dW, dL/db partials) and k_head_reduce.
//
// Layout: one thread per splat point; grid (workgroups per object, B). The UNet output is channel-planar
// ([B*V, 14, h, w]): a wave's 64 points read each channel as one contiguous row. The Gaussians are point-major
// ([B, N, 14]): a workgroup's 256 rows are staged in LDS and stored as contiguous float4s. HBM-bound. All
// reductions run in a fixed order: the results are deterministic (no float atomics).
#include <hip/hip_runtime.h>

#include "common.h"
#include "lgm_head.h"

namespace lgm {
namespace {

constexpr int HC = 14, HT = 256, HNP = HC * HC + HC;  // channels, threads (= points) per workgroup, dW/db partials
constexpr int HEAD_MAX_BLOCKS = 2048;                 // backward workgroups (all objects), grid-stride beyond

template <typename TX> __device__ __forceinline__ float ld(const TX *p) { return (float)*p; }
template <typename TX> __device__ __forceinline__ TX st(float v) { return (TX)v; }

// torch semantics (core/models.py:40-44): clamp, sigmoid, 0.1 softplus (beta 1, threshold 20), 0.5 tanh + 0.5;
// the rotation channels are left raw here (normalised over the object by k_head_rot)
__device__ __forceinline__ void activate(const float y[HC], float g[HC]) {
#pragma unroll
    for (int c = 0; c < 3; c++) g[c] = fminf(fmaxf(y[c], -1.f), 1.f);
    g[3] = 1.f / (1.f + expf(-y[3]));
#pragma unroll
    for (int c = 4; c < 7; c++) g[c] = 0.1f * (y[c] > 20.f ? y[c] : log1pf(expf(y[c])));
#pragma unroll
    for (int c = 7; c < 11; c++) g[c] = y[c];
#pragma unroll
    for (int c = 11; c < 14; c++) g[c] = 0.5f * tanhf(y[c]) + 0.5f;
}

// dL/dy from dL/dgaussians (torch's backward formulas). Rotation: r = y / max(n, eps) with n the object's column
// norm; dL/dy = (d - r S) / n with S = sum over the object of r . d (n > eps), else d / eps.
__device__ __forceinline__ void activate_bwd(const float y[HC], const float d[HC], const float nrm[4],
                                             const float S[4], float dy[HC]) {
#pragma unroll
    for (int c = 0; c < 3; c++) dy[c] = (y[c] >= -1.f && y[c] <= 1.f) ? d[c] : 0.f;
    {
        const float s = 1.f / (1.f + expf(-y[3]));
        dy[3] = d[3] * s * (1.f - s);
    }
#pragma unroll
    for (int c = 4; c < 7; c++) {
        const float z = expf(y[c]);
        dy[c] = 0.1f * d[c] * (y[c] > 20.f ? 1.f : z / (z + 1.f));
    }
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float n = nrm[c];
        dy[7 + c] = n > 1e-12f ? (d[7 + c] - (y[7 + c] / n) * S[c]) / n : d[7 + c] / 1e-12f;
    }
#pragma unroll
    for (int c = 11; c < 14; c++) {
        const float t = tanhf(y[c]);
        dy[c] = d[c] * 0.5f * (1.f - t * t);
    }
}

__device__ __forceinline__ void load_params(const float *__restrict__ W, const float *__restrict__ bias, float *sW,
                                            float *sB) {
    const int t = threadIdx.x;
    if (t < HC * HC) sW[t] = W[t];
    else if (t < HNP) sB[t - HC * HC] = bias ? bias[t - HC * HC] : 0.f;
}

// output channels [o0, o1) of the 1x1 conv at one point (torch's order: bias + sum_i w[o][i] x[i])
template <typename TX, int O0 = 0, int O1 = HC>
__device__ __forceinline__ void conv_point(const TX *__restrict__ xp, int hw, const float *sW, const float *sB,
                                           float xi[HC], float y[HC]) {
#pragma unroll
    for (int i = 0; i < HC; i++) xi[i] = ld(xp + (size_t)i * hw);
#pragma unroll
    for (int o = O0; o < O1; o++) {
        float a = sB[o];
#pragma unroll
        for (int i = 0; i < HC; i++) a = fmaf(sW[o * HC + i], xi[i], a);
        y[o] = a;
    }
}

// Sum of a per-workgroup [nblk][4] partial array, component c = wave index (waves 0..3), in a fixed order.
__device__ __forceinline__ void reduce4(const float *__restrict__ part, int nblk, float *out4) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float s = 0.f;
    for (int j = lane; j < nblk; j += 64) s += part[(size_t)j * 4 + w];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) out4[w] = s;
}

// block-wide sum of 4 per-thread values (fixed order) -> written by thread 0
__device__ __forceinline__ void block_sum4(const float v[4], float *s4 /* LDS [4][4] */, float *dst) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        float x = v[c];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) s4[w * 4 + c] = x;
    }
    __syncthreads();
    if (threadIdx.x < 4) dst[threadIdx.x] = ((s4[threadIdx.x] + s4[4 + threadIdx.x]) + s4[8 + threadIdx.x]) + s4[12 + threadIdx.x];
}

// grid (nbx, B): rows of object b, points n = blockIdx.x * 256 + t
template <typename TX>
__global__ __launch_bounds__(HT) void k_head_fwd(int Nb, int hw, const TX *__restrict__ x, const float *__restrict__ W,
                                                 const float *__restrict__ bias, float *__restrict__ out,
                                                 float *__restrict__ sq_part) {
    __shared__ float sW[HC * HC], sB[HC], s4[16];
    __shared__ __attribute__((aligned(16))) float sOut[HT * HC];
    load_params(W, bias, sW, sB);
    __syncthreads();
    const int t = threadIdx.x, b = blockIdx.y;
    const int n0 = blockIdx.x * HT, n = n0 + t;
    const long long p0 = (long long)b * Nb + n0;
    float sq[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < Nb) {
        const long long p = p0 + t, bvi = p / hw;
        const int s = (int)(p - bvi * hw);
        float xi[HC], y[HC], g[HC];
        conv_point(x + bvi * HC * hw + s, hw, sW, sB, xi, y);
        activate(y, g);
#pragma unroll
        for (int c = 0; c < 4; c++) sq[c] = y[7 + c] * y[7 + c];
#pragma unroll
        for (int c = 0; c < HC; c++) sOut[t * HC + c] = g[c];
    }
    block_sum4(sq, s4, sq_part + ((size_t)b * gridDim.x + blockIdx.x) * 4);  // (contains a barrier)
    const int nv = min(HT, Nb - n0) * HC;  // this workgroup's rows, contiguous in out
    float *dst = out + p0 * HC;
    // p0 * 14 floats: 8-B aligned always, 16-B aligned when p0 is even
    if ((p0 & 1) == 0) {
        const int n4 = nv >> 2;
        for (int k = t; k < n4; k += HT) reinterpret_cast<float4 *>(dst)[k] = reinterpret_cast<const float4 *>(sOut)[k];
        for (int k = (n4 << 2) + t; k < nv; k += HT) dst[k] = sOut[k];
    } else {
        for (int k = t; k < (nv >> 1); k += HT) reinterpret_cast<float2 *>(dst)[k] = reinterpret_cast<const float2 *>(sOut)[k];
    }
}

// grid (nbx, B): the object's rotation column norms (fixed-order reduction of k_head_fwd's partials), then its
// rows' rotation channels divided in place: r = y / max(n, 1e-12) (F.normalize). Workgroup (0, b) stores n.
__global__ __launch_bounds__(HT) void k_head_rot(int Nb, const float *__restrict__ sq_part, float *__restrict__ out,
                                                 float *__restrict__ rot_norm) {
    __shared__ float sN[4];
    const int b = blockIdx.y;
    reduce4(sq_part + (size_t)b * gridDim.x * 4, gridDim.x, sN);
    __syncthreads();
    const int t = threadIdx.x, n = blockIdx.x * HT + t;
    if (t < 4) {
        const float nr = sqrtf(sN[t]);
        if (blockIdx.x == 0 && rot_norm) rot_norm[b * 4 + t] = nr;
    }
    if (n < Nb) {
        float *rf = out + ((long long)b * Nb + n) * HC + 7;
#pragma unroll
        for (int c = 0; c < 4; c++) rf[c] = rf[c] / fmaxf(sqrtf(sN[c]), 1e-12f);
    }
}

// grid (nbx, B): per-workgroup sums of r . dL/dr per rotation component (the normalisation's backward needs them)
template <typename TX>
__global__ __launch_bounds__(HT) void k_head_rotdot(int Nb, int hw, const TX *__restrict__ x,
                                                    const float *__restrict__ W, const float *__restrict__ bias,
                                                    const float *__restrict__ rot_norm, const float *__restrict__ dg,
                                                    float *__restrict__ dot_part) {
    __shared__ float sW[HC * HC], sB[HC], s4[16];
    load_params(W, bias, sW, sB);
    __syncthreads();
    const int t = threadIdx.x, b = blockIdx.y, n = blockIdx.x * HT + t;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < Nb) {
        const long long p = (long long)b * Nb + n, bvi = p / hw;
        const int s = (int)(p - bvi * hw);
        float xi[HC], y[HC];
        conv_point<TX, 7, 11>(x + bvi * HC * hw + s, hw, sW, sB, xi, y);
#pragma unroll
        for (int c = 0; c < 4; c++) v[c] = (y[7 + c] / fmaxf(rot_norm[b * 4 + c], 1e-12f)) * dg[p * HC + 7 + c];
    }
    block_sum4(v, s4, dot_part + ((size_t)b * gridDim.x + blockIdx.x) * 4);
}

// grid (nbg, B), grid-stride over the object's points
template <typename TX>
__global__ __launch_bounds__(HT) void k_head_bwd(int Nb, int hw, int nbx, const TX *__restrict__ x,
                                                 const float *__restrict__ W, const float *__restrict__ bias,
                                                 const float *__restrict__ rot_norm, const float *__restrict__ dot_part,
                                                 const float *__restrict__ dg, TX *__restrict__ dx,
                                                 float *__restrict__ partials) {
    __shared__ float sW[HC * HC], sB[HC], sS[4];
    __shared__ __attribute__((aligned(16))) float sD[HT * HC];  // dL/dgaussians rows, then dL/dy rows
    __shared__ float sX[HT * HC];                               // x rows (point-major)
    load_params(W, bias, sW, sB);
    const int t = threadIdx.x, b = blockIdx.y;
    reduce4(dot_part + (size_t)b * nbx * 4, nbx, sS);
    float nrm[4];
#pragma unroll
    for (int c = 0; c < 4; c++) nrm[c] = rot_norm[b * 4 + c];
    const int eo = t / HC, ei = t - eo * HC;  // this thread's weight entry (t < 196) / bias entry (196 <= t < 210)
    float acc = 0.f;
    for (int n0 = blockIdx.x * HT; n0 < Nb; n0 += gridDim.x * HT) {
        const int nvp = min(HT, Nb - n0), nv = nvp * HC;
        const long long p0 = (long long)b * Nb + n0;
        __syncthreads();  // previous round's readers of sD / sX are done (parameters and sS visible)
        const float *src = dg + p0 * HC;
        if ((p0 & 1) == 0) {
            const int n4 = nv >> 2;
            for (int k = t; k < n4; k += HT) reinterpret_cast<float4 *>(sD)[k] = reinterpret_cast<const float4 *>(src)[k];
            for (int k = (n4 << 2) + t; k < nv; k += HT) sD[k] = src[k];
        } else {
            for (int k = t; k < (nv >> 1); k += HT) reinterpret_cast<float2 *>(sD)[k] = reinterpret_cast<const float2 *>(src)[k];
        }
        __syncthreads();
        if (t < nvp) {
            const long long p = p0 + t, bvi = p / hw;
            const int s = (int)(p - bvi * hw);
            const size_t xo = (size_t)bvi * HC * hw + s;
            float xi[HC], y[HC], d[HC], dy[HC], S[4];
            conv_point(x + xo, hw, sW, sB, xi, y);
#pragma unroll
            for (int c = 0; c < HC; c++) d[c] = sD[t * HC + c];
#pragma unroll
            for (int c = 0; c < 4; c++) S[c] = sS[c];
            activate_bwd(y, d, nrm, S, dy);
#pragma unroll
            for (int i = 0; i < HC; i++) {
                float a = 0.f;
#pragma unroll
                for (int o = 0; o < HC; o++) a = fmaf(sW[o * HC + i], dy[o], a);
                dx[xo + (size_t)i * hw] = st<TX>(a);
            }
#pragma unroll
            for (int c = 0; c < HC; c++) {
                sD[t * HC + c] = dy[c];  // own row only
                sX[t * HC + c] = xi[c];
            }
        }
        __syncthreads();
        if (t < HC * HC) {
            for (int r = 0; r < nvp; r++) acc = fmaf(sD[r * HC + eo], sX[r * HC + ei], acc);
        } else if (t < HNP) {
            for (int r = 0; r < nvp; r++) acc += sD[r * HC + (t - HC * HC)];
        }
    }
    if (t < HNP) partials[((size_t)b * gridDim.x + blockIdx.x) * HNP + t] = acc;
}

// grid (HNP): workgroup e sums entry e of the nblk per-workgroup partials -- lane l the partials l, l + 64, ...
// (independent loads, unrolled), then a fixed shuffle tree: deterministic, and no longer one thread walking all
// nblk partials of its entry in a dependent chain (139 us at cfg5's 600 partials, now a few us).
constexpr int HR_LANES = 64, HR_UNROLL = 8;
__global__ __launch_bounds__(HR_LANES) void k_head_reduce(int nblk, const float *__restrict__ partials,
                                                          float *__restrict__ dW, float *__restrict__ db) {
    const int e = blockIdx.x, l = threadIdx.x;
    float s = 0.f;
    for (int b0 = 0; b0 < nblk; b0 += HR_LANES * HR_UNROLL) {
        float v[HR_UNROLL];
#pragma unroll
        for (int u = 0; u < HR_UNROLL; u++) {
            const int b = b0 + u * HR_LANES + l;
            v[u] = b < nblk ? partials[(size_t)b * HNP + e] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < HR_UNROLL; u++) s += v[u];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (l == 0) {
        if (e < HC * HC) dW[e] = s;
        else if (db) db[e - HC * HC] = s;
    }
}

struct HeadGrid {
    int Nb, nbx, nbg;
};
HeadGrid head_grid(int B, int V, int h, int w) {
    HeadGrid g;
    g.Nb = V * h * w;
    g.nbx = (g.Nb + HT - 1) / HT;
    g.nbg = B > 0 ? std::max(1, std::min(g.nbx, HEAD_MAX_BLOCKS / B)) : 1;
    return g;
}

int check_head(int dtype, int B, int V, int h, int w, const void *x, const float *W) {
    if (dtype != 0 && dtype != 1) {
        set_error("dtype must be 0 (fp32) or 1 (bf16), got %d", dtype);
        return LGM_E_INVALID;
    }
    if (B < 0 || B > 65535 || V <= 0 || h <= 0 || w <= 0 || (long long)V * h * w > 0x7fffffffLL - HT) {
        set_error("invalid sizes (B=%d V=%d h=%d w=%d)", B, V, h, w);
        return LGM_E_INVALID;
    }
    if ((B > 0 && !x) || !W) {
        set_error("null x / weight");
        return LGM_E_INVALID;
    }
    return LGM_OK;
}

}  // namespace
}  // namespace lgm

extern "C" {

size_t lgm_gaussian_head_workspace_size(int B, int V, int h, int w) {
    if (B < 0 || V <= 0 || h <= 0 || w <= 0) return 0;
    const lgm::HeadGrid g = lgm::head_grid(B, V, h, w);
    return ((size_t)B * g.nbx * 4 + (size_t)B * g.nbg * lgm::HNP) * sizeof(float);
}

int lgm_gaussian_head_forward(int dtype, int B, int V, int h, int w, const void *x, const float *weight,
                              const float *bias, float *gaussians, float *rot_norm, void *workspace,
                              size_t workspace_bytes, void *stream, const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    int rc = lgm::check_head(dtype, B, V, h, w, x, weight);
    if (rc) return rc;
    if (B == 0) return LGM_OK;
    if (!gaussians) {
        lgm::set_error("null gaussians");
        return LGM_E_INVALID;
    }
    const lgm::HeadGrid g = lgm::head_grid(B, V, h, w);
    if (!workspace || workspace_bytes < (size_t)B * g.nbx * 4 * sizeof(float)) {
        lgm::set_error("workspace too small");
        return LGM_E_WORKSPACE;
    }
    hipStream_t st = (hipStream_t)stream;
    float *sq = (float *)workspace;
    const dim3 grid(g.nbx, B);
    if (dtype == 0)
        LGM_LAUNCH("k_head_fwd", st, (lgm::k_head_fwd<float><<<grid, lgm::HT, 0, st>>>(g.Nb, h * w, (const float *)x,
                                                                                     weight, bias, gaussians, sq)));
    else
        LGM_LAUNCH("k_head_fwd", st, (lgm::k_head_fwd<__bf16><<<grid, lgm::HT, 0, st>>>(g.Nb, h * w, (const __bf16 *)x,
                                                                                      weight, bias, gaussians, sq)));
    LGM_LAUNCH("k_head_rot", st, (lgm::k_head_rot<<<grid, lgm::HT, 0, st>>>(g.Nb, sq, gaussians, rot_norm)));
    return LGM_OK;
}

int lgm_gaussian_head_backward(int dtype, int B, int V, int h, int w, const void *x, const float *weight,
                               const float *bias, const float *rot_norm, const float *d_gaussians, void *dx,
                               float *d_weight, float *d_bias, void *workspace, size_t workspace_bytes,
                               void *stream, const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    int rc = lgm::check_head(dtype, B, V, h, w, x, weight);
    if (rc) return rc;
    hipStream_t st = (hipStream_t)stream;
    if (!d_weight || (B > 0 && (!d_gaussians || !dx || !rot_norm))) {
        lgm::set_error("null pointer in backward");
        return LGM_E_INVALID;
    }
    if (B == 0) {
        if (hipMemsetAsync(d_weight, 0, lgm::HC * lgm::HC * 4, st) != hipSuccess ||
            (d_bias && hipMemsetAsync(d_bias, 0, lgm::HC * 4, st) != hipSuccess)) {
            lgm::set_error("hipMemsetAsync failed");
            return LGM_E_HIP;
        }
        return LGM_OK;
    }
    const lgm::HeadGrid g = lgm::head_grid(B, V, h, w);
    if (!workspace || workspace_bytes < lgm_gaussian_head_workspace_size(B, V, h, w)) {
        lgm::set_error("workspace too small");
        return LGM_E_WORKSPACE;
    }
    float *dot = (float *)workspace, *part = dot + (size_t)B * g.nbx * 4;
    const dim3 g1(g.nbx, B), g2(g.nbg, B);
    if (dtype == 0) {
        LGM_LAUNCH("k_head_rotdot", st, (lgm::k_head_rotdot<float><<<g1, lgm::HT, 0, st>>>(
                                            g.Nb, h * w, (const float *)x, weight, bias, rot_norm, d_gaussians, dot)));
        LGM_LAUNCH("k_head_bwd", st, (lgm::k_head_bwd<float><<<g2, lgm::HT, 0, st>>>(
                                         g.Nb, h * w, g.nbx, (const float *)x, weight, bias, rot_norm, dot,
                                         d_gaussians, (float *)dx, part)));
    } else {
        LGM_LAUNCH("k_head_rotdot", st, (lgm::k_head_rotdot<__bf16><<<g1, lgm::HT, 0, st>>>(
                                            g.Nb, h * w, (const __bf16 *)x, weight, bias, rot_norm, d_gaussians, dot)));
        LGM_LAUNCH("k_head_bwd", st, (lgm::k_head_bwd<__bf16><<<g2, lgm::HT, 0, st>>>(
                                         g.Nb, h * w, g.nbx, (const __bf16 *)x, weight, bias, rot_norm, dot,
                                         d_gaussians, (__bf16 *)dx, part)));
    }
    LGM_LAUNCH("k_head_reduce", st, (lgm::k_head_reduce<<<lgm::HNP, lgm::HR_LANES, 0, st>>>(B * g.nbg, part, d_weight,
                                                                                        d_bias)));
    return LGM_OK;
}

}  // extern "C"
