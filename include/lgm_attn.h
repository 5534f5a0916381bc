/*
 * lgm_attn.h -- C ABI of the multi-view attention kernels in liblgm_amd.so (lgm_amd/csrc/attention.hip).
 *
 * Replaces the xformers call of core/attention.py:74-84 (MemEffAttention.forward:
 *     x = memory_efficient_attention(q, k, v, attn_bias=None)   with q, k, v = unbind(qkv.reshape(B, L, 3, H, D), 2))
 * and the fp32 torch fallback core/attention.py:51-64 (Attention.forward: softmax(q k^T * scale) v), both reached
 * from core/unet.py:35-49 (MVAttention: L = num_frames * h * w tokens). Its backward replaces autograd through
 * the same op (xformers' memory_efficient_attention backward / the fallback's matmul + softmax backward).
 *
 * Tensors (device pointers, element type `dtype`):
 *   q, k, v : rows of the packed qkv Linear output [B, L, 3, H, D]; q = base, k = base + H*D, v = base + 2*H*D;
 *             token rows are ld_qkv elements apart (3*H*D when packed). Must be 16-byte aligned.
 *   o       : [B, L, H, D] contiguous (xformers output layout, core/attention.py:79).
 *   lse     : [B, H, L] fp32, natural-log row log-sum-exp of scale * q k^T (saved for the backward).
 *   d_o     : [B, L, H, D] contiguous; dq/dk/dv: same layout as q/k/v with row stride ld_dqkv.
 * D must be 32, 64 or 128 (LGM's UNet: 16 heads over 512 or 1024 channels -> D = 32 or 64); accumulation is fp32.
 * All work is enqueued on `stream` (a hipStream_t, NULL = default stream); nothing synchronises. `diag`: per-call
 * diagnostics (lgm_common.h), NULL = none.
 */
#ifndef LGM_ATTN_H
#define LGM_ATTN_H
#include <stddef.h>

#include "lgm_common.h"

#ifdef __cplusplus
extern "C" {
#endif

#define LGM_ATTN_F32 0
#define LGM_ATTN_BF16 1
#define LGM_ATTN_F16 2

/* Bytes of device scratch lgm_attn_backward needs: fp32: the delta = rowsum(dO * O) buffer; 16-bit dtypes: the
 * per-row constants the dQ pass hands to the dK/dV pass (-lse * log2(e) and -delta, rows padded to a multiple of 64)
 * and the rounded Q * scale * log2(e) rows (both passes recompute the forward's P from the same rounded operands). */
size_t lgm_attn_workspace_size(int dtype, int B, int L, int H, int D);

/* o = softmax(scale * q k^T) v per (batch, head); also writes lse. */
int lgm_attn_forward(int dtype, int B, int L, int H, int D, float scale, const void *q, const void *k,
                     const void *v, long long ld_qkv, void *o, float *lse, void *stream, const lgm_diag *diag);

/* dq, dk, dv of the forward above given d_o (o and lse from the forward). Overwrites dq/dk/dv. */
int lgm_attn_backward(int dtype, int B, int L, int H, int D, float scale, const void *q, const void *k,
                      const void *v, long long ld_qkv, const void *o, const float *lse, const void *d_o, void *dq,
                      void *dk, void *dv, long long ld_dqkv, void *workspace, size_t workspace_bytes, void *stream,
                      const lgm_diag *diag);

/* MVAttention's token layout around the core (core/unet.py:35-49), fused with its GroupNorm and residual.
 *
 * lgm_mva_norm_tokens: GroupNorm(x) (core/unet.py:40, nn.GroupNorm(groups, C, eps, affine); fp32 statistics,
 * biased variance) of x [B*F, C, HW] (NCHW, dtype_x) written in the token layout of core/unet.py:41-42,
 * tokens[b][f*HW + hw][c] (dtype_tok: what the qkv Linear consumes, bf16 under autocast). gamma/beta fp32 [C]
 * (NULL: 1/0). mean/rstd [B*F, groups] fp32 are saved for the backward (torch's native_group_norm_backward).
 * workspace: lgm_mva_workspace_size bytes of device scratch (per-chunk statistics; deterministic merge).
 * Replaces the GroupNorm module call + reshape/permute/reshape copy + autocast cast of the reference.
 *
 * lgm_mva_tokens_out: out[b*F+f][c][hw] = (y[b][f*HW + hw][c] + res[b*F+f][c][hw]) * skip (core/unet.py:45-48:
 * reshape/permute back, residual, skip_scale); res NULL: out = the permuted y. out is contiguous [B*F, C, HW]. */
size_t lgm_mva_workspace_size(int B, int F, int C, int HW, int groups); /* chunk statistics, bytes */
int lgm_mva_norm_tokens(int dtype_x, int dtype_tok, int B, int F, int C, int HW, int groups, float eps, const void *x,
                        const float *gamma, const float *beta, void *tokens, float *mean, float *rstd, void *workspace,
                        size_t workspace_bytes, void *stream, const lgm_diag *diag);
int lgm_mva_tokens_out(int dtype_y, int dtype_res, int dtype_out, int B, int F, int C, int HW, const void *y,
                       const void *res, float skip, void *out, void *stream, const lgm_diag *diag);

/* Backward of the two passes above (autograd through core/unet.py:40-48), replacing torch's permute copies, cast,
 * native_group_norm_backward and the residual's gradient sum:
 *
 * lgm_mva_tokens_out_backward: g = d_out * scale rounded to d_out's dtype (scale = skip_scale with a residual, 1
 * without: torch's `d_out * skip`); d_y [B, F*HW, C] (dtype_dy) = g in the token layout, and, if d_res is not NULL,
 * d_res [B*F, C, HW] (dtype_dres) = g.
 *
 * lgm_mva_norm_tokens_backward: the GroupNorm backward (torch's fused parameters: dx = rstd gamma dy + c2 x + c3 per
 * (sample, group); dgamma_c = sum_n (sum dy x - mean sum dy) rstd, dbeta_c = sum dy) of dy = d_tokens read back
 * from the token layout, with mean / rstd from lgm_mva_norm_tokens; dx [B*F, C, HW] (dtype_x) = that + d_res (the
 * residual's gradient, dtype_x, NULL = none) in one rounding. dx, dgamma, dbeta (fp32 [C]) may be NULL. Every sum is
 * in a fixed order (bitwise reproducible). Channels per group <= 256. workspace: lgm_mva_backward_workspace_size. */
size_t lgm_mva_backward_workspace_size(int B, int F, int C, int HW, int groups);
int lgm_mva_tokens_out_backward(int dtype_dout, int dtype_dy, int dtype_dres, int B, int F, int C, int HW,
                                const void *d_out, float scale, void *d_y, void *d_res, void *stream,
                                const lgm_diag *diag);
int lgm_mva_norm_tokens_backward(int dtype_x, int dtype_tok, int B, int F, int C, int HW, int groups, const void *x,
                                 const float *gamma, const float *mean, const float *rstd, const void *d_tokens,
                                 const void *d_res, void *dx, float *dgamma, float *dbeta, void *workspace,
                                 size_t workspace_bytes, void *stream, const lgm_diag *diag);

#ifdef __cplusplus
}
#endif
#endif
