/*
 * lgm_linear.h -- C ABI of the weight-gradient GEMM of MVAttention's Linears in liblgm_amd.so (lgm_amd/csrc/wgrad.hip).
 *
 * Replaces the weight / bias part of autograd through nn.Linear for the qkv and proj projections of
 * core/attention.py:46,48 (MemEffAttention, called at :75 and :82 inside core/unet.py:35-49 MVAttention) under
 * accelerate's bf16 (or fp16) autocast: torch's `grad_weight = grad_out^T @ input` (a K-long reduction over every token
 * of the batch, K = B * num_frames * h * w) and `grad_bias = grad_out.sum(0)`. The input gradient (grad_out @ weight)
 * and the forward stay on the library GEMM.
 *
 *   dw[m][n] = sum_k dy[k][m] * x[k][n]     (fp32, [M][N] contiguous: M = out_features, N = in_features)
 *   db[m]    = sum_k dy[k][m]               (fp32 [M]; db NULL: not computed)
 *
 * dy: [K][M] rows ld_dy elements apart; x: [K][N] rows ld_x apart; dtype LGM_ATTN_BF16 or LGM_ATTN_F16 (lgm_attn.h
 * codes), both tensors of that type. Products are exact and accumulated in fp32 (MFMA), so dw / db are the fp32 sums of
 * the 16-bit operands -- torch rounds its bf16 weight gradient to bf16 before the cast back to the fp32 parameter.
 * Every sum runs in a fixed order (bitwise reproducible). M, N, ld_dy, ld_x must be multiples of 8 and dy / x 16-byte
 * aligned. workspace: lgm_linear_wgrad_workspace_size bytes of device scratch (fp32 split-K partials), any contents.
 * Enqueued on `stream`; nothing synchronises.
 */
#ifndef LGM_LINEAR_H
#define LGM_LINEAR_H
#include <stddef.h>

#include "lgm_common.h"

#ifdef __cplusplus
extern "C" {
#endif

size_t lgm_linear_wgrad_workspace_size(int K, int M, int N, int want_db);
int lgm_linear_wgrad(int dtype, int K, int M, int N, const void *dy, long long ld_dy, const void *x, long long ld_x,
                     float *dw, float *db, void *workspace, size_t workspace_bytes, void *stream, const lgm_diag *diag);

#ifdef __cplusplus
}
#endif
#endif
