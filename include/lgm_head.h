/*
 * lgm_head.h -- C ABI of the fused Gaussian head of LGM (liblgm_amd.so): the epilogue of LGM.forward_gaussians
 * (core/models.py:95-117) after the UNet, i.e.
 *     y = self.conv(x)                                   (1x1 conv 14 -> 14, core/models.py:34,96)
 *     y = y.reshape(B, V, 14, h, w).permute(0, 1, 3, 4, 2).reshape(B, V*h*w, 14)   (:98-107)
 *     gaussians = cat(clamp(y[:3], -1, 1), sigmoid(y[3]), 0.1 softplus(y[4:7]), F.normalize(y[7:11]),
 *                     0.5 tanh(y[11:]) + 0.5)            (:40-44, :109-115; F.normalize's default dim=1: over N)
 * as one pass over the UNet output (plus an in-place pass over the rotation columns for the per-object norm) that
 * writes the [B,N,14] fp32 Gaussians the renderer takes, and its backward (dL/dx, dL/dweight, dL/dbias) as two
 * passes plus a fixed-order reduction (deterministic).
 * The reference runs this as a cuDNN conv, a permute copy, five strided activation kernels and a cat.
 *
 * Conventions: DEVICE pointers, contiguous. dtype 0 = fp32, 1 = bf16 for x / dx (the UNet runs under bf16
 * autocast in training, core/options.py:89-104 mixed_precision='bf16'); weight [14,14] (the conv's [14,14,1,1]),
 * bias [14] (may be NULL: zero), gaussians / d_gaussians [B, V*h*w, 14] and d_weight / d_bias are fp32.
 * Returns 0 or a negative LGM_E* code (lgm_last_error()); stream-ordered, no host synchronisation; `diag`: per-call
 * diagnostics (lgm_common.h), NULL = none.
 */
#ifndef LGM_HEAD_H
#define LGM_HEAD_H
#include <stddef.h>

#include "lgm_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Scratch for the per-workgroup partial sums of the forward and the backward (same size for both). */
size_t lgm_gaussian_head_workspace_size(int B, int V, int h, int w);

/* x -> gaussians [B, N, 14]. rot_norm [B, 4] (may be NULL) receives the per-object column norms of the raw
 * rotation channels: the reference's rot_act is F.normalize with its default dim=1, i.e. over the N Gaussians of
 * the [B, N, 4] slice (core/models.py:43,112); the backward needs them. */
int lgm_gaussian_head_forward(int dtype, int B, int V, int h, int w, const void *x, const float *weight,
                              const float *bias, float *gaussians, float *rot_norm, void *workspace,
                              size_t workspace_bytes, void *stream, const lgm_diag *diag);

/* d_gaussians -> dx (x's dtype and layout, overwritten), d_weight [14,14] and d_bias [14] (overwritten; d_bias
 * may be NULL). rot_norm: the forward's. */
int lgm_gaussian_head_backward(int dtype, int B, int V, int h, int w, const void *x, const float *weight,
                               const float *bias, const float *rot_norm, const float *d_gaussians, void *dx,
                               float *d_weight, float *d_bias, void *workspace, size_t workspace_bytes,
                               void *stream, const lgm_diag *diag);

#ifdef __cplusplus
}
#endif
#endif
