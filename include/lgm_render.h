/*
 * lgm_render.h -- C ABI of the MI355X-native Gaussian-splat render path (liblgm_amd.so).
 *
 * Replaces the external CUDA extension `diff_gaussian_rasterization._C` that LGM reaches through
 * core/gs.py:7-10 and calls once per (scene b, view v) at core/gs.py:58-85:
 *   - lgm_render_forward  replaces _C.rasterize_gaussians          (the per-view forward behind
 *                         GaussianRasterizer(...)(...) at core/gs.py:73-85), batched over all B x V views;
 *   - lgm_render_backward replaces _C.rasterize_gaussians_backward (driven by autograd from main.py:102
 *                         through the EXT autograd Function), batched likewise, and additionally performs the
 *                         sum over views + slice-gradient scatter that autograd does through the slices of
 *                         core/gs.py:45-49, writing dL/dgaussians [B,N,14] directly.
 * The Python side (lgm_amd/gs.py) keeps the reference's GaussianRenderer API (core/gs.py:16-98).
 *
 * Conventions (all pointers are DEVICE pointers unless stated; all arrays dense, row-major, fp32):
 *   gaussians      [B,N,14]  pos(3) opacity(1) scale(3) rotation(4: w,x,y,z) rgb(3)   (core/gs.py:45-49)
 *   cam_view       [B,V,4,4] the transposed w2c exactly as core/gs.py:54 passes it (read column-major)
 *   cam_view_proj  [B,V,4,4] likewise (core/gs.py:55)
 *   bg             [3]
 *   image          [B,V,3,H,W] unclamped, or clamp(0, 1) as core/gs.py:87 when options has LGM_RENDER_CLAMP_IMAGE
 *   depth, alpha   [B,V,1,H,W]
 * Error behaviour: every entry point returns 0 on success and a negative LGM_E* code on failure; it never
 * throws across the ABI. lgm_last_error() returns a thread-local description of the last failure.
 * Threading: stream-ordered (all work is enqueued on `stream`, a hipStream_t passed as void*), no host
 * synchronisation inside forward/backward, reentrant; no global mutable state other than the error string: every
 * behaviour switch is a per-call `options` bit and diagnostics are a per-call `diag` (lgm_common.h; NULL = none).
 * Memory: caller-owned. Scratch and saved-for-backward state live in ONE caller-allocated workspace whose size
 * is given by lgm_render_workspace_size(); the same workspace must be passed, untouched, to the backward.
 */
#ifndef LGM_RENDER_H
#define LGM_RENDER_H

#include <stddef.h>
#include <stdint.h>

#include "lgm_common.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Workspace bytes for B x V renders of N Gaussians at H x W. pair_capacity <= 0 selects SLOT mode: every tile owns
 * room for N pairs (B*V*N*tiles*8 bytes, no counting pass, no host sync). pair_capacity > 0 selects PACKED mode
 * with room for that many (Gaussian, tile) pairs in total (from lgm_render_count_pairs). */
size_t lgm_render_workspace_size(int B, int V, int N, int H, int W, long long pair_capacity);

/* Exact pair counts over all B x V views. Enqueues a counting pass and writes pairs_out (a DEVICE int64[2]):
 *   [0] pairs actually binned (upstream's 3-sigma tile rect minus tiles where alpha < 1/255 is provable for every
 *       pixel -- the capacity a packed workspace needs), [1] upstream's num_rendered summed over views.
 * Used by callers that cannot afford the slot workspace; they synchronise once, size the workspace from [0] and
 * call lgm_render_forward with that pair_capacity. */
int lgm_render_count_pairs(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                           const float *cam_view_proj, float tanfovx, float tanfovy, float scale_modifier,
                           void *workspace, size_t workspace_bytes, long long *pairs_out, void *stream,
                           const lgm_diag *diag);

/* Forward of all B x V renders (replaces B*V calls of _C.rasterize_gaussians). radii_out [B,V,N] int32 may be
 * NULL. stats_out, if not NULL, is a DEVICE int64[2] with the counts described at lgm_render_count_pairs. */
int lgm_render_forward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                       const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                       float scale_modifier, float *image, float *depth, float *alpha, int *radii_out,
                       void *workspace, size_t workspace_bytes, long long pair_capacity, long long *stats_out,
                       int options, void *stream, const lgm_diag *diag);

/* Backward of all B x V renders (replaces B*V calls of _C.rasterize_gaussians_backward plus the autograd sum
 * over views). d_image / d_depth / d_alpha may be NULL (treated as zero). Writes d_gaussians [B,N,14] (overwrites).
 * d_means2D [B,V,N,2] (screen-space gradients, what upstream returns for means2D) may be NULL. */
int lgm_render_backward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                        const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                        float scale_modifier, const float *d_image, const float *d_depth, const float *d_alpha,
                        float *d_gaussians, float *d_means2D, void *workspace, size_t workspace_bytes,
                        long long pair_capacity, int options, void *stream, const lgm_diag *diag);

/* Loss-fused variants for training (core/models.py:133-167): with gt_images [B,V,3,H,W] and gt_masks [B,V,1,H,W]
 * (DEVICE fp32), the forward also composites the ground truth over bg (gt * mask + bg * (1 - mask)) and writes
 * loss_out (DEVICE float[4]) = (loss_mse, mse_image, mse_alpha, psnr) with loss_mse = F.mse_loss(image, gt) +
 * F.mse_loss(alpha, mask) and psnr = -10 log10(mse_image) -- per-tile partial sums inside the compositing kernel,
 * one fixed-order reduction, no separate loss kernels. The backward seeds dL/dimage and dL/dalpha in-kernel from
 * d_loss (DEVICE float[2] = dL/dmse_image, dL/dmse_alpha; both equal dL/dloss_mse for the plain sum) and the same
 * ground truth: 2 (image - gt) d_loss[0] / numel(image) (image after the clamp when LGM_RENDER_CLAMP_IMAGE) and
 * 2 (alpha - mask) d_loss[1] / numel(alpha), plus the optional d_image / d_alpha of other losses on the same
 * outputs (e.g. LPIPS, core/models.py:150-158; NULL = none). Pass the same options to both. */
int lgm_render_forward_loss(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                            const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                            float scale_modifier, float *image, float *depth, float *alpha, const float *gt_images,
                            const float *gt_masks, float *loss_out, void *workspace, size_t workspace_bytes,
                            long long pair_capacity, int options, void *stream, const lgm_diag *diag);
int lgm_render_backward_loss(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                             const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                             float scale_modifier, const float *d_image, const float *d_alpha,
                             const float *gt_images, const float *gt_masks, const float *d_loss,
                             float *d_gaussians, void *workspace, size_t workspace_bytes, long long pair_capacity,
                             int options, void *stream, const lgm_diag *diag);

/* Inspection of the state a forward left in its workspace (the equivalent of upstream's saved binningBuffer /
 * imgBuffer: point_list + ranges, n_contrib, accum_alpha), for parity tests and debugging. Stream-ordered.
 * lgm_render_tile_lists: tile_counts_out (DEVICE int32 [B*V*T], T = ceil(W/16)*ceil(H/16), tile-major per view)
 * receives each (view, tile)'s list length; if ids_out is not NULL, the tile's Gaussian ids in compositing
 * (depth, then id) order are copied to ids_out[offsets[bv*T + t] ...] (offsets: DEVICE int64 [B*V*T], e.g. the
 * exclusive cumsum of the counts). Replaces reading point_list[ranges[t].x .. ranges[t].y) of the EXT.
 * lgm_render_pixel_state: per-pixel n_contrib (1 + list position of the last accepted entry) and final
 * transmittance, [B,V,H,W] each (DEVICE; either may be NULL). */
int lgm_render_tile_lists(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                          long long pair_capacity, int *tile_counts_out, const long long *offsets,
                          unsigned *ids_out, void *stream);
int lgm_render_pixel_state(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                           long long pair_capacity, int *n_contrib_out, float *final_T_out, void *stream);
/* lgm_render_records: the per-(view, Gaussian) compositing records the binning wrote (upstream's geomBuffer:
 * means2D, conic_opacity, depths, tile rects), DEVICE, each [B,V,N,...] and each may be NULL:
 *   P_out [4] = (x, y, A', B'), Q_out [4] = (C', log2 opacity, tau', depth) with the conic pre-scaled as
 *   A' = -log2(e)/2 A, B' = -log2(e) B, C' = -log2(e)/2 C (tau' likewise; render_common.h rec_p / rec_q);
 *   rects_out [2] u32 = (x0 | y0 << 16, x1 | y1 << 16 | needle << 31), needle = the record's conic partials are
 *   accumulated in fp64 (float mode). Invisible records: rects (0, 0). */
int lgm_render_records(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                       long long pair_capacity, float *P_out, float *Q_out, unsigned *rects_out, void *stream);
/* lgm_render_needle_flags: the float mode's needle decision (render_common.h rec_needle: conic condition
 * (A + C)^2 / (AC - B^2) above 300, or not positive definite; the record's conic partials then go to fp64
 * accumulators) evaluated on n caller-given DEVICE triples abc [n,3] = (A', B', C') as a record stores them ->
 * flags_out [n] (DEVICE u8, 1 = needle). The binning and the backward's flush take this same decision on the stored
 * record; a test pins it to separately rounded IEEE operations (no FP contraction) near the threshold. */
int lgm_render_needle_flags(long long n, const float *abc, unsigned char *flags_out, void *stream);
/* lgm_render_det_flush_limit_log2: LGM_RENDER_DETERMINISTIC's overflow bound, log2 of the largest |flush| (in
 * fixed-point units) the backward accepts into one int64 accumulator of a render with `views` views per scene and
 * `tiles` tiles per view: 62 - ceil(log2 F), F = the flushes one accumulator can take -- `tiles` for the per-view
 * records (mean2D, conic, depth), views * tiles for the per-scene ones (scene_record != 0: opacity, colour, summed
 * over the scene's views). Pure host function (no GPU); the kernel derives the same value. A flush above it is
 * counted and the call's gradients are poisoned with NaN. */
int lgm_render_det_flush_limit_log2(int views, int tiles, int scene_record);

/* Diagnostics: when diag->render_counters (a DEVICE uint64 buffer, caller-zeroed) is set, that call's render kernels
 * record per-workgroup timelines in it: [0..7] the backward's section cycles in the LGM_BWD_STAMPS diagnostic build (else unused);
 * then 8 entries per tile t (B*V*T tiles): s_memrealtime stamps (100 MHz) [8+8t] fwd start, [+1] fwd end,
 * [+2], [+3] the start / end of preprocess-backward workgroup t (t < its grid), [+4] sort start, [+5] sort end,
 * [+6] the tile's binned list length (low 32 bits; k_sort writes it, k_render_fwd rewrites it with the HW_ID of the
 * wave that composited the tile -- SE / CU / SIMD / slot -- in the high 32 bits), [+7] list entries the forward
 * staged (bits 0-31), wave 0's 4-entry steps (bits 32-55) and the XCC_ID of the XCD it ran on (bits 56-63); then 8
 * entries per binning workgroup
 * (room for B*V*ceil(N/512); the binning launch uses its first B*ceil(V/3)*ceil(N/512)): phase stamps [0] start,
 * [1] preprocessed, [2] tile tests done, [3] reserved, [4] end, [5] its binned pairs, [6] HW_ID and [7] XCC_ID of where it
 * ran; then 4 entries per backward work item (at most 3*B*V*tiles + 16 items: one per tile, rounded up to 8, and
 * one per checkpoint slot): start/end stamps, (entries | chunk << 20 | tile << 40) and (XCC_ID | HW_ID << 8) -- so the buffer
 * must hold 8 + 8*B*V*tiles + 8*B*V*ceil(N/512) + 4*(3*B*V*tiles + 16) entries. */

/* Per-call `options` of lgm_render_forward / lgm_render_backward (pass the same value to both).
 * LGM_RENDER_CLAMP_IMAGE: the forward writes clamp(image, 0, 1) (core/gs.py:87) and keeps a per-pixel mask in
 * the workspace; the backward passes d_image only where 0 <= unclamped <= 1 (torch's clamp gradient), so no
 * separate clamp kernels or unclamped copy are needed. */
#define LGM_RENDER_CLAMP_IMAGE 2
/* LGM_RENDER_BACKWARD_AGAIN (lgm_render_backward only): this workspace's forward has already been through a
 * backward (autograd with retain_graph): its gradient accumulators are cleared first. The forward's binning
 * zeroes them, so a first backward needs no clearing pass. */
#define LGM_RENDER_BACKWARD_AGAIN 4
/* (internal) set by lgm_render_forward_loss / lgm_render_backward_loss; ignored in `options`. */
#define LGM_RENDER_FUSED_LOSS 8
/* LGM_RENDER_DETERMINISTIC: bit-reproducible gradients. The per-view gradient accumulators become
 * int64 fixed point (integer atomics commute, so the sums do not depend on the order in which the backward's work
 * items finish) instead of fp32 float atomics. The units follow the data: 2^-30 of the call's largest per-pixel
 * seed |dL/dpixel| (found by one extra pass over the seeds), times per-(view, Gaussian) power-of-two normalisers of
 * the screen-space mean and conic partials -- so a mean-MSE loss's ~1e-9 seeds keep full resolution and large
 * footprints cannot overflow. The forward is deterministic in either mode. The workspace is larger: size it with
 * lgm_render_workspace_size_opts(..., options). Pass it to forward and backward alike. */
#define LGM_RENDER_DETERMINISTIC 16
size_t lgm_render_workspace_size_opts(int B, int V, int N, int H, int W, long long pair_capacity, int options);

/* LGM_RENDER_NO_CULL: bin upstream's full 3-sigma tile rects instead of dropping (Gaussian, tile) pairs where
 * alpha < 1/255 is provable for every pixel; outputs are identical either way
 * (tests/test_render_gpu.py::test_exact_culling_is_output_preserving), only the work differs. A packed workspace for
 * it needs lgm_render_count_pairs' pairs_out[1] (upstream's count) as its capacity. Per call, like every option. */
#define LGM_RENDER_NO_CULL 1

#ifdef __cplusplus
}
#endif
#endif
