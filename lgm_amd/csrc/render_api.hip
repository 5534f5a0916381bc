// lgm_amd/csrc/render_api.hip -- extern "C" entry points of include/lgm_render.h.
//
// lgm_render_forward  replaces the B*V calls of _C.rasterize_gaussians made by core/gs.py:73-85;
// lgm_render_backward replaces the B*V calls of _C.rasterize_gaussians_backward plus autograd's sum over views
// through the slices of core/gs.py:45-49. Kernels: render_bin.hip (preprocess, binning, sort) and
// render_raster.hip (compositing forward/backward, projection backward).
#include "render_common.h"

namespace {

int check_common(int B, int V, int N, int H, int W, const void *g, const void *cv, const void *cvp, float tanx,
                 float tany, float mod, lgm::Dims &d) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0 || H > lgm::BY * 65535 || W > lgm::BX * 65535) {
        lgm::set_error("invalid sizes (B=%d V=%d N=%d H=%d W=%d)", B, V, N, H, W);
        return LGM_E_INVALID;
    }
    if ((N > 0 && !g) || !cv || !cvp) {
        lgm::set_error("null input pointer");
        return LGM_E_INVALID;
    }
    if (!(tanx > 0.f) || !(tany > 0.f)) {
        lgm::set_error("tanfov must be positive");
        return LGM_E_INVALID;
    }
    d.B = B; d.V = V; d.N = N; d.H = H; d.W = W;
    d.gx = (W + lgm::BX - 1) / lgm::BX;
    d.gy = (H + lgm::BY - 1) / lgm::BY;
    d.T = d.gx * d.gy;
    d.BV = B * V;
    d.ck_shift = lgm::ck_shift_for((size_t)d.BV * d.T);
    d.tanx = tanx; d.tany = tany;
    d.fx = W / (2.0f * tanx);
    d.fy = H / (2.0f * tany);
    d.mod = mod;
    const lgm_diag *diag = lgm::call_diag();  // this call's diagnostics (DiagScope), or none
    d.counters = diag ? diag->render_counters : nullptr;
    d.det_lim_log2 = diag ? diag->det_limit_log2 : 0;
    d.options = 0;
    d.gt_img = d.gt_mask = nullptr;
    d.loss_part = d.loss_out = nullptr;
    d.d_loss = nullptr;
    return LGM_OK;
}

bool capacity_ok(long long cap) { return cap <= 0x7fffffffLL; }

// lgm_render_needle_flags: render_common.h rec_needle (the decision the binning and the backward's flush both take
// on a stored record) evaluated on caller-given (A', B', C')
__global__ __launch_bounds__(256) void k_needle_flags(long long n, const float *__restrict__ abc,
                                                      unsigned char *__restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    out[i] = lgm::rec_needle(abc[3 * i], abc[3 * i + 1], abc[3 * i + 2]) ? 1 : 0;
}

// Inspection kernels (lgm_render_tile_lists / lgm_render_pixel_state): plain copies out of the workspace.
__global__ __launch_bounds__(256) void k_tile_counts(int M, long long slot_stride, const int *__restrict__ tile_start,
                                                     const int *__restrict__ tile_count, int *__restrict__ out) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= M) return;
    long long base;
    int n;
    lgm::tile_range(t, slot_stride, tile_start, tile_count, base, n);
    out[t] = n;
}
// one workgroup per (view, tile): its sorted ids (u32, in place at the start of its pair range) -> ids_out
__global__ __launch_bounds__(256) void k_tile_ids(long long slot_stride, const int *__restrict__ tile_start,
                                                  const int *__restrict__ tile_count,
                                                  const unsigned long long *__restrict__ pairs,
                                                  const long long *__restrict__ offsets, unsigned *__restrict__ ids_out) {
    const int t = blockIdx.x;
    long long base;
    int n;
    lgm::tile_range(t, slot_stride, tile_start, tile_count, base, n);
    const unsigned *ids = reinterpret_cast<const unsigned *>(pairs + base);
    unsigned *dst = ids_out + offsets[t];
    for (int e = threadIdx.x; e < n; e += 256) dst[e] = ids[e];
}

int check_ws(int B, int V, int N, int H, int W, const void *ws, size_t ws_bytes, long long cap, lgm::Layout &L) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0) {
        lgm::set_error("invalid sizes (B=%d V=%d N=%d H=%d W=%d)", B, V, N, H, W);
        return LGM_E_INVALID;
    }
    L = lgm::make_layout(B, V, N, H, W, cap, false);
    if (!ws || ws_bytes < L.total) {
        lgm::set_error("workspace too small (%zu < %zu)", ws_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    return LGM_OK;
}

}  // namespace

extern "C" {

size_t lgm_render_workspace_size(int B, int V, int N, int H, int W, long long pair_capacity) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0) return 0;
    return lgm::make_layout(B, V, N, H, W, pair_capacity).total;
}

size_t lgm_render_workspace_size_opts(int B, int V, int N, int H, int W, long long pair_capacity, int options) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0) return 0;
    return lgm::make_layout(B, V, N, H, W, pair_capacity, (options & LGM_RENDER_DETERMINISTIC) != 0).total;
}

int lgm_render_count_pairs(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                           const float *cam_view_proj, float tanfovx, float tanfovy, float scale_modifier,
                           void *workspace, size_t workspace_bytes, long long *pairs_out, void *stream,
                           const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    lgm::Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, d);
    if (rc) return rc;
    if (!pairs_out) {
        lgm::set_error("null pairs_out");
        return LGM_E_INVALID;
    }
    const lgm::Layout L = lgm::make_layout(B, V, N, H, W, 1);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small for counting (%zu < %zu)", workspace_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    return lgm::launch_binning(d, gaussians, cam_view, cam_view_proj, (char *)workspace, L, nullptr, pairs_out,
                               true, (hipStream_t)stream);
}

}  // extern "C"

static int forward_impl(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                        const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                        float scale_modifier, float *image, float *depth, float *alpha, int *radii_out,
                        const float *gt_images, const float *gt_masks, float *loss_out, void *workspace,
                        size_t workspace_bytes, long long pair_capacity, long long *stats_out, int options,
                        void *stream, const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    lgm::Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, d);
    if (rc) return rc;
    if (!bg || !image || !depth || !alpha) {
        lgm::set_error("null output pointer");
        return LGM_E_INVALID;
    }
    const lgm::Layout L = lgm::make_layout(B, V, N, H, W, pair_capacity, (options & LGM_RENDER_DETERMINISTIC) != 0);
    if (!L.slot && !capacity_ok(L.cap)) {  // packed tile offsets are int32; slot offsets are 64-bit
        lgm::set_error("pair capacity %lld exceeds 2^31", L.cap);
        return LGM_E_INVALID;
    }
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small (%zu < %zu)", workspace_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    char *ws = (char *)workspace;
    d.options = options & ~LGM_RENDER_FUSED_LOSS;
    if (gt_images || gt_masks || loss_out) {
        if (!gt_images || !gt_masks || !loss_out) {
            lgm::set_error("fused loss needs gt_images, gt_masks and loss_out");
            return LGM_E_INVALID;
        }
        d.options |= LGM_RENDER_FUSED_LOSS;
        d.gt_img = gt_images;
        d.gt_mask = gt_masks;
        d.loss_part = (float *)(ws + L.lossp);
        d.loss_out = loss_out;
    }
    hipStream_t st = (hipStream_t)stream;
    rc = lgm::launch_binning(d, gaussians, cam_view, cam_view_proj, ws, L, radii_out, stats_out, false, st);
    if (rc) return rc;
    rc = lgm::launch_render_fwd(d, gaussians, bg, image, depth, alpha, ws, L, st);
    if (rc || !(d.options & LGM_RENDER_FUSED_LOSS)) return rc;
    return lgm::launch_loss_reduce(d, ws, L, st);
}

static int backward_impl(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                         const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                         float scale_modifier, const float *d_image, const float *d_depth, const float *d_alpha,
                         const float *gt_images, const float *gt_masks, const float *d_loss, float *d_gaussians,
                         float *d_means2D, void *workspace, size_t workspace_bytes, long long pair_capacity,
                         int options, void *stream, const lgm_diag *diag) {
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    lgm::Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, d);
    if (rc) return rc;
    if (!bg || (N > 0 && !d_gaussians)) {
        lgm::set_error("null pointer in backward");
        return LGM_E_INVALID;
    }
    const lgm::Layout L = lgm::make_layout(B, V, N, H, W, pair_capacity, (options & LGM_RENDER_DETERMINISTIC) != 0);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small (%zu < %zu)", workspace_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    if (N == 0) return LGM_OK;
    d.options = options & ~LGM_RENDER_FUSED_LOSS;
    if (gt_images || gt_masks || d_loss) {
        if (!gt_images || !gt_masks || !d_loss) {
            lgm::set_error("fused loss backward needs gt_images, gt_masks and d_loss");
            return LGM_E_INVALID;
        }
        d.options |= LGM_RENDER_FUSED_LOSS;
        d.gt_img = gt_images;
        d.gt_mask = gt_masks;
        d.d_loss = d_loss;
    }
    return lgm::launch_render_bwd(d, gaussians, cam_view, cam_view_proj, bg, d_image, d_depth, d_alpha, d_gaussians,
                                  d_means2D, (char *)workspace, L, (hipStream_t)stream);
}

extern "C" {

int lgm_render_forward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                       const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                       float scale_modifier, float *image, float *depth, float *alpha, int *radii_out,
                       void *workspace, size_t workspace_bytes, long long pair_capacity, long long *stats_out,
                       int options, void *stream, const lgm_diag *diag) {
    return forward_impl(B, V, N, H, W, gaussians, cam_view, cam_view_proj, bg, tanfovx, tanfovy, scale_modifier,
                        image, depth, alpha, radii_out, nullptr, nullptr, nullptr, workspace, workspace_bytes,
                        pair_capacity, stats_out, options, stream, diag);
}

int lgm_render_forward_loss(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                            const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                            float scale_modifier, float *image, float *depth, float *alpha, const float *gt_images,
                            const float *gt_masks, float *loss_out, void *workspace, size_t workspace_bytes,
                            long long pair_capacity, int options, void *stream, const lgm_diag *diag) {
    if (!gt_images || !gt_masks || !loss_out) {
        lgm::set_error("null gt_images / gt_masks / loss_out");
        return LGM_E_INVALID;
    }
    return forward_impl(B, V, N, H, W, gaussians, cam_view, cam_view_proj, bg, tanfovx, tanfovy, scale_modifier,
                        image, depth, alpha, nullptr, gt_images, gt_masks, loss_out, workspace, workspace_bytes,
                        pair_capacity, nullptr, options, stream, diag);
}

int lgm_render_backward_loss(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                             const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                             float scale_modifier, const float *d_image, const float *d_alpha,
                             const float *gt_images, const float *gt_masks, const float *d_loss,
                             float *d_gaussians, void *workspace, size_t workspace_bytes, long long pair_capacity,
                             int options, void *stream, const lgm_diag *diag) {
    if (!gt_images || !gt_masks || !d_loss) {
        lgm::set_error("null gt_images / gt_masks / d_loss");
        return LGM_E_INVALID;
    }
    return backward_impl(B, V, N, H, W, gaussians, cam_view, cam_view_proj, bg, tanfovx, tanfovy, scale_modifier,
                         d_image, nullptr, d_alpha, gt_images, gt_masks, d_loss, d_gaussians, nullptr, workspace,
                         workspace_bytes, pair_capacity, options, stream, diag);
}

int lgm_render_tile_lists(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                          long long pair_capacity, int *tile_counts_out, const long long *offsets,
                          unsigned *ids_out, void *stream) {
    lgm::clear_error();
    lgm::Layout L;
    int rc = check_ws(B, V, N, H, W, workspace, workspace_bytes, pair_capacity, L);
    if (rc) return rc;
    if (!tile_counts_out || (ids_out && !offsets)) {
        lgm::set_error("null tile_counts_out / offsets");
        return LGM_E_INVALID;
    }
    const int T = ((W + lgm::BX - 1) / lgm::BX) * ((H + lgm::BY - 1) / lgm::BY), M = B * V * T;
    const char *ws = (const char *)workspace;
    const long long stride = L.slot ? (long long)N : -1LL;
    const int *ts = (const int *)(ws + L.tile_start), *tc = (const int *)(ws + L.tile_count);
    hipStream_t st = (hipStream_t)stream;
    LGM_LAUNCH("k_tile_counts", st, (k_tile_counts<<<(M + 255) / 256, 256, 0, st>>>(M, stride, ts, tc, tile_counts_out)));
    if (ids_out && N > 0)
        LGM_LAUNCH("k_tile_ids", st, (k_tile_ids<<<M, 256, 0, st>>>(stride, ts, tc,
                                     (const unsigned long long *)(ws + L.pairs), offsets, ids_out)));
    return LGM_OK;
}

int lgm_render_pixel_state(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                           long long pair_capacity, int *n_contrib_out, float *final_T_out, void *stream) {
    lgm::clear_error();
    lgm::Layout L;
    int rc = check_ws(B, V, N, H, W, workspace, workspace_bytes, pair_capacity, L);
    if (rc) return rc;
    const size_t P = (size_t)B * V * H * W;
    const char *ws = (const char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    if (n_contrib_out && hipMemcpyAsync(n_contrib_out, ws + L.n_contrib, P * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) {
        lgm::set_error("hipMemcpyAsync failed");
        return LGM_E_HIP;
    }
    if (final_T_out && hipMemcpyAsync(final_T_out, ws + L.final_T, P * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) {
        lgm::set_error("hipMemcpyAsync failed");
        return LGM_E_HIP;
    }
    return LGM_OK;
}

int lgm_render_records(int B, int V, int N, int H, int W, const void *workspace, size_t workspace_bytes,
                       long long pair_capacity, float *P_out, float *Q_out, unsigned *rects_out, void *stream) {
    lgm::clear_error();
    lgm::Layout L;
    int rc = check_ws(B, V, N, H, W, workspace, workspace_bytes, pair_capacity, L);
    if (rc) return rc;
    const size_t BVN = (size_t)B * V * N;
    const char *ws = (const char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    const struct { void *dst; size_t off, bytes; } cp[3] = {
        {P_out, L.gP, BVN * 16}, {Q_out, L.gQ, BVN * 16}, {rects_out, L.rects, BVN * 8}};
    for (const auto &c : cp) {
        if (c.dst && c.bytes && hipMemcpyAsync(c.dst, ws + c.off, c.bytes, hipMemcpyDeviceToDevice, st) != hipSuccess) {
            lgm::set_error("hipMemcpyAsync failed");
            return LGM_E_HIP;
        }
    }
    return LGM_OK;
}

int lgm_render_needle_flags(long long n, const float *abc, unsigned char *flags_out, void *stream) {
    lgm::clear_error();
    if (n < 0 || (n > 0 && (!abc || !flags_out))) {
        lgm::set_error("invalid needle-flag arguments");
        return LGM_E_INVALID;
    }
    if (n == 0) return LGM_OK;
    hipStream_t st = (hipStream_t)stream;
    LGM_LAUNCH("k_needle_flags", st, (k_needle_flags<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(n, abc, flags_out)));
    return LGM_OK;
}

int lgm_render_det_flush_limit_log2(int views, int tiles, int scene_record) {
    lgm::clear_error();
    if (views <= 0 || tiles <= 0) {
        lgm::set_error("lgm_render_det_flush_limit_log2: views and tiles must be positive");
        return LGM_E_INVALID;
    }
    return lgm::det_flush_limit_log2(views, tiles, scene_record != 0);
}

int lgm_render_backward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                        const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                        float scale_modifier, const float *d_image, const float *d_depth, const float *d_alpha,
                        float *d_gaussians, float *d_means2D, void *workspace, size_t workspace_bytes,
                        long long pair_capacity, int options, void *stream, const lgm_diag *diag) {
    return backward_impl(B, V, N, H, W, gaussians, cam_view, cam_view_proj, bg, tanfovx, tanfovy, scale_modifier,
                         d_image, d_depth, d_alpha, nullptr, nullptr, nullptr, d_gaussians, d_means2D, workspace,
                         workspace_bytes, pair_capacity, options, stream, diag);
}

}  // extern "C"
