// lgm_amd/csrc/render_api.hip -- extern "C" entry points of include/lgm_render.h.
//
// lgm_render_forward  replaces the B*V calls of _C.rasterize_gaussians made by core/gs.py:73-85;
// lgm_render_backward replaces the B*V calls of _C.rasterize_gaussians_backward plus autograd's sum over views
// through the slices of core/gs.py:45-49. Kernels: render_bin.hip (preprocess, binning, sort) and
// render_raster.hip (compositing forward/backward, projection backward).
#include "render_common.h"

namespace {

// Diagnostic work counters (lgm_render_debug_counters) and option flags (lgm_render_set_flags): process-wide.
unsigned long long *g_counters = nullptr;
int g_flags = 0;

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
    d.tanx = tanx; d.tany = tany;
    d.fx = W / (2.0f * tanx);
    d.fy = H / (2.0f * tany);
    d.mod = mod;
    d.counters = g_counters;
    d.flags = g_flags;
    d.options = 0;
    return LGM_OK;
}

bool capacity_ok(long long cap) { return cap <= 0x7fffffffLL; }

}  // namespace

extern "C" {

int lgm_render_debug_counters(unsigned long long *device_counters) {
    g_counters = device_counters;
    return LGM_OK;
}

int lgm_render_set_flags(int flags) {
    g_flags = flags;
    return LGM_OK;
}

size_t lgm_render_workspace_size(int B, int V, int N, int H, int W, long long pair_capacity) {
    if (B <= 0 || V <= 0 || N < 0 || H <= 0 || W <= 0) return 0;
    return lgm::make_layout(B, V, N, H, W, pair_capacity).total;
}

int lgm_render_count_pairs(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                           const float *cam_view_proj, float tanfovx, float tanfovy, float scale_modifier,
                           void *workspace, size_t workspace_bytes, long long *pairs_out, void *stream) {
    lgm::clear_error();
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

int lgm_render_forward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                       const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                       float scale_modifier, float *image, float *depth, float *alpha, int *radii_out,
                       void *workspace, size_t workspace_bytes, long long pair_capacity, long long *stats_out,
                       int options, void *stream) {
    lgm::clear_error();
    lgm::Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, d);
    if (rc) return rc;
    if (!bg || !image || !depth || !alpha) {
        lgm::set_error("null output pointer");
        return LGM_E_INVALID;
    }
    const lgm::Layout L = lgm::make_layout(B, V, N, H, W, pair_capacity);
    if (!capacity_ok(L.cap)) {
        lgm::set_error("pair capacity %lld exceeds 2^31; use lgm_render_count_pairs + an exact capacity", L.cap);
        return LGM_E_INVALID;
    }
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small (%zu < %zu)", workspace_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    d.options = options;
    char *ws = (char *)workspace;
    hipStream_t st = (hipStream_t)stream;
    rc = lgm::launch_binning(d, gaussians, cam_view, cam_view_proj, ws, L, radii_out, stats_out, false, st);
    if (rc) return rc;
    return lgm::launch_render_fwd(d, gaussians, bg, image, depth, alpha, ws, L, st);
}

int lgm_render_backward(int B, int V, int N, int H, int W, const float *gaussians, const float *cam_view,
                        const float *cam_view_proj, const float *bg, float tanfovx, float tanfovy,
                        float scale_modifier, const float *d_image, const float *d_depth, const float *d_alpha,
                        float *d_gaussians, float *d_means2D, void *workspace, size_t workspace_bytes,
                        long long pair_capacity, int options, void *stream) {
    lgm::clear_error();
    lgm::Dims d;
    int rc = check_common(B, V, N, H, W, gaussians, cam_view, cam_view_proj, tanfovx, tanfovy, scale_modifier, d);
    if (rc) return rc;
    if (!bg || !d_image || (N > 0 && !d_gaussians)) {
        lgm::set_error("null pointer in backward");
        return LGM_E_INVALID;
    }
    const lgm::Layout L = lgm::make_layout(B, V, N, H, W, pair_capacity);
    if (!workspace || workspace_bytes < L.total) {
        lgm::set_error("workspace too small (%zu < %zu)", workspace_bytes, L.total);
        return LGM_E_WORKSPACE;
    }
    if (N == 0) return LGM_OK;
    d.options = options;
    return lgm::launch_render_bwd(d, gaussians, cam_view, cam_view_proj, bg, d_image, d_depth, d_alpha, d_gaussians,
                                  d_means2D, (char *)workspace, L, (hipStream_t)stream);
}

}  // extern "C"
