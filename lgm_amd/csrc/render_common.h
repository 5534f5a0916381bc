// lgm_amd/csrc/render_common.h -- shared constants, workspace layout and device math of the render path.
//
// Numerics restate SURVEY.md §2.3 (the upstream algorithm behind core/gs.py:58-85; CPU restatement in
// oracle/raster_oracle.c): 0.3 dilation, 1.3 tanfov clamp inside J, depth cull 0.2, radius = ceil(3 sqrt(lmax))
// with max(0.1, mid^2 - det), ndc2Pix in double, integer tile-rect math, alpha cap 0.99 / floor 1/255,
// transmittance floor 1e-4 tested before accumulation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "lgm_render.h"

namespace lgm {

constexpr int BX = 16, BY = 16, TILE_PIX = BX * BY;  // 256 pixels per tile = 4 wavefronts (8x8 quadrants)
constexpr int NACC = 10;  // gradient partials per (view, Gaussian): mean2D(2) conic(3) opacity rgb(3) depth
// Accumulator layout (elements: fp32, or int64 fixed point in deterministic mode): the view-dependent partials
// (mean2D, conic, depth) per (view, Gaussian) in records of NACC_V, then the view-independent ones (opacity,
// colour) per (scene, Gaussian) in records of NACC_S -- the views of a scene add into one record, so the forward
// zeroes and k_preproc_bwd reads 24 + 16 / V bytes per (view, Gaussian) instead of 40.
constexpr int NACC_V = 6, NACC_S = 4;
__host__ __device__ __forceinline__ size_t acc_index(int q, size_t bvN_i, size_t bN_i, size_t BVN) {
    return q < 5 ? bvN_i * NACC_V + q : q < 9 ? BVN * NACC_V + bN_i * NACC_S + (q - 5) : bvN_i * NACC_V + 5;
}
__host__ __device__ inline size_t acc_elems(size_t B, size_t V, size_t N) { return B * V * N * NACC_V + B * N * NACC_S; }
// Float mode: the conic partials (q = 2..4) of NEEDLE records go to fp64 side accumulators, 3 per (view, Gaussian),
// placed after the fp32 ones (float offset acc_side_offset, 8-B aligned). A needle is a record whose conic
// condition (A + C)^2 / (AC - B^2) exceeds ACC_NEEDLE (or is not positive definite), decided on the
// stored record (rec_needle) identically by the binning, the backward's flush and the preprocess backward (via a
// flag in bit 31 of the record's rect).
__host__ __device__ inline size_t acc_side_offset(size_t B, size_t V, size_t N) { return (acc_elems(B, V, N) + 1) & ~(size_t)1; }
// Deterministic mode's per-flush overflow bound (k_render_bwd): in that mode an accumulator takes at most one flush
// per tile list its Gaussian appears in -- one work item per tile, an entry once per list. A per-view record (mean2D,
// conic, depth) sees the T tiles of its view; a per-scene record (opacity, colour: acc_index q = 5..8) the V * T
// tiles of all views of its scene. With every flush |a| <= 2^62 / 2^ceil(log2 flushes), no sum of them reaches 2^62,
// whatever their signs, so int64 cannot wrap. (The design value of a flush is <= ~2^51: DET_BITS below.)
__host__ __device__ inline int det_flush_limit_log2(int V, int T, bool scene_record) {
    const long long f = scene_record ? (long long)V * T : (long long)T;
    int c = 0;
    while ((1ll << c) < f) c++;  // ceil(log2 f)
    return 62 - c;
}
constexpr int LDS_HIST_MAX = 8192;                   // tiles per view for the LDS-histogram binning path
constexpr float LOG2E = 1.4426950408889634f;

inline size_t align_up(size_t x) { return (x + 255) & ~size_t(255); }
// Deterministic mode takes no backward checkpoints: one backward work item per tile, so how a tile's walk splits into
// work items cannot depend on which tiles won the shared pool's slot counters (a racing split changes the backward's
// per-chunk partials in their last bits). A per-tile checkpoint quota was measured (profiles/r03/ab_det):
// deterministic k_render_bwd 1950 / 1306 / 955 / 787 / 685 / 650 us at quota 16 / 8 / 4 / 2 / 1 / 0 (float mode
// 626) -- in the fixed-point mode the split costs more than its load balance returns.
// Float mode's gradient accumulators: fp32, and fp64 for the conic partials of needle-like records. A needle's conic
// partials from different tiles and views largely cancel and the cov2D inverse amplifies what is left (conditions
// 1e3-2e4), so fp32 atomic sums made its scale / rotation gradients a draw of the atomic order (single runs up to ~3x
// the fp32 oracle's error vs fp64 at 512^2, profiles/r03/diag_float_spread); fp64 sums of the same fp32 partials are
// order-independent to ~2^-50 of the partials (the deterministic mode's int64 sums are exact). Measured: all
// accumulators fp64 +37 us per pool step, the needle side accumulators +24 us (profiles/r03/ab_acc_side).
constexpr float ACC_NEEDLE = 300.0f;  // conic condition above which a record's conic partials are summed in fp64

// Workspace layout. Pair storage `pairs` holds one u64 key (depth_bits << 32 | gaussian id) per (Gaussian, tile)
// pair; after sorting, the tile's u32 ids are written in place at the start of its range.
//   slot mode   (pair_capacity <= 0): tile (bv, t) owns pairs[(bv*T + t) * N, +N): no counting pass, no scan.
//   packed mode (pair_capacity  > 0): tiles are packed by an exclusive scan of exact counts.
struct Layout {
    size_t gP, gQ, rects, tile_count, tile_start, order, pairs, final_T, n_contrib, wlast, cfin, ck, cklist, nck, cmask,
        accum, lossp, lossw, detmax, misc, total;
    long long cap;
    int ck_region;  // backward checkpoint slots per region (8 regions; the forward shards tiles over them)
    int ck_slots;   // checkpoint slots in all: 8 ck_region (none in deterministic mode)
    bool slot;
};

// det (LGM_RENDER_DETERMINISTIC): the per-view gradient accumulators are int64 fixed point (data-scaled units, see
// render_raster.hip det_norm) instead of fp32: integer atomics commute, so the backward's sums do not depend on the
// order of its work items.
// Backward work items span 2^ck_shift staged forward chunks (of TILE_PIX entries): 2 chunks for launches of at least
// CK_LONG_TILES tiles, where the many short checkpoint items run at the end of k_render_bwd at about half its slots
// (each workgroup hand-over idles a slot for a few us); one for smaller launches, whose head items already exceed
// one residency round. Pool (12,288 tiles): k_render_bwd 599 -> 588 us and k_render_fwd -6 us (fewer checkpoints);
// one cfg3 scene (1,536 tiles) with 2: bwd 92.7 -> 102.8 us (profiles/r06/ab_bwd_cks).
#ifndef LGM_CK_LONG_TILES
#define LGM_CK_LONG_TILES 4096
#endif
constexpr size_t CK_LONG_TILES = LGM_CK_LONG_TILES;
#ifdef LGM_CK_SHIFT0  // (A/B: one chunk per item at every size)
__host__ __device__ __forceinline__ int ck_shift_for(size_t) { return 0; }
#else
__host__ __device__ __forceinline__ int ck_shift_for(size_t tiles) { return tiles >= CK_LONG_TILES ? 1 : 0; }
#endif

inline Layout make_layout(int B, int V, int N, int H, int W, long long pair_capacity, bool det = false) {
    const size_t BV = (size_t)B * V, T = (size_t)((W + BX - 1) / BX) * ((H + BY - 1) / BY), P = (size_t)H * W;
    Layout L;
    L.slot = pair_capacity <= 0;
    L.cap = L.slot ? (long long)(BV * T * (size_t)N) : pair_capacity;
    size_t o = 0;
    auto take = [&](size_t bytes) { size_t r = o; o = align_up(o + bytes); return r; };
    L.gP = take(BV * N * 16);  // (x, y, A, B): centre and conic A, B (one 16-B row per (view, Gaussian))
    L.gQ = take(BV * N * 16);  // (C, opacity, tau, depth)
    L.rects = take(BV * N * 8);
    L.tile_count = take(BV * T * 4);
    L.misc = take(64);  // right after tile_count: the binning clears both with one memset (u64 [0..1]: pair
                        // counts of k_bin; u32 [4..11]: the backward-checkpoint region counters; u32 [12]: the
                        // fused loss reduction's arrival counter; u32 [13]: deterministic mode's saturated flushes)
    L.tile_start = take((BV * T + 1) * 4);
    L.order = take(T * 4);  // k_sort's centre-first tile table (center_order)
    L.pairs = take((size_t)L.cap * 8);
    L.final_T = take(BV * P * 4);
    L.n_contrib = take(BV * P * 4);
    L.wlast = take(BV * T * 16);  // per tile: the four waves' largest last contributor (forward -> backward)
    L.cfin = take(BV * P * 16);  // per-pixel pre-background colour and depth totals (forward -> backward)
    // backward checkpoints (k_render_fwd -> k_render_bwd), 5 planes of 256 floats each, in 8 regional pools (a
    // region is one eighth of the launch's tiles). k_render_bwd launches one workgroup per slot, and an unused slot's
    // workgroup still pays a dispatch and a counter round trip before it exits: at 2 slots per tile the pool (8 scenes,
    // ~0.53 used per tile) left 18k such workgroups and cost k_render_bwd ~15 us. A region holds min(2 per tile,
    // 0.75 per tile + 256): the 8-scene pool 1,408 per region (its busiest uses ~860), one cfg3 scene keeps 2 per
    // tile (384: its central regions need ~1 per tile), BASELINE config 2 keeps 64 (profiles/r06/ab_bwd_ckcap,
    // abfull_cap). A full region leaves the rest of a tile's walk to its last checkpointed item (slower, same result).
    L.ck_region = (int)std::min((2 * BV * T + 7) / 8, ((3 * BV * T / 4) >> ck_shift_for(BV * T)) / 8 + 1 + 256);
    L.ck_slots = det ? 0 : 8 * L.ck_region;
    L.ck = take((size_t)L.ck_slots * 5 * TILE_PIX * 4);
    L.cklist = take((size_t)L.ck_slots * 8);
    L.nck = take(BV * T * 4);
    L.cmask = take(BV * P);
    L.accum = take(det ? acc_elems(B, V, N) * 8 : acc_side_offset(B, V, N) * 4 + BV * N * 3 * 8);
    L.lossp = take(BV * T * 2 * 4);  // per-tile sums of squared image / alpha residuals (fused loss)
    L.lossw = take(((BV * T + 2047) / 2048) * 16);  // their per-workgroup double2 partials (k_loss_reduce)
    L.detmax = take(64 * 4);  // deterministic mode: max |dL/dpixel| over the seeds, in 64 atomicMax slots
    L.total = o;
    return L;
}

struct Dims {
    int B, V, N, H, W, gx, gy, T, BV;
    float tanx, tany, fx, fy, mod;
    unsigned long long *counters;  // this call's device work counters (lgm_diag.render_counters), or null
    int det_lim_log2;              // lgm_diag.det_limit_log2 (test hook; 0 = the derived bound)
    int options;                   // per-call LGM_RENDER_* bits (NO_CULL, CLAMP_IMAGE, FUSED_LOSS, DETERMINISTIC)
    int ck_shift;                  // backward work items span 2^ck_shift forward chunks (ck_shift_for(BV * T))
    // LGM_RENDER_FUSED_LOSS (core/models.py:138-160): ground truth [BV,3,P] / [BV,P], the per-tile loss partials
    // (forward) and the gradients of the two MSE terms (backward)
    const float *gt_img, *gt_mask;
    float *loss_part;  // workspace: per-tile (image, alpha) sums of squared residuals
    float *loss_out;   // DEVICE float[4]: loss_mse, mse_image, mse_alpha, psnr
    const float *d_loss;  // DEVICE float[2]: dL/dmse_image, dL/dmse_alpha
};

// ------------------------------------------------------------------------------------------------------------
// Camera helpers: the 4x4 matrices are the row-major torch tensors of core/gs.py:54-55 read column-major.
//
// Every helper of the forward preprocess runs with FP contraction OFF and in the oracle's operation order
// (oracle/raster_oracle.c: glm-order matrix products, left-to-right sums): the integer results derived from it
// -- radii, tile rects, (Gaussian, tile) pair counts and the depth sort keys -- are then bit-identical to the
// restatement (tests/test_render_parity_gpu.py), not merely close.
__device__ __forceinline__ void xf43(const float *M, float x, float y, float z, float o[3]) {
#pragma clang fp contract(off)
    o[0] = M[0] * x + M[4] * y + M[8] * z + M[12];
    o[1] = M[1] * x + M[5] * y + M[9] * z + M[13];
    o[2] = M[2] * x + M[6] * y + M[10] * z + M[14];
}
__device__ __forceinline__ void xf44(const float *M, float x, float y, float z, float o[4]) {
#pragma clang fp contract(off)
    o[0] = M[0] * x + M[4] * y + M[8] * z + M[12];
    o[1] = M[1] * x + M[5] * y + M[9] * z + M[13];
    o[2] = M[2] * x + M[6] * y + M[10] * z + M[14];
    o[3] = M[3] * x + M[7] * y + M[11] * z + M[15];
}

// glm-convention rotation matrix R[col][row] from the un-normalised quaternion (r,x,y,z) (upstream semantics).
__device__ __forceinline__ void quat_rot(const float q[4], float R[3][3]) {
#pragma clang fp contract(off)
    const float r = q[0], x = q[1], y = q[2], z = q[3];
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// Sigma = M^T M with M = S*R (glm): M[c][k] = s_k R[c][k], Sigma[c][r] = sum_k M[r][k] M[c][k] (the oracle's
// m3_mul order); stored (00,01,02,11,12,22).
__device__ __forceinline__ void cov3d(const float s[3], const float R[3][3], float c3[6]) {
#pragma clang fp contract(off)
    float M[3][3];
#pragma unroll
    for (int c = 0; c < 3; c++)
#pragma unroll
        for (int k = 0; k < 3; k++) M[c][k] = s[k] * R[c][k];
#define LGM_SIG(c, r) (M[r][0] * M[c][0] + M[r][1] * M[c][1] + M[r][2] * M[c][2])
    c3[0] = LGM_SIG(0, 0); c3[1] = LGM_SIG(0, 1); c3[2] = LGM_SIG(0, 2);
    c3[3] = LGM_SIG(1, 1); c3[4] = LGM_SIG(1, 2); c3[5] = LGM_SIG(2, 2);
#undef LGM_SIG
}

// The two non-zero glm columns of T = W*J (with the 1.3 tanfov clamp on t), SURVEY §2.3 row 1.
struct ProjCtx {
    float T0[3], T1[3];  // glm T[0][*], T[1][*]
    float t[3];          // clamped view-space mean
    float xmul, ymul;    // 0 where the clamp was active (gradient cut, as upstream)
};
__device__ __forceinline__ ProjCtx make_proj(const float *Vw, float mx, float my, float mz, float fx, float fy,
                                             float tanx, float tany) {
#pragma clang fp contract(off)
    ProjCtx P;
    xf43(Vw, mx, my, mz, P.t);
    const float limx = 1.3f * tanx, limy = 1.3f * tany;
    const float txtz = P.t[0] / P.t[2], tytz = P.t[1] / P.t[2];
    P.t[0] = fminf(limx, fmaxf(-limx, txtz)) * P.t[2];
    P.t[1] = fminf(limy, fmaxf(-limy, tytz)) * P.t[2];
    P.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    P.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float tz = P.t[2];
    const float J00 = fx / tz, J02 = -(fx * P.t[0]) / (tz * tz);
    const float J11 = fy / tz, J12 = -(fy * P.t[1]) / (tz * tz);
#pragma unroll
    for (int r = 0; r < 3; r++) {
        P.T0[r] = Vw[4 * r + 0] * J00 + Vw[4 * r + 2] * J02;
        P.T1[r] = Vw[4 * r + 1] * J11 + Vw[4 * r + 2] * J12;
    }
    return P;
}
// cov = T^T Sigma^T T (glm order, as the oracle's cov2d): with s0 = Sigma T0 and s1 = Sigma T1 (T0, T1 the
// non-zero columns of T), a = T0 . s0, b = T0 . s1, c = T1 . s1, each summed left to right.
__device__ __forceinline__ void cov2d(const ProjCtx &P, const float c3[6], float &a, float &b, float &c) {
#pragma clang fp contract(off)
    const float S[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float s0[3], s1[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        s0[k] = S[k][0] * P.T0[0] + S[k][1] * P.T0[1] + S[k][2] * P.T0[2];
        s1[k] = S[k][0] * P.T1[0] + S[k][1] * P.T1[1] + S[k][2] * P.T1[2];
    }
    a = P.T0[0] * s0[0] + P.T0[1] * s0[1] + P.T0[2] * s0[2] + 0.3f;
    b = s1[0] * P.T0[0] + s1[1] * P.T0[1] + s1[2] * P.T0[2];
    c = P.T1[0] * s1[0] + P.T1[1] * s1[1] + P.T1[2] * s1[2] + 0.3f;
}

__device__ __forceinline__ float ndc2pix(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// Can any integer pixel of [rx0, rx1] x [ry0, ry1] reach q = A dx^2 + 2B dx dy + C dy^2 <= tau around (x, y)?
// Exact minimum of the (convex) quadratic over the rectangle: 0 if the centre is inside, else the minimum over the
// four edges (1-D minimiser clamped to the edge). Conservative for the integer pixels it contains.
// invA = 1/A, invC = 1/C (precomputed once per Gaussian).
__device__ __forceinline__ bool ellipse_hits_rect(float x, float y, float A, float B, float C, float invA,
                                                  float invC, float tau, float rx0, float rx1, float ry0, float ry1) {
    if (tau >= 3.0e38f) return true;
    if (x >= rx0 && x <= rx1 && y >= ry0 && y <= ry1) return true;
    float best = 3.0e38f;
    const float ex[2] = {rx0, rx1}, ey[2] = {ry0, ry1};
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const float dx = x - ex[e];
        const float dy = fminf(fmaxf(-B * dx * invC, y - ry1), y - ry0);
        best = fminf(best, A * dx * dx + 2.f * B * dx * dy + C * dy * dy);
    }
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const float dy = y - ey[e];
        const float dx = fminf(fmaxf(-B * dy * invA, x - rx1), x - rx0);
        best = fminf(best, A * dx * dx + 2.f * B * dx * dy + C * dy * dy);
    }
    return best <= tau;
}

// Compositing records (k_bin -> k_render_fwd / k_render_bwd), two float4 per (view, Gaussian):
//   P = (x, y, A', B'),  Q = (C', L, tau', depth)
// with the conic pre-scaled so that one (entry, pixel) evaluation is 5 VALU + exp2:
//   power * log2(e) + log2(opacity) = A' dx^2 + B' dx dy + C' dy^2 + L,   alpha = min(0.99, exp2(that)),
//   A' = -KQ A, B' = -2 KQ B, C' = -KQ C (KQ = log2(e) / 2), L = log2(opacity) (-inf for opacity <= 0).
// Upstream's `power > 0` skip is `that > L`; dL/dG = opacity dL/dalpha uses exp2(that) = opacity G directly.
// The culling threshold tau (on q = A dx^2 + 2B dx dy + C dy^2) is stored as tau' = KQ tau, so the quadrant tests
// run ellipse_hits_rect on (-A', -B'/2, -C', tau') = KQ (A, B, C, tau): the same test scaled by a positive constant
// (within tau's inflation). tau >= 3e38 (never cull) is kept as is.
constexpr float KQ = 0.5f * LOG2E;
__device__ __forceinline__ float4 rec_p(float x, float y, float A, float B) {
    return make_float4(x, y, -KQ * A, -LOG2E * B);
}
__device__ __forceinline__ float4 rec_q(float C, float opacity, float tau, float depth) {
    return make_float4(-KQ * C, opacity > 0.f ? log2f(opacity) : -INFINITY, tau >= 3.0e38f ? tau : KQ * tau, depth);
}
// Needle-like record (see acc_side_offset): on the stored pre-scaled conic A', B', C' (the condition is
// scale-invariant: (A' + C')^2 / (A'C' - B'^2 / 4) = (A + C)^2 / (AC - B^2)).
// FP contraction OFF: k_bin evaluates it on the record still in registers (right after the multiplications that
// form A', B', C'), k_render_bwd on the record loaded back from memory; with contraction a fused multiply-add could
// round differently in one of them and flip the decision for a record at the threshold. Evaluated as
// separately rounded IEEE operations it is a pure function of the stored bits in both (tests/test_render_gpu.py
// test_needle_flag_is_a_function_of_the_stored_record).
__device__ __forceinline__ bool rec_needle(float Ap, float Bp, float Cp) {
#pragma clang fp contract(off)
    const float sac = Ap + Cp, dq = Ap * Cp - 0.25f * Bp * Bp;
    return !(sac * sac <= ACC_NEEDLE * dq);  // (dq <= 0 or NaN: flagged)
}
__device__ __forceinline__ bool rec_hits_rect(const float4 &p, const float4 &q, float rx0, float rx1, float ry0,
                                              float ry1) {
    const float A = -p.z, B = -0.5f * p.w, C = -q.x;
    return ellipse_hits_rect(p.x, p.y, A, B, C, 1.0f / A, 1.0f / C, q.z, rx0, rx1, ry0, ry1);
}
// the upstream conic and opacity back from a record (the backward's per-entry gradient conversion)
__device__ __forceinline__ void rec_conic(const float4 &p, const float4 &q, float &A, float &B, float &C, float &op) {
    A = p.z * (-1.0f / KQ);
    B = p.w * (-1.0f / LOG2E);
    C = q.x * (-1.0f / KQ);
    op = exp2f(q.y);
}

struct Geo {
    float x, y, depth, A, B, C, opacity;  // pixel centre, view depth, conic (A, B, C), opacity
    float hx, hy;                         // half-extents of the alpha >= 1/255 ellipse's bounding box (pixels)
    float tau;                            // inflated alpha >= 1/255 threshold on q (3e38: never cull)
    int x0, y0, x1, y1;                   // reference tile rect (3-sigma)
    int cx0, cy0, cx1, cy1;               // emitted tile rect: reference rect ∩ tiles the alpha ellipse can reach
    int radius;
};

// Per-Gaussian forward preprocess. Returns false if culled (radius 0 upstream).
//
// Exact opacity-aware tile culling: upstream keeps every tile of the 3-sigma rect, but a tile in which
// alpha = min(0.99, o exp(-q/2)) < 1/255 for every pixel is skipped by every pixel (`continue`), changing
// nothing but the internal contributor counter. alpha >= 1/255 <=> q <= tau = 2 ln(255 o); the ellipse
// {q <= tau} lies inside |dx| <= sqrt(tau a), |dy| <= sqrt(tau c) (a, c: the dilated 2D covariance), which
// bounds the candidate tiles; the emitter then keeps a tile only if ellipse_hits_rect() says some pixel of it
// can reach q <= tau. tau is inflated (below) so fp32 rounding of q can never re-admit a culled pixel.
__device__ __forceinline__ bool preprocess_one(const float *g, const float *Vw, const float *Pm, const Dims &d,
                                               Geo &o) {
#pragma clang fp contract(off)
    float hom[4], pv[3];
    xf44(Pm, g[0], g[1], g[2], hom);
    const float pw = 1.0f / (hom[3] + 0.0000001f);
    const float ppx = hom[0] * pw, ppy = hom[1] * pw;
    xf43(Vw, g[0], g[1], g[2], pv);
    if (pv[2] <= 0.2f) return false;
    float R[3][3];
    const float q[4] = {g[7], g[8], g[9], g[10]};
    quat_rot(q, R);
    const float s[3] = {d.mod * g[4], d.mod * g[5], d.mod * g[6]};
    float c3[6];
    cov3d(s, R, c3);
    const ProjCtx P = make_proj(Vw, g[0], g[1], g[2], d.fx, d.fy, d.tanx, d.tany);
    float a, b, c;
    cov2d(P, c3, a, b, c);
    const float det = a * c - b * b;
    if (det == 0.0f) return false;
    const float det_inv = 1.f / det;
    const float mid = 0.5f * (a + c);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    const float px = ndc2pix(ppx, d.W), py = ndc2pix(ppy, d.H);
    const int r = (int)rad;
    const int x0 = min(d.gx, max(0, (int)((px - r) / BX)));
    const int y0 = min(d.gy, max(0, (int)((py - r) / BY)));
    const int x1 = min(d.gx, max(0, (int)((px + r + BX - 1) / BX)));
    const int y1 = min(d.gy, max(0, (int)((py + r + BY - 1) / BY)));
    if ((x1 - x0) * (y1 - y0) == 0) return false;
    o.x = px; o.y = py; o.depth = pv[2];
    o.A = c * det_inv; o.B = -b * det_inv; o.C = a * det_inv;
    o.opacity = g[3];
    o.x0 = x0; o.y0 = y0; o.x1 = x1; o.y1 = y1; o.radius = r;
    // --- exact opacity-aware cull of the emitted rect
    const float op = g[3];
    if (d.options & LGM_RENDER_NO_CULL) {
        o.hx = o.hy = 3.0e38f;
        o.tau = 3.0e38f;
        o.cx0 = x0; o.cx1 = x1; o.cy0 = y0; o.cy1 = y1;
        return true;
    }
    if (!(op * 255.0f > 1.0f)) {  // o <= 1/255: alpha < 1/255 everywhere (and NaN-safe)
        o.hx = o.hy = -1.f;
        o.tau = -1.f;
        o.cx0 = o.cx1 = x0; o.cy0 = o.cy1 = y0;
        return true;
    }
    // fp32 evaluation of q = A dx^2 + 2B dx dy + C dy^2 loses ~eps * kappa relative accuracy on elongated
    // ellipses; cond = (a + c)^2 / det ~ kappa. Inflate tau by 1e-3 + 2e-5 * cond (>= 80x the rounding bound) and
    // do not cull ill-conditioned or non-positive-definite ones at all (keep upstream's full rect).
    const float cond = (a + c) * (a + c) * __builtin_amdgcn_rcpf(det);  // (a threshold: 1 ulp is immaterial)
    if (!(det > 0.f) || !(cond < 4e4f)) {
        o.hx = o.hy = 3.0e38f;
        o.tau = 3.0e38f;
        o.cx0 = x0; o.cx1 = x1; o.cy0 = y0; o.cy1 = y1;
        return true;
    }
    // 2 ln(255 o) by v_log_f32 (log2, ~1 ulp): the 1e-3 inflation dwarfs it
    const float tau = (2.0f * 0.6931471805599453f) * __builtin_amdgcn_logf(255.0f * op) * (1.001f + 2e-5f * cond) + 1e-3f;
    o.tau = tau;
    o.hx = sqrtf(tau * fmaxf(a, 0.f));
    o.hy = sqrtf(tau * fmaxf(c, 0.f));
    const float lx = fmaxf(-1.0f, fminf((float)d.gx, (px - o.hx - (BX - 1)) / BX));
    const float hxt = fmaxf(-1.0f, fminf((float)d.gx, (px + o.hx) / BX));
    const float ly = fmaxf(-1.0f, fminf((float)d.gy, (py - o.hy - (BY - 1)) / BY));
    const float hyt = fmaxf(-1.0f, fminf((float)d.gy, (py + o.hy) / BY));
    o.cx0 = max(x0, (int)ceilf(lx));
    o.cx1 = min(x1, (int)floorf(hxt) + 1);
    o.cy0 = max(y0, (int)ceilf(ly));
    o.cy1 = min(y1, (int)floorf(hyt) + 1);
    if (o.cx1 < o.cx0) o.cx1 = o.cx0;
    if (o.cy1 < o.cy0) o.cy1 = o.cy0;
    return true;
}

__device__ __forceinline__ void load_gaussian(const float *__restrict__ src, float g[14]) {
    // rows are 56 B, always 8-B aligned: 7 x dwordx2
    const float2 *p = reinterpret_cast<const float2 *>(src);
#pragma unroll
    for (int k = 0; k < 7; k++) {
        const float2 v = p[k];
        g[2 * k] = v.x;
        g[2 * k + 1] = v.y;
    }
}

// Tile bucket of one (view, tile): base offset into `pairs` and entry count.
// slot_stride < 0 selects packed mode; slot mode uses stride N (possibly 0: then every bucket is empty).
__device__ __forceinline__ void tile_range(int tile, long long slot_stride, const int *__restrict__ tile_start,
                                           const int *__restrict__ tile_count, long long &base, int &n) {
    if (slot_stride >= 0) {
        base = (long long)tile * slot_stride;
        n = tile_count[tile];
    } else {
        base = tile_start[tile];
        n = tile_start[tile + 1] - tile_start[tile];
    }
}

// XCD-grouped work order of the (view, tile) items (sort and both compositing kernels). Workgroups are dealt
// round-robin over the 8 XCDs (MI355X_MICROARCH.md: blocks b and b + 8 share an XCD and its 4 MB L2), so block b
// takes item xcd_item(b): the blocks of group g = b % 8 walk one contiguous eighth of the items, in (view, tile)
// order, and neighbouring tiles -- which gather mostly the same Gaussians -- run on one L2 at about the same time.
// (The previous LPT order dealt neighbouring tiles to all eight L2s: 5-17 % L2 hit rates in the compositing
// kernels.) Bijective on [0, M) for any M (group sizes q + 1 for g < r, else q). Speed only, never correctness.
__host__ __device__ __forceinline__ int xcd_item(int b, int M) {
    const int q = M >> 3, r = M & 7, g = b & 7, i = b >> 3;
    return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}
__host__ __device__ __forceinline__ int xcd_group(int t, int M) {  // the block group (b % 8) that runs item t
    const int q = M >> 3, r = M & 7;
    return t < r * (q + 1) ? t / (q + 1) : r + (t - r * (q + 1)) / (q > 0 ? q : 1);
}
__host__ __device__ __forceinline__ int round8(int x) { return (x + 7) & ~7; }

// Pixel of thread t inside a 16x16 tile: wavefront w owns the 8x8 quadrant (w & 1, w >> 1).
__device__ __forceinline__ void tile_pixel(int t, int &lx, int &ly) {
    const int w = t >> 6, l = t & 63;
    lx = ((w & 1) << 3) + (l & 7);
    ly = ((w >> 1) << 3) + (l >> 3);
}

// ---- host launchers (defined in render_bin.hip / render_raster.hip)
int launch_binning(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                   char *ws, const Layout &L, int *radii_out, long long *stats_out, bool count_only,
                   hipStream_t st);
int launch_render_fwd(const Dims &d, const float *gaussians, const float *bg, float *image, float *depth,
                      float *alpha, char *ws, const Layout &L, hipStream_t st);
// the fused loss's final reduction (after launch_render_fwd with LGM_RENDER_FUSED_LOSS): d.loss_out receives
// (loss_mse, mse_image, mse_alpha, psnr)
int launch_loss_reduce(const Dims &d, char *ws, const Layout &L, hipStream_t st);
int launch_render_bwd(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                      const float *bg, const float *d_image, const float *d_depth, const float *d_alpha,
                      float *d_gaussians, float *d_means2D, char *ws, const Layout &L, hipStream_t st);

}  // namespace lgm
