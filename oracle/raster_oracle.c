/*
 * oracle/raster_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, fp32 arithmetic, sequential per-pixel compositing) of the differentiable
 * Gaussian rasterizer that LGM calls through `diff_gaussian_rasterization` at core/gs.py:58-85.
 * That rasterizer is an EXTERNAL dependency (ashawkey fork of graphdeco-inria/diff-gaussian-rasterization,
 * installed from git HEAD with no pinned commit: readme.md:13-15) whose source is absent from
 * /root/reference and from this container. This file restates its published algorithm as written out in
 * SURVEY.md §2.3 (preprocess -> tile binning -> stable depth sort -> front-to-back compositing; reverse
 * compositing gradient -> cov2D backward -> preprocess backward).
 *
 * PARITY UNPINNED: the reference ships no tests, fixtures or golden vectors for the rasterizer
 * (SURVEY.md §4, §8c), and the rasterizer cannot be built or run here. This restatement is pinned only by
 * (a) closed-form known-answer cases (single Gaussian, tests/test_oracle.py), (b) float64 autograd of a
 * differentiable restatement of the same forward (oracle/raster_autograd.py), and (c) the committed golden
 * fixtures generated from it (tests/golden/make_golden.py).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library. The product
 * path (lgm_amd/) never links or calls it.
 *
 * Deliberate, documented deviations from upstream (see DESIGN.md §"Parity notes"):
 *   - dL/dscale is the exact derivative w.r.t. `scale` (includes the scale_modifier factor); identical to
 *     upstream at scale_modifier = 1, the only value training uses (core/gs.py:31, core/models.py:141).
 *   - dL/dmean3D from dL/ddepth uses the exact row (view[2], view[6], view[10]); identical to upstream for
 *     every affine view matrix (view[3] = view[7] = view[11] = 0), which is all LGM ever passes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Arithmetic type: fp32 by default (the restatement); -DLGM_ORACLE_F64 builds the same algorithm in fp64 (the
 * "truth" used to judge fp32 rounding noise on ill-conditioned Gaussians; API pointers become double*). */
#ifdef LGM_ORACLE_F64
typedef double real;
#define expf exp
#define sqrtf sqrt
#define fminf fmin
#define fmaxf fmax
#define ceilf ceil
#else
typedef float real;
#endif

#define BLOCK_X 16
#define BLOCK_Y 16

#include <omp.h>

/* Threads over the Gaussians / tiles of ONE view (preprocess, per-tile sort, render_fwd / render_bwd), nested
 * inside the batch's threads over views, for the CPU baseline on all host cores (bench.py cpu_baseline).
 * 1 (default) keeps the sequential order. The backward then accumulates into per-thread double records, summed in
 * thread order. */
static int g_tile_threads = 1;
void lgm_oracle_set_tile_threads(int n) { g_tile_threads = n > 1 ? n : 1; }

/* ---------- small glm-style helpers (glm mat3 is column-major: m[col][row]) ---------- */
typedef struct { real m[3][3]; } mat3;

static mat3 m3_mul(const mat3 *A, const mat3 *B) { /* glm A*B: R[c][r] = sum_k A[k][r]*B[c][k] */
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++)
            R.m[c][r] = A->m[0][r] * B->m[c][0] + A->m[1][r] * B->m[c][1] + A->m[2][r] * B->m[c][2];
    return R;
}
static mat3 m3_T(const mat3 *A) {
    mat3 R;
    for (int c = 0; c < 3; c++)
        for (int r = 0; r < 3; r++) R.m[c][r] = A->m[r][c];
    return R;
}
static mat3 m3_cols(real a0, real a1, real a2, real b0, real b1, real b2, real c0, real c1, real c2) {
    mat3 R;
    R.m[0][0] = a0; R.m[0][1] = a1; R.m[0][2] = a2;
    R.m[1][0] = b0; R.m[1][1] = b1; R.m[1][2] = b2;
    R.m[2][0] = c0; R.m[2][1] = c1; R.m[2][2] = c2;
    return R;
}

/* column-major 4x4 (the transposed torch matrices of core/gs.py:54-55) */
static void xform4x3(const real *M, const real p[3], real o[3]) {
    o[0] = M[0] * p[0] + M[4] * p[1] + M[8] * p[2] + M[12];
    o[1] = M[1] * p[0] + M[5] * p[1] + M[9] * p[2] + M[13];
    o[2] = M[2] * p[0] + M[6] * p[1] + M[10] * p[2] + M[14];
}
static void xform4x4(const real *M, const real p[3], real o[4]) {
    o[0] = M[0] * p[0] + M[4] * p[1] + M[8] * p[2] + M[12];
    o[1] = M[1] * p[0] + M[5] * p[1] + M[9] * p[2] + M[13];
    o[2] = M[2] * p[0] + M[6] * p[1] + M[10] * p[2] + M[14];
    o[3] = M[3] * p[0] + M[7] * p[1] + M[11] * p[2] + M[15];
}
static real ndc2pix(real v, int S) { return (real)((((double)v + 1.0) * S - 1.0) * 0.5); }
static int imin(int a, int b) { return a < b ? a : b; }
static int imax(int a, int b) { return a > b ? a : b; }
static void get_rect(real px, real py, int r, int gx, int gy, int mn[2], int mx[2]) {
    mn[0] = imin(gx, imax(0, (int)((px - r) / BLOCK_X)));
    mn[1] = imin(gy, imax(0, (int)((py - r) / BLOCK_Y)));
    mx[0] = imin(gx, imax(0, (int)((px + r + BLOCK_X - 1) / BLOCK_X)));
    mx[1] = imin(gy, imax(0, (int)((py + r + BLOCK_Y - 1) / BLOCK_Y)));
}

/* quaternion (r,x,y,z) -> glm rotation matrix, un-normalised as upstream */
static mat3 quat_R(const real *q) {
    real r = q[0], x = q[1], y = q[2], z = q[3];
    return m3_cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                   2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                   2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
}

static void cov3d(const real *s, real mod, const real *q, real out[6]) {
    mat3 S = m3_cols(mod * s[0], 0, 0, 0, mod * s[1], 0, 0, 0, mod * s[2]);
    mat3 R = quat_R(q);
    mat3 M = m3_mul(&S, &R);
    mat3 Mt = m3_T(&M);
    mat3 Sig = m3_mul(&Mt, &M);
    out[0] = Sig.m[0][0]; out[1] = Sig.m[0][1]; out[2] = Sig.m[0][2];
    out[3] = Sig.m[1][1]; out[4] = Sig.m[1][2]; out[5] = Sig.m[2][2];
}

/* W*J with the 1.3*tanfov clamp; returns T (glm) and the clamped t */
typedef struct { mat3 T, W; real t[3]; real xmul, ymul; } proj_ctx;

static proj_ctx make_proj(const real *mean, real fx, real fy, real tanx, real tany, const real *view) {
    proj_ctx P;
    xform4x3(view, mean, P.t);
    const real limx = 1.3f * tanx, limy = 1.3f * tany;
    const real txtz = P.t[0] / P.t[2], tytz = P.t[1] / P.t[2];
    P.t[0] = fminf(limx, fmaxf(-limx, txtz)) * P.t[2];
    P.t[1] = fminf(limy, fmaxf(-limy, tytz)) * P.t[2];
    P.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    P.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const real tz = P.t[2];
    mat3 J = m3_cols(fx / tz, 0.0f, -(fx * P.t[0]) / (tz * tz), 0.0f, fy / tz, -(fy * P.t[1]) / (tz * tz), 0, 0, 0);
    P.W = m3_cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    P.T = m3_mul(&P.W, &J);
    return P;
}

static void cov2d(const proj_ctx *P, const real *c3, real out[3]) {
    mat3 V = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
    mat3 Tt = m3_T(&P->T), Vt = m3_T(&V);
    mat3 A = m3_mul(&Tt, &Vt);
    mat3 C = m3_mul(&A, &P->T);
    C.m[0][0] += 0.3f;
    C.m[1][1] += 0.3f;
    out[0] = C.m[0][0]; out[1] = C.m[0][1]; out[2] = C.m[1][1];
}

/* ---------- per-view state ---------- */
typedef struct {
    int N, H, W, gx, gy;
    real fx, fy, tanx, tany, mod;
    const real *g; /* [N,14] */
    const real *view, *proj;
    int *radii;
    real *xy;     /* [N,2] */
    real *depth;  /* [N] */
    real *conic;  /* [N,4] conic.x, conic.y, conic.z, opacity */
    real *cov3;   /* [N,6] */
    int *rect;     /* [N,4] */
    uint64_t *keys;
    int *tile_start; /* [gx*gy+1] */
    real *final_T;
    int *n_contrib;
    long long K;
} view_state;

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : (x > y ? 1 : 0);
}

static void preprocess(view_state *S) {
#pragma omp parallel for schedule(static, 256) num_threads(g_tile_threads)
    for (int i = 0; i < S->N; i++) {
        const real *gi = S->g + 14 * (size_t)i;
        S->radii[i] = 0;
        S->rect[4 * i + 0] = S->rect[4 * i + 1] = S->rect[4 * i + 2] = S->rect[4 * i + 3] = 0;
        real hom[4], pv[3];
        xform4x4(S->proj, gi, hom);
        const real pw = 1.0f / (hom[3] + 0.0000001f);
        const real ppx = hom[0] * pw, ppy = hom[1] * pw;
        xform4x3(S->view, gi, pv);
        if (pv[2] <= 0.2f) continue; /* near cull */
        cov3d(gi + 4, S->mod, gi + 7, S->cov3 + 6 * (size_t)i);
        proj_ctx P = make_proj(gi, S->fx, S->fy, S->tanx, S->tany, S->view);
        real cv[3];
        cov2d(&P, S->cov3 + 6 * (size_t)i, cv);
        const real det = cv[0] * cv[2] - cv[1] * cv[1];
        if (det == 0.0f) continue;
        const real det_inv = 1.f / det;
        const real mid = 0.5f * (cv[0] + cv[2]);
        const real l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
        const real l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
        const real rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
        const real px = ndc2pix(ppx, S->W), py = ndc2pix(ppy, S->H);
        int mn[2], mx[2];
        get_rect(px, py, (int)rad, S->gx, S->gy, mn, mx);
        if ((mx[0] - mn[0]) * (mx[1] - mn[1]) == 0) continue;
        S->depth[i] = pv[2];
        S->radii[i] = (int)rad;
        S->xy[2 * i] = px;
        S->xy[2 * i + 1] = py;
        S->conic[4 * i + 0] = cv[2] * det_inv;
        S->conic[4 * i + 1] = -cv[1] * det_inv;
        S->conic[4 * i + 2] = cv[0] * det_inv;
        S->conic[4 * i + 3] = gi[3];
        S->rect[4 * i + 0] = mn[0]; S->rect[4 * i + 1] = mn[1];
        S->rect[4 * i + 2] = mx[0]; S->rect[4 * i + 3] = mx[1];
    }
}

/* bin + sort: tile lists ordered by (depth bits, gaussian index) == upstream stable LSD radix sort on
 * (tile << 32 | depth bits) applied to pairs emitted in gaussian-index order. */
static void bin_and_sort(view_state *S) {
    const int T = S->gx * S->gy;
    int *cnt = (int *)calloc((size_t)T + 1, sizeof(int));
    long long K = 0;
    for (int i = 0; i < S->N; i++) {
        if (S->radii[i] <= 0) continue;
        const int *r = S->rect + 4 * (size_t)i;
        for (int y = r[1]; y < r[3]; y++)
            for (int x = r[0]; x < r[2]; x++) { cnt[y * S->gx + x]++; K++; }
    }
    S->K = K;
    S->tile_start[0] = 0;
    for (int t = 0; t < T; t++) S->tile_start[t + 1] = S->tile_start[t] + cnt[t];
    S->keys = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(K > 0 ? K : 1));
    memset(cnt, 0, sizeof(int) * (size_t)T);
    for (int i = 0; i < S->N; i++) {
        if (S->radii[i] <= 0) continue;
        uint32_t db;
        const float fdepth = (float)S->depth[i]; /* fp32 depth bits, as upstream's sort key */
        memcpy(&db, &fdepth, 4);
        const int *r = S->rect + 4 * (size_t)i;
        for (int y = r[1]; y < r[3]; y++)
            for (int x = r[0]; x < r[2]; x++) {
                const int t = y * S->gx + x;
                S->keys[S->tile_start[t] + cnt[t]++] = ((uint64_t)db << 32) | (uint32_t)i;
            }
    }
#pragma omp parallel for schedule(dynamic, 4) num_threads(g_tile_threads)
    for (int t = 0; t < T; t++)
        qsort(S->keys + S->tile_start[t], (size_t)(S->tile_start[t + 1] - S->tile_start[t]), sizeof(uint64_t), cmp_u64);
    free(cnt);
}

static void render_fwd(view_state *S, const real *bg, real *out_color, real *out_depth, real *out_alpha,
                       long long *evals) {
    const int H = S->H, W = S->W;
    long long ev = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(g_tile_threads) reduction(+ : ev)
    for (int t = 0; t < S->gx * S->gy; t++) {
        {
            const int tx = t % S->gx, ty = t / S->gx;
            const int s0 = S->tile_start[t], s1 = S->tile_start[t + 1];
            for (int ly = 0; ly < BLOCK_Y; ly++)
                for (int lx = 0; lx < BLOCK_X; lx++) {
                    const int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= W || py >= H) continue;
                    const real pfx = (real)px, pfy = (real)py;
                    real T = 1.0f, C[3] = {0, 0, 0}, D = 0.f;
                    int contributor = 0, last = 0;
                    for (int j = s0; j < s1; j++) {
                        const int gi = (int)(uint32_t)S->keys[j];
                        contributor++;
                        ev++;
                        const real *co = S->conic + 4 * (size_t)gi;
                        const real dx = S->xy[2 * gi] - pfx, dy = S->xy[2 * gi + 1] - pfy;
                        const real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const real alpha = fminf(0.99f, co[3] * expf(power));
                        if (alpha < 1.0f / 255.0f) continue;
                        const real test_T = T * (1 - alpha);
                        if (test_T < 0.0001f) break;
                        const real *col = S->g + 14 * (size_t)gi + 11;
                        for (int ch = 0; ch < 3; ch++) C[ch] += col[ch] * alpha * T;
                        D += S->depth[gi] * alpha * T;
                        T = test_T;
                        last = contributor;
                    }
                    const int pid = W * py + px;
                    S->final_T[pid] = T;
                    S->n_contrib[pid] = last;
                    for (int ch = 0; ch < 3; ch++) out_color[(size_t)ch * H * W + pid] = C[ch] + T * bg[ch];
                    out_depth[pid] = D;
                    out_alpha[pid] = 1 - T;
                }
        }
    }
    if (evals) *evals += ev;
}

/* per-Gaussian 2D gradient accumulators (double) */
typedef struct { double m2[2], con[3], op, col[3], dep; } g2d;

static void render_bwd(view_state *S, const real *bg, const real *dLdc, const real *dLdd, const real *dLda,
                       g2d *acc_out) {
    const int H = S->H, W = S->W;
    const real ddelx_dx = (real)(0.5 * W), ddely_dy = (real)(0.5 * H);
    const int nthr = g_tile_threads;
    g2d *accs = acc_out;
    if (nthr > 1) {
        accs = (g2d *)calloc((size_t)nthr * (S->N > 0 ? S->N : 1), sizeof(g2d));
        if (!accs) { accs = acc_out; }
    }
#pragma omp parallel for schedule(dynamic, 1) num_threads(accs == acc_out ? 1 : nthr)
    for (int t = 0; t < S->gx * S->gy; t++) {
        g2d *acc = accs == acc_out ? acc_out : accs + (size_t)omp_get_thread_num() * S->N;
        {
            const int tx = t % S->gx, ty = t / S->gx;
            const int s0 = S->tile_start[t];
            for (int ly = 0; ly < BLOCK_Y; ly++)
                for (int lx = 0; lx < BLOCK_X; lx++) {
                    const int px = tx * BLOCK_X + lx, py = ty * BLOCK_Y + ly;
                    if (px >= W || py >= H) continue;
                    const int pid = W * py + px;
                    const real pfx = (real)px, pfy = (real)py;
                    const real T_final = S->final_T[pid];
                    real T = T_final;
                    const int last = S->n_contrib[pid];
                    real dpix[3], accum_rec[3] = {0, 0, 0}, last_color[3] = {0, 0, 0};
                    for (int ch = 0; ch < 3; ch++) dpix[ch] = dLdc[(size_t)ch * H * W + pid];
                    const real dpix_d = dLdd ? dLdd[pid] : 0.f;
                    const real dpix_a = dLda ? dLda[pid] : 0.f;
                    real accum_d = 0, accum_a = 0, last_alpha = 0, last_depth = 0;
                    real bg_dot = 0;
                    for (int ch = 0; ch < 3; ch++) bg_dot += bg[ch] * dpix[ch];
                    for (int j = s0 + last - 1; j >= s0; j--) {
                        const int gi = (int)(uint32_t)S->keys[j];
                        const real *co = S->conic + 4 * (size_t)gi;
                        const real dx = S->xy[2 * gi] - pfx, dy = S->xy[2 * gi + 1] - pfy;
                        const real power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                        if (power > 0.0f) continue;
                        const real G = expf(power);
                        const real alpha = fminf(0.99f, co[3] * G);
                        if (alpha < 1.0f / 255.0f) continue;
                        T = T / (1.f - alpha);
                        const real dchannel_dcolor = alpha * T;
                        real dL_dopa = 0.0f;
                        const real *col = S->g + 14 * (size_t)gi + 11;
                        g2d *A = acc + gi;
                        for (int ch = 0; ch < 3; ch++) {
                            const real c = col[ch];
                            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
                            last_color[ch] = c;
                            dL_dopa += (c - accum_rec[ch]) * dpix[ch];
                            A->col[ch] += dchannel_dcolor * dpix[ch];
                        }
                        const real c_d = S->depth[gi];
                        accum_d = last_alpha * last_depth + (1.f - last_alpha) * accum_d;
                        last_depth = c_d;
                        dL_dopa += (c_d - accum_d) * dpix_d;
                        A->dep += dchannel_dcolor * dpix_d;
                        accum_a = last_alpha + (1.f - last_alpha) * accum_a;
                        dL_dopa += (1 - accum_a) * dpix_a;
                        dL_dopa *= T;
                        last_alpha = alpha;
                        dL_dopa += (-T_final / (1.f - alpha)) * bg_dot;
                        const real dL_dG = co[3] * dL_dopa;
                        const real gdx = G * dx, gdy = G * dy;
                        const real dG_ddelx = -gdx * co[0] - gdy * co[1];
                        const real dG_ddely = -gdy * co[2] - gdx * co[1];
                        A->m2[0] += dL_dG * dG_ddelx * ddelx_dx;
                        A->m2[1] += dL_dG * dG_ddely * ddely_dy;
                        A->con[0] += -0.5f * gdx * dx * dL_dG;
                        A->con[1] += -0.5f * gdx * dy * dL_dG;
                        A->con[2] += -0.5f * gdy * dy * dL_dG;
                        A->op += G * dL_dopa;
                    }
                }
        }
    }
    if (accs != acc_out) {
        for (int k = 0; k < nthr; k++) {
            const g2d *a = accs + (size_t)k * S->N;
            for (int i = 0; i < S->N; i++) {
                g2d *o = acc_out + i;
                o->m2[0] += a[i].m2[0]; o->m2[1] += a[i].m2[1];
                o->con[0] += a[i].con[0]; o->con[1] += a[i].con[1]; o->con[2] += a[i].con[2];
                o->op += a[i].op;
                o->col[0] += a[i].col[0]; o->col[1] += a[i].col[1]; o->col[2] += a[i].col[2];
                o->dep += a[i].dep;
            }
        }
        free(accs);
    }
}

/* cov2D backward + projection backward + cov3D backward */
static void preprocess_bwd(view_state *S, const g2d *acc, real *dLdg, real *dmean2d_out) {
    for (int i = 0; i < S->N; i++) {
        if (S->radii[i] <= 0) continue;
        const real *gi = S->g + 14 * (size_t)i;
        const g2d *A = acc + i;
        real *o = dLdg + 14 * (size_t)i;
        const real dcon[3] = {(real)A->con[0], (real)A->con[1], (real)A->con[2]};
        const real dm2[2] = {(real)A->m2[0], (real)A->m2[1]};
        if (dmean2d_out) { dmean2d_out[2 * i] += dm2[0]; dmean2d_out[2 * i + 1] += dm2[1]; }
        /* --- computeCov2D backward --- */
        const real *c3 = S->cov3 + 6 * (size_t)i;
        proj_ctx P = make_proj(gi, S->fx, S->fy, S->tanx, S->tany, S->view);
        mat3 V = m3_cols(c3[0], c3[1], c3[2], c3[1], c3[3], c3[4], c3[2], c3[4], c3[5]);
        const mat3 *T = &P.T;
        const mat3 *Wm = &P.W;
        real cv[3];
        cov2d(&P, c3, cv);
        const real a = cv[0], b = cv[1], c = cv[2];
        const real denom = a * c - b * b;
        real dL_da = 0, dL_db = 0, dL_dc = 0;
        const real denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
        real dcov[6] = {0, 0, 0, 0, 0, 0};
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dcon[0] + 2 * b * c * dcon[1] + (denom - a * c) * dcon[2]);
            dL_dc = denom2inv * (-a * a * dcon[2] + 2 * a * b * dcon[1] + (denom - a * c) * dcon[0]);
            dL_db = denom2inv * 2 * (b * c * dcon[0] - (denom + 2 * b * b) * dcon[1] + a * b * dcon[2]);
            const real (*t)[3] = T->m;
            dcov[0] = (t[0][0] * t[0][0] * dL_da + t[0][0] * t[1][0] * dL_db + t[1][0] * t[1][0] * dL_dc);
            dcov[3] = (t[0][1] * t[0][1] * dL_da + t[0][1] * t[1][1] * dL_db + t[1][1] * t[1][1] * dL_dc);
            dcov[5] = (t[0][2] * t[0][2] * dL_da + t[0][2] * t[1][2] * dL_db + t[1][2] * t[1][2] * dL_dc);
            dcov[1] = 2 * t[0][0] * t[0][1] * dL_da + (t[0][0] * t[1][1] + t[0][1] * t[1][0]) * dL_db + 2 * t[1][0] * t[1][1] * dL_dc;
            dcov[2] = 2 * t[0][0] * t[0][2] * dL_da + (t[0][0] * t[1][2] + t[0][2] * t[1][0]) * dL_db + 2 * t[1][0] * t[1][2] * dL_dc;
            dcov[4] = 2 * t[0][2] * t[0][1] * dL_da + (t[0][1] * t[1][2] + t[0][2] * t[1][1]) * dL_db + 2 * t[1][1] * t[1][2] * dL_dc;
        }
        const real (*t)[3] = T->m;
        const real (*v)[3] = V.m;
        /* dL/dT rows 0,1 (glm columns 0,1 of T) */
        real dT0[3], dT1[3];
        for (int k = 0; k < 3; k++) {
            const real s0 = t[0][0] * v[k][0] + t[0][1] * v[k][1] + t[0][2] * v[k][2];
            const real s1 = t[1][0] * v[k][0] + t[1][1] * v[k][1] + t[1][2] * v[k][2];
            dT0[k] = 2 * s0 * dL_da + s1 * dL_db;
            dT1[k] = 2 * s1 * dL_dc + s0 * dL_db;
        }
        const real (*w)[3] = Wm->m;
        const real dJ00 = w[0][0] * dT0[0] + w[0][1] * dT0[1] + w[0][2] * dT0[2];
        const real dJ02 = w[2][0] * dT0[0] + w[2][1] * dT0[1] + w[2][2] * dT0[2];
        const real dJ11 = w[1][0] * dT1[0] + w[1][1] * dT1[1] + w[1][2] * dT1[2];
        const real dJ12 = w[2][0] * dT1[0] + w[2][1] * dT1[1] + w[2][2] * dT1[2];
        const real tz = 1.f / P.t[2], tz2 = tz * tz, tz3 = tz2 * tz;
        const real hx = S->fx, hy = S->fy;
        const real dtx = P.xmul * -hx * tz2 * dJ02;
        const real dty = P.ymul * -hy * tz2 * dJ12;
        const real dtz = -hx * tz2 * dJ00 - hy * tz2 * dJ11 + (2 * hx * P.t[0]) * tz3 * dJ02 + (2 * hy * P.t[1]) * tz3 * dJ12;
        const real *vm = S->view;
        real dmean[3] = {vm[0] * dtx + vm[1] * dty + vm[2] * dtz,
                          vm[4] * dtx + vm[5] * dty + vm[6] * dtz,
                          vm[8] * dtx + vm[9] * dty + vm[10] * dtz};
        /* --- projection (perspective divide) backward --- */
        const real *pm = S->proj;
        real hom[4];
        xform4x4(pm, gi, hom);
        const real m_w = 1.0f / (hom[3] + 0.0000001f);
        const real mul1 = (pm[0] * gi[0] + pm[4] * gi[1] + pm[8] * gi[2] + pm[12]) * m_w * m_w;
        const real mul2 = (pm[1] * gi[0] + pm[5] * gi[1] + pm[9] * gi[2] + pm[13]) * m_w * m_w;
        dmean[0] += (pm[0] * m_w - pm[3] * mul1) * dm2[0] + (pm[1] * m_w - pm[3] * mul2) * dm2[1];
        dmean[1] += (pm[4] * m_w - pm[7] * mul1) * dm2[0] + (pm[5] * m_w - pm[7] * mul2) * dm2[1];
        dmean[2] += (pm[8] * m_w - pm[11] * mul1) * dm2[0] + (pm[9] * m_w - pm[11] * mul2) * dm2[1];
        /* --- depth backward (exact row of the view matrix) --- */
        const real ddep = (real)A->dep;
        dmean[0] += vm[2] * ddep;
        dmean[1] += vm[6] * ddep;
        dmean[2] += vm[10] * ddep;
        /* --- cov3D backward --- */
        const real *q = gi + 7;
        const real r = q[0], x = q[1], y = q[2], z = q[3];
        mat3 R = quat_R(q);
        const real sm[3] = {S->mod * gi[4], S->mod * gi[5], S->mod * gi[6]};
        mat3 Sd = m3_cols(sm[0], 0, 0, 0, sm[1], 0, 0, 0, sm[2]);
        mat3 M = m3_mul(&Sd, &R);
        mat3 dSig = m3_cols(dcov[0], 0.5f * dcov[1], 0.5f * dcov[2], 0.5f * dcov[1], dcov[3], 0.5f * dcov[4],
                            0.5f * dcov[2], 0.5f * dcov[4], dcov[5]);
        mat3 MdS = m3_mul(&M, &dSig);
        mat3 dM;
        for (int cc = 0; cc < 3; cc++)
            for (int rr = 0; rr < 3; rr++) dM.m[cc][rr] = 2.0f * MdS.m[cc][rr];
        mat3 Rt = m3_T(&R), dMt = m3_T(&dM);
        real dscale[3];
        for (int k = 0; k < 3; k++)
            dscale[k] = (Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1] + Rt.m[k][2] * dMt.m[k][2]) * S->mod;
        for (int k = 0; k < 3; k++)
            for (int rr = 0; rr < 3; rr++) dMt.m[k][rr] *= sm[k];
        const real (*d)[3] = dMt.m;
        real dq[4];
        dq[0] = 2 * z * (d[0][1] - d[1][0]) + 2 * y * (d[2][0] - d[0][2]) + 2 * x * (d[1][2] - d[2][1]);
        dq[1] = 2 * y * (d[1][0] + d[0][1]) + 2 * z * (d[2][0] + d[0][2]) + 2 * r * (d[1][2] - d[2][1]) - 4 * x * (d[2][2] + d[1][1]);
        dq[2] = 2 * x * (d[1][0] + d[0][1]) + 2 * r * (d[2][0] - d[0][2]) + 2 * z * (d[1][2] + d[2][1]) - 4 * y * (d[2][2] + d[0][0]);
        dq[3] = 2 * r * (d[0][1] - d[1][0]) + 2 * x * (d[2][0] + d[0][2]) + 2 * y * (d[1][2] + d[2][1]) - 4 * z * (d[1][1] + d[0][0]);
        o[0] += dmean[0]; o[1] += dmean[1]; o[2] += dmean[2];
        o[3] += (real)A->op;
        o[4] += dscale[0]; o[5] += dscale[1]; o[6] += dscale[2];
        o[7] += dq[0]; o[8] += dq[1]; o[9] += dq[2]; o[10] += dq[3];
        o[11] += (real)A->col[0]; o[12] += (real)A->col[1]; o[13] += (real)A->col[2];
    }
}

/*
 * One rasterizer call for one (scene, view): the per-(b, v) body of core/gs.py:45-85.
 *   g [N,14] fp32 (pos 0:3, opacity 3, scale 4:7, rot(w,x,y,z) 7:11, rgb 11:14; core/gs.py:45-49)
 *   view/proj: 16 floats each, the row-major torch cam_view / cam_view_proj (read column-major)
 *   outputs: color [3,H,W] (NOT clamped; the clamp is core/gs.py:87's, applied by the caller), depth [H,W],
 *            alpha [H,W], radii [N] (optional), stats[0] = K (num_rendered), stats[1] = pixel-Gaussian evaluations.
 *   backward (optional; dLdc != NULL): accumulates (+=) dL/dg [N,14] and dL/dmeans2D [N,2] (optional).
 * Returns 0 on success, -1 on allocation failure.
 */
int lgm_oracle_render_view(int N, const real *g, const real *view, const real *proj, real tanfovx,
                           real tanfovy, real scale_modifier, const real *bg, int H, int W, real *out_color,
                           real *out_depth, real *out_alpha, int *radii_out, long long *stats,
                           const real *dLdc, const real *dLdd, const real *dLda, real *dLdg,
                           real *dmean2d_out) {
    view_state S;
    memset(&S, 0, sizeof(S));
    S.N = N; S.H = H; S.W = W;
    S.gx = (W + BLOCK_X - 1) / BLOCK_X;
    S.gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    S.tanx = tanfovx; S.tany = tanfovy;
    S.fy = H / (2.0f * tanfovy);
    S.fx = W / (2.0f * tanfovx);
    S.mod = scale_modifier;
    S.g = g; S.view = view; S.proj = proj;
    const size_t n = N > 0 ? (size_t)N : 1;
    S.radii = (int *)calloc(n, sizeof(int));
    S.xy = (real *)calloc(2 * n, sizeof(real));
    S.depth = (real *)calloc(n, sizeof(real));
    S.conic = (real *)calloc(4 * n, sizeof(real));
    S.cov3 = (real *)calloc(6 * n, sizeof(real));
    S.rect = (int *)calloc(4 * n, sizeof(int));
    S.tile_start = (int *)calloc((size_t)S.gx * S.gy + 1, sizeof(int));
    S.final_T = (real *)calloc((size_t)H * W, sizeof(real));
    S.n_contrib = (int *)calloc((size_t)H * W, sizeof(int));
    if (!S.radii || !S.xy || !S.depth || !S.conic || !S.cov3 || !S.rect || !S.tile_start || !S.final_T || !S.n_contrib)
        return -1;
    preprocess(&S);
    bin_and_sort(&S);
    long long ev = 0;
    render_fwd(&S, bg, out_color, out_depth, out_alpha, &ev);
    if (radii_out) memcpy(radii_out, S.radii, sizeof(int) * (size_t)N);
    if (stats) { stats[0] = S.K; stats[1] = ev; }
    if (dLdc && dLdg) {
        g2d *acc = (g2d *)calloc(n, sizeof(g2d));
        if (!acc) return -1;
        render_bwd(&S, bg, dLdc, dLdd, dLda, acc);
        preprocess_bwd(&S, acc, dLdg, dmean2d_out);
        free(acc);
    }
    free(S.radii); free(S.xy); free(S.depth); free(S.conic); free(S.cov3); free(S.rect);
    free(S.tile_start); free(S.final_T); free(S.n_contrib); free(S.keys);
    return 0;
}

/*
 * Batched form of core/gs.py:42-93: B scenes x V views, views parallel over OpenMP threads.
 *   g [B,N,14]; view/proj [B,V,16]; bg [3]; color [B,V,3,H,W]; depth/alpha [B,V,1,H,W].
 *   dLdg [B,N,14] (zeroed and filled when dLdc != NULL): sum over views of each scene, as autograd does
 *   through the per-b slices of core/gs.py:45-49.
 */
int lgm_oracle_render_batch(int B, int V, int N, const real *g, const real *views, const real *projs,
                            real tanfovx, real tanfovy, real scale_modifier, const real *bg, int H, int W,
                            real *color, real *depth, real *alpha, long long *stats, const real *dLdc,
                            const real *dLdd, const real *dLda, real *dLdg, int nthreads) {
    const size_t P = (size_t)H * W;
    const int BV = B * V;
    real *tmp = NULL;
    if (dLdc) {
        tmp = (real *)calloc((size_t)BV * N * 14 + 1, sizeof(real));
        if (!tmp) return -1;
    }
    int err = 0;
    long long st[2] = {0, 0};
    if (g_tile_threads > 1) omp_set_max_active_levels(2);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : err)
    for (int bv = 0; bv < BV; bv++) {
        const int b = bv / V;
        long long s[2] = {0, 0};
        err += lgm_oracle_render_view(N, g + (size_t)b * N * 14, views + 16 * (size_t)bv, projs + 16 * (size_t)bv,
                                      tanfovx, tanfovy, scale_modifier, bg, H, W, color + 3 * P * bv,
                                      depth + P * bv, alpha + P * bv, NULL, s,
                                      dLdc ? dLdc + 3 * P * bv : NULL, dLdd ? dLdd + P * bv : NULL,
                                      dLda ? dLda + P * bv : NULL, tmp ? tmp + (size_t)bv * N * 14 : NULL, NULL);
#pragma omp critical
        { st[0] += s[0]; st[1] += s[1]; }
    }
    if (stats) { stats[0] = st[0]; stats[1] = st[1]; }
    if (dLdc) {
        memset(dLdg, 0, sizeof(real) * (size_t)B * N * 14);
        for (int bv = 0; bv < BV; bv++) {
            real *dst = dLdg + (size_t)(bv / V) * N * 14;
            const real *src = tmp + (size_t)bv * N * 14;
            for (size_t k = 0; k < (size_t)N * 14; k++) dst[k] += src[k];
        }
        free(tmp);
    }
    return err ? -1 : 0;
}

/*
 * Per-Gaussian preprocess records of one view, for tests that compare intermediates:
 *   radii [N] int, xy [N,2], depth [N], conic_opacity [N,4], rect [N,4] (min x, min y, max x, max y tiles).
 * Returns K (num_rendered) or -1.
 */
long long lgm_oracle_preprocess_view(int N, const real *g, const real *view, const real *proj, real tanfovx,
                                     real tanfovy, real scale_modifier, int H, int W, int *radii, real *xy,
                                     real *depth, real *conic, int *rect) {
    view_state S;
    memset(&S, 0, sizeof(S));
    S.N = N; S.H = H; S.W = W;
    S.gx = (W + BLOCK_X - 1) / BLOCK_X;
    S.gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    S.tanx = tanfovx; S.tany = tanfovy;
    S.fy = H / (2.0f * tanfovy);
    S.fx = W / (2.0f * tanfovx);
    S.mod = scale_modifier;
    S.g = g; S.view = view; S.proj = proj;
    const size_t n = N > 0 ? (size_t)N : 1;
    S.radii = radii; S.xy = xy; S.depth = depth; S.conic = conic; S.rect = rect;
    S.cov3 = (real *)calloc(6 * n, sizeof(real));
    if (!S.cov3) return -1;
    for (int i = 0; i < N; i++) { xy[2 * i] = xy[2 * i + 1] = 0; depth[i] = 0; conic[4 * i] = conic[4 * i + 1] = conic[4 * i + 2] = conic[4 * i + 3] = 0; }
    preprocess(&S);
    long long K = 0;
    for (int i = 0; i < N; i++)
        if (radii[i] > 0) K += (long long)(rect[4 * i + 2] - rect[4 * i]) * (rect[4 * i + 3] - rect[4 * i + 1]);
    free(S.cov3);
    return K;
}

/* Sorted tile lists of one view: tile_start [gx*gy+1], ids [K] (gaussian indices). Returns K or -1.
 * Call with ids == NULL to get K only. */
long long lgm_oracle_tile_lists(int N, const real *g, const real *view, const real *proj, real tanfovx,
                                real tanfovy, real scale_modifier, int H, int W, int *tile_start, int *ids,
                                long long ids_cap) {
    view_state S;
    memset(&S, 0, sizeof(S));
    S.N = N; S.H = H; S.W = W;
    S.gx = (W + BLOCK_X - 1) / BLOCK_X;
    S.gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    S.tanx = tanfovx; S.tany = tanfovy;
    S.fy = H / (2.0f * tanfovy);
    S.fx = W / (2.0f * tanfovx);
    S.mod = scale_modifier;
    S.g = g; S.view = view; S.proj = proj;
    const size_t n = N > 0 ? (size_t)N : 1;
    S.radii = (int *)calloc(n, sizeof(int));
    S.xy = (real *)calloc(2 * n, sizeof(real));
    S.depth = (real *)calloc(n, sizeof(real));
    S.conic = (real *)calloc(4 * n, sizeof(real));
    S.cov3 = (real *)calloc(6 * n, sizeof(real));
    S.rect = (int *)calloc(4 * n, sizeof(int));
    S.tile_start = tile_start;
    preprocess(&S);
    bin_and_sort(&S);
    const long long K = S.K;
    if (ids && K <= ids_cap)
        for (long long k = 0; k < K; k++) ids[k] = (int)(uint32_t)S.keys[k];
    free(S.radii); free(S.xy); free(S.depth); free(S.conic); free(S.cov3); free(S.rect); free(S.keys);
    return K;
}

/*
 * Forward state of one view (what upstream's imgBuffer keeps for the backward): per-pixel n_contrib (1 + list
 * position of the last accepted entry) and final transmittance, [H,W] each. Returns K or -1.
 */
long long lgm_oracle_forward_state(int N, const real *g, const real *view, const real *proj, real tanfovx,
                                   real tanfovy, real scale_modifier, int H, int W, int *n_contrib, real *final_T) {
    const size_t P = (size_t)H * W;
    real *c = (real *)calloc(3 * P, sizeof(real)), *d = (real *)calloc(P, sizeof(real)),
         *a = (real *)calloc(P, sizeof(real));
    view_state S;
    memset(&S, 0, sizeof(S));
    S.N = N; S.H = H; S.W = W;
    S.gx = (W + BLOCK_X - 1) / BLOCK_X;
    S.gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    S.tanx = tanfovx; S.tany = tanfovy;
    S.fy = H / (2.0f * tanfovy);
    S.fx = W / (2.0f * tanfovx);
    S.mod = scale_modifier;
    S.g = g; S.view = view; S.proj = proj;
    const size_t n = N > 0 ? (size_t)N : 1;
    S.radii = (int *)calloc(n, sizeof(int));
    S.xy = (real *)calloc(2 * n, sizeof(real));
    S.depth = (real *)calloc(n, sizeof(real));
    S.conic = (real *)calloc(4 * n, sizeof(real));
    S.cov3 = (real *)calloc(6 * n, sizeof(real));
    S.rect = (int *)calloc(4 * n, sizeof(int));
    S.tile_start = (int *)calloc((size_t)S.gx * S.gy + 1, sizeof(int));
    S.final_T = final_T;
    S.n_contrib = n_contrib;
    long long K = -1;
    if (c && d && a && S.radii && S.xy && S.depth && S.conic && S.cov3 && S.rect && S.tile_start) {
        const real bg[3] = {0, 0, 0};
        preprocess(&S);
        bin_and_sort(&S);
        render_fwd(&S, bg, c, d, a, NULL);
        K = S.K;
    }
    free(S.radii); free(S.xy); free(S.depth); free(S.conic); free(S.cov3); free(S.rect);
    free(S.tile_start); free(S.keys); free(c); free(d); free(a);
    return K;
}
