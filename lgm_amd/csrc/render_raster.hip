// lgm_amd/csrc/render_raster.hip -- per-tile alpha compositing (forward), its reverse-order gradient pass, and
// the per-Gaussian projection backward.
//
// One 256-thread workgroup per 16x16 tile; wavefront w owns the 8x8 quadrant (w & 1, w >> 1). The tile's sorted
// Gaussians are staged 256 at a time in LDS; the loader thread of each entry also tests the entry's alpha >= 1/255
// bounding box (render_common.h) against the four quadrants, and every wavefront then compacts the batch to the
// entries that can touch its quadrant (ballot + popcount prefix), so it only iterates over Gaussians for which
// some of its pixels pass upstream's `alpha >= 1/255` test. Per-pixel arithmetic, thresholds, the early
// termination and the reverse recurrences are upstream's; alpha is v_exp_f32 of the pre-scaled quadratic form plus
// log2(opacity) (the compositing records of render_common.h: 5 VALU + exp per (entry, pixel)).
#include "render_common.h"

#include <type_traits>

namespace lgm {
namespace {

__device__ __forceinline__ unsigned long long lanemask_lt(int lane) { return (1ull << lane) - 1ull; }

// Section stamps of the diagnostic builds LGM_BWD_STAMPS / LGM_FWD_STAMPS (shares only: the stamps' waits change
// the schedule).
#if defined(LGM_BWD_STAMPS) || defined(LGM_FWD_STAMPS)
__device__ __forceinline__ unsigned long long sec_stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define SEC_T(v) const unsigned long long v = sec_stamp()
#define SEC_ADD(acc, a, b) acc += (b) - (a)
#else
#define SEC_T(v)
#define SEC_ADD(acc, a, b)
#endif

// min(0.99, e) for e = exp2(.) >= 0 as an integer min on the bits (ordered like the floats for e >= 0; NaN -> 0.99
// as fminf): one VALU, where fminf on an exp result costs a canonicalising v_max first
__device__ __forceinline__ float alpha_cap(float e) {
    return __uint_as_float(min(__float_as_uint(e), 0x3f7d70a4u));
}

__device__ __forceinline__ int __reduce_add_wave(unsigned v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (unsigned)__shfl_xor((int)v, o, 64);
    return (int)v;
}

__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}


typedef __attribute__((ext_vector_type(4))) float f32x4;
constexpr int WU_LD = 68;  // row stride of the per-wave [16 columns][64 pixels] gradient image (16-B aligned rows)
// Columns 4..11 of that image hold pixel p at p ^ 8 (WU_SWZ): with the 17-slot row stride this puts the 16 lanes of
// every ds_read_b128 group of the batch reads (lanes {0-3, 12-15, 20-27}, ... : MI355X_MICROARCH.md §LDS) on 16
// distinct 16-B slots; unswizzled, columns 10, 11 and 12, 13 of one group shared two slots (2-way).
__device__ __forceinline__ int wu_swz(int col) { return (col >= 4 && col < 12) ? 8 : 0; }
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;
typedef __attribute__((ext_vector_type(2))) float f32x2v;
constexpr int MB = 8;      // entries per moment-MFMA batch (columns 0..7: w, 8..15: u)

// One staged 256-entry chunk, written by LDS DMA (global_load_lds: 16-B lane stride for both the 16-B and the
// 12-B form): P from gP, Q from gQ, R.xyz from the Gaussian row's colour; R.w holds the Gaussian id (written
// at commit). Two of these alternate: chunk c+1 streams into one while chunk c is composited from the other.
template <int ROWS>  // entries per chunk; row ROWS is the sentinel
struct StageBufT {
    float4 P[ROWS + 1];  // x, y, A, B
    float4 Q[ROWS + 1];  // C, opacity, tau, depth
    float4 R[ROWS + 1];  // r, g, b, id bits
};
using StageBuf = StageBufT<TILE_PIX>;
template <int NB, int PAD, int ROWS = TILE_PIX>  // NB 2: double-buffered, 1: synchronous staging
struct StageT {                                   // PAD: list padding = entries evaluated per step (multiple of 4)
    static constexpr int kRows = ROWS;
    using Buf = StageBufT<ROWS>;
    Buf buf[NB];
    unsigned char mask[ROWS];                 // quadrant mask of the current chunk's entries
    unsigned short list[4][ROWS + PAD];       // per-wave compacted entry indices, padded with the sentinel (ROWS)
};
// Forward: staged synchronously, chunk by chunk (double-buffered staging measured +20 us on the pool: most tiles
// saturate within a chunk or two, and the prefetch costs LDS and registers); FWD_FU = 4 entries evaluated per step
// (8 per step spilled). Backward: 64-entry chunks, double-buffered.
constexpr int FWD_FU = 4;
#ifndef LGM_FWD_SMALL_TILES
#define LGM_FWD_SMALL_TILES 256
#endif
constexpr int FWD_SMALL_TILES = LGM_FWD_SMALL_TILES;  // launches of at most this many tiles take k_render_fwd<., 8>
constexpr int BWD_CHUNK = 64;
// backward lists are padded to MB with the sentinel: every list position is one MFMA batch column (k_render_bwd)
using StageBwd = StageT<2, MB, BWD_CHUNK>;

// Wait for every outstanding vector-memory operation of this wave (incl. its LDS DMA). A hard s_waitcnt: the
// compiler's waitcnt pass sees it, and does not itself track LDS written by DMA.
__device__ __forceinline__ void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0) only

// LDS DMA (global_load_lds_dwordx{3,4}: lane i's bytes land at M0 + 16 i). Issued from inline asm on purpose:
// the compiler's waitcnt pass treats any later LDS access that may alias a pending DMA as dependent on it and
// would wait for the prefetch right after issuing it. Hidden from the pass, the DMA only makes the pass's own
// vmcnt waits more conservative (still correct); its completion is ordered explicitly by vm_wait_all() plus a
// barrier. M0 is saved and restored around it (the compiler owns M0), with the M0 -> LDS-DMA wait state.
// The LDS address of a shared-memory pointer as a 32-bit offset (an address-space cast, not the 64-bit flat pointer:
// kept live across the staging loop, the flat pointers were spilled and each reload's vmcnt(0) serialised the DMAs).
__device__ __forceinline__ unsigned lds_offset(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
template <int BYTES>
__device__ __forceinline__ void lds_dma(const void *src, unsigned lds_row0) {
    const unsigned m = __builtin_amdgcn_readfirstlane(lds_row0);
    unsigned saved;
    if (BYTES == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(saved)
                     : "s"(m), "v"(src)
                     : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx3 %2, off\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(saved)
                     : "s"(m), "v"(src)
                     : "memory");
}

// Issue the LDS DMA of one entry (this lane's row of wave w's 64-row slice). Asynchronous: the rows are valid
// after vm_wait_all() in every issuing wave followed by a barrier.
template <class Buf>
__device__ __forceinline__ void stage_dma(Buf &B, int w, unsigned gid, size_t gbase, int b, int N,
                                          const float4 *__restrict__ gP, const float4 *__restrict__ gQ,
                                          const float *__restrict__ gauss) {
    // one 32-bit LDS base, the three rows at constant offsets from it
    const unsigned base = lds_offset(&B) + (unsigned)(w * 64 * 16);
    lds_dma<16>(gP + gbase + gid, base + (unsigned)offsetof(Buf, P));
    lds_dma<16>(gQ + gbase + gid, base + (unsigned)offsetof(Buf, Q));
    lds_dma<12>(gauss + ((size_t)b * N + gid) * 14 + 11, base + (unsigned)offsetof(Buf, R));
}

// Entry j of a landed chunk: its quadrant mask (the alpha >= 1/255 ellipse against the four 8x8 quadrants) and,
// for the backward's gradient flush, its Gaussian id.
template <class Stage>
__device__ __forceinline__ void stage_commit(Stage &S, typename Stage::Buf &B, int j, bool have, unsigned gid, int tx0, int ty0,
                                             bool store_id) {
    unsigned char mask = 0;
    if (have) {
        const float4 p = B.P[j], q = B.Q[j];
        if (store_id) reinterpret_cast<unsigned *>(&B.R[j])[3] = gid;
        const float A = -p.z, Bc = -0.5f * p.w, C = -q.x, iA = 1.0f / A, iC = 1.0f / C;  // KQ-scaled (render_common.h)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float qx = (float)(tx0 + ((k & 1) << 3)), qy = (float)(ty0 + ((k >> 1) << 3));
            if (ellipse_hits_rect(p.x, p.y, A, Bc, C, iA, iC, q.z, qx, qx + 7.0f, qy, qy + 7.0f))
                mask |= (unsigned char)(1u << k);
        }
    }
    S.mask[j] = mask;
}

template <class Stage>
__device__ __forceinline__ int compact_wave(Stage &S, int w, int lane, int jmin = 0, int jend = Stage::kRows) {
    constexpr int PAD = (int)(sizeof(S.list[0]) / sizeof(S.list[0][0])) - Stage::kRows;
    int cnt = 0;
    const unsigned long long lt = lanemask_lt(lane);
#pragma unroll
    for (int c = 0; c < Stage::kRows / 64; c++) {
        const int j = c * 64 + lane;
        const bool bit = ((S.mask[j] >> w) & 1u) && j >= jmin && j < jend;
        const unsigned long long bal = __ballot(bit);
        if (bit) S.list[w][cnt + __popcll(bal & lt)] = (unsigned short)j;
        cnt += __popcll(bal);
    }
    if (lane < PAD) S.list[w][cnt + lane] = (unsigned short)Stage::kRows;  // pad to the next multiple of PAD
    return cnt;
}

// U (a multiple of 4) consecutive list entries from kk (a multiple of 4): list_raw reads them (an LDS read that can
// be issued a step ahead), list_decode makes them wave-uniform (scalar) indices.
template <int U, class Stage>
__device__ __forceinline__ void list_raw(const Stage &S, int w, int kk, uint2 (&raw)[U / 4]) {
    static_assert(U % 4 == 0, "list reads are 8-B words");
#pragma unroll
    for (int h = 0; h < U / 4; h++) raw[h] = *reinterpret_cast<const uint2 *>(&S.list[w][kk + 4 * h]);
}
template <int U>
__device__ __forceinline__ void list_decode(const uint2 (&raw)[U / 4], int (&jj)[U]) {
#pragma unroll
    for (int h = 0; h < U / 4; h++) {
        const unsigned lo = __builtin_amdgcn_readfirstlane(raw[h].x), hi = __builtin_amdgcn_readfirstlane(raw[h].y);
        jj[4 * h + 0] = lo & 0xffffu;
        jj[4 * h + 1] = lo >> 16;
        jj[4 * h + 2] = hi & 0xffffu;
        jj[4 * h + 3] = hi >> 16;
    }
}
template <class Stage>
__device__ __forceinline__ void init_sentinel(Stage &S) {
    if (threadIdx.x < sizeof(S.buf) / sizeof(S.buf[0])) {
        auto &B = S.buf[threadIdx.x];
        B.P[Stage::kRows] = make_float4(0.f, 0.f, 0.f, 0.f);
        B.Q[Stage::kRows] = make_float4(0.f, -INFINITY, 0.f, 0.f);  // L = -inf: alpha 0
        B.R[Stage::kRows] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// k_render_fwd: grid (B*V*T), block 256, tile xcd_item(blockIdx). 7 waves per SIMD: <= 72 VGPRs (spills outside
// the compositing loop only): 327 vs 336 us at 6, 411 at 8 (pool).
// FU: entries evaluated per step. 4 for every launch that fills the chip; launches of at most one tile per CU
// (FWD_SMALL_TILES: a single 256^2 view, BASELINE config 2) run one wave per SIMD, where nothing hides a wave's own
// dependency chains, and take FU = 8 at 2 waves per SIMD (more registers: twice the independent evaluations in flight).
// The serial T / colour chain is in list order either way: the outputs are bitwise the same.
template <bool LOSS, int FU>  // LOSS: LGM_RENDER_FUSED_LOSS compiled in (its epilogue registers stay out otherwise)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(FU == FWD_FU ? 7 : 2))) void k_render_fwd(Dims d, long long slot_stride,
                                                    const int *__restrict__ tile_start,
                                                    const int *__restrict__ tile_count,
                                                    const unsigned long long *__restrict__ pairs,
                                                    const float4 *__restrict__ gP, const float4 *__restrict__ gQ,
                                                    const float *__restrict__ gauss,
                                                    const float *__restrict__ bg, float *__restrict__ out_img,
                                                    float *__restrict__ out_depth, float *__restrict__ out_alpha,
                                                    float *__restrict__ final_T, int *__restrict__ n_contrib,
                                                    int *__restrict__ wlast_out,
                                                    unsigned char *__restrict__ cmask, float4 *__restrict__ cfin,
                                                    float *__restrict__ ck, int2 *__restrict__ cklist,
                                                    int *__restrict__ nck, unsigned *__restrict__ ckctr,
                                                    int ck_region, float4 *__restrict__ zero_base,
                                                    long long zero_n16) {
    __shared__ StageT<1, FU> S;
    __shared__ int s_ck[2];
    const int tile = xcd_item(blockIdx.x, d.BV * d.T);
    const int bv = tile / d.T, t = tile - bv * d.T, b = bv / d.V;
    const int tx0 = (t % d.gx) * BX, ty0 = (t / d.gx) * BY;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    int lx, ly;
    tile_pixel(tid, lx, ly);
    const int px = tx0 + lx, py = ty0 + ly;
    const bool inside = px < d.W && py < d.H;
    const float pfx = (float)px, pfy = (float)py;
    long long base;
    int n;
    tile_range(tile, slot_stride, tile_start, tile_count, base, n);
    const unsigned *ids = reinterpret_cast<const unsigned *>(pairs + base);
    const size_t gbase = (size_t)bv * d.N;
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    init_sentinel(S);
    // Tr < 0 marks a saturated pixel (|Tr| its final transmittance): outside pixels start saturated
    float Tr = inside ? 1.0f : -1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, D = 0.f;
    int last = 0;
    unsigned c_iter = 0, c_list = 0;  // diagnostic work counters (Dims::counters)
    // Staging: chunk c's entries land by LDS DMA, synchronously; the sorted ids run two chunks ahead in registers.
    // Each lane tests its own entry as soon as its row has landed, so one barrier publishes rows and masks together.
    unsigned id_a = tid < n ? ids[tid] : 0u;                        // chunk c
    unsigned id_b = TILE_PIX + tid < n ? ids[TILE_PIX + tid] : 0u;  // chunk c + 1
    // Backward checkpoints: entering every chunk c >= 1 the per-pixel state (T and the prefix colour / depth sums)
    // goes to a pool slot, reserved one chunk ahead from the region's counter (thread 0), so that k_render_bwd can
    // take the chunk as a work item of its own. The pool is sharded by tile over ckctr's 8 counters; a full region
    // just leaves the rest of the tile to the previous chunk's item.
    // (the region is the tile's XCD block group and its slots are interleaved by region, so the backward's
    // checkpoint items run on the XCD that composited the tile). Deterministic mode takes none (render_common.h).
    const int ck_reg = xcd_group(tile, d.BV * d.T);
    const bool det_ck = (d.options & LGM_RENDER_DETERMINISTIC) != 0;
    int ck_slot = -1, ck_written = 0;  // thread 0: slot reserved for the next boundary; checkpoints written
#ifdef LGM_FWD_STAMPS  // wave cycles per section (diagnostic build; per-tile counters +2..+5, scripts/diag_fwd_stamps.py)
    unsigned long long fs_head = 0, fs_mid = 0, fs_comp = 0;
    const unsigned long long fs_t0 = sec_stamp();
#endif
    for (int b0 = 0, c = 0; b0 < n; b0 += TILE_PIX, c++) {
#ifdef LGM_FWD_STAMPS
        const unsigned long long fs_a = sec_stamp();
#endif
        if (tid == 0) s_ck[c & 1] = ck_slot;  // reserved during chunk c - 1 (its atomic has long returned)
        if (__syncthreads_count(Tr < 0.f) == TILE_PIX) break;  // also: every wave is done with the previous chunk
        c_list += min(TILE_PIX, n - b0);
        const int k = b0 + tid;
        StageBuf &B = S.buf[0];
        if (k < n) stage_dma(B, w, id_a, gbase, b, d.N, gP, gQ, gauss);
        vm_wait_all();
        stage_commit(S, B, tid, k < n, 0u, tx0, ty0, false);
        __syncthreads();
#ifdef LGM_FWD_STAMPS
        const unsigned long long fs_b = sec_stamp();
        fs_head += fs_b - fs_a;
#endif
        // checkpoint stores and the next reservation go out after this chunk's DMA wait, so they have the whole
        // chunk's compositing to complete before the next wait
        if (tid == 0) {
            ck_slot = -1;
            if (b0 + TILE_PIX < n && !det_ck && ((c + 1) & ((1 << d.ck_shift) - 1)) == 0) {
                const unsigned l = atomicAdd(&ckctr[ck_reg], 1u);
                if (l < (unsigned)ck_region) ck_slot = (int)l * 8 + ck_reg;
            }
        }
        if (c >= 1) {
            const int sl = s_ck[c & 1];  // workgroup-uniform
            if (sl >= 0) {
                int ctid = tid;
                // (the lane's checkpoint address recomputed here: hoisted out of the chunk loop, ck + tid was spilled
                // and its reload's vmcnt(0) waited for the chunk's outstanding loads)
                asm volatile("" : "+v"(ctid));
                float *cp = ck + (size_t)sl * 5 * TILE_PIX + ctid;
                cp[0] = fabsf(Tr);
                cp[TILE_PIX] = C0;
                cp[2 * TILE_PIX] = C1;
                cp[3 * TILE_PIX] = C2;
                cp[4 * TILE_PIX] = D;
                if (tid == 0) {
                    cklist[sl] = make_int2(tile, c >> d.ck_shift);
                    ck_written = c >> d.ck_shift;
                }
            }
        }
        id_a = id_b;
        id_b = k + 2 * TILE_PIX < n ? ids[k + 2 * TILE_PIX] : 0u;
        const int cnt = compact_wave(S, w, lane);
#ifdef LGM_FWD_STAMPS
        const unsigned long long fs_c = sec_stamp();
        fs_mid += fs_c - fs_b;
#endif
        // FU = 4 entries per step: their alphas are independent of the running transmittance, so they are evaluated
        // together (ILP, branch-free: list padded with the opacity-0 sentinel); only the short T / colour update
        // chain stays serial, in list order, as upstream.
        uint2 lraw[FU / 4];  // the next step's list words, read one step ahead (the list is fixed for the chunk)
        list_raw<FU>(S, w, 0, lraw);
        for (int kk = 0; kk < cnt; kk += FU) {
            if (__ballot(Tr > 0.f) == 0ull) break;
            c_iter += min(FU, cnt - kk);
            int jj[FU];
            list_decode<FU>(lraw, jj);
            float al[FU];
            float4 cc[FU], Pv[FU], Qv[FU];
            // all the batch's LDS reads first, then one wait: the scheduler would otherwise interleave them with the
            // arithmetic entry by entry (its register-pressure heuristics) and expose the LDS latency FU times
#pragma unroll
            for (int u = 0; u < FU; u++) {
                Pv[u] = B.P[jj[u]];
                Qv[u] = B.Q[jj[u]];
                const float4 R = B.R[jj[u]];
                cc[u] = make_float4(R.x, R.y, R.z, 0.f);
            }
            list_raw<FU>(S, w, kk + FU, lraw);  // in bounds: the list rows hold kRows + FU words
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < FU; u++) {
                const float4 P = Pv[u], Q = Qv[u];
                cc[u].w = Q.w;
                // pre-scaled records (render_common.h): lp = power log2(e) + log2(opacity), e = opacity G
                const float dx = P.x - pfx, dy = P.y - pfy;
                const float lp = fmaf(Q.x * dy, dy, fmaf(fmaf(P.w, dy, P.z * dx), dx, Q.y));
                const float e = __builtin_amdgcn_exp2f(lp);
                const float alpha = alpha_cap(e);
                al[u] = (lp > Q.y || e < 1.0f / 255.0f) ? 0.f : alpha;  // 0 == skipped (power > 0 <=> lp > L)
            }
            // the serial chain as selects (no per-lane branches for the compiler to sink the alpha evaluations into,
            // so the FU evaluations above stay independent): upstream's test_T = T (1 - alpha) and T < 1e-4
            // termination, with the termination kept in Tr's sign -- a skipped entry (alpha 0) leaves test_T = T,
            // a saturated pixel (Tr < 0) has test_T <= 0, so one compare decides both
#pragma unroll
            for (int u = 0; u < FU; u++) {
                const float alpha = al[u];
                const float test_T = Tr * (1 - alpha);
                const bool keep = test_T >= 0.0001f;
                const float aw = keep ? alpha * Tr : 0.f;
                C0 = fmaf(cc[u].x, aw, C0);
                C1 = fmaf(cc[u].y, aw, C1);
                C2 = fmaf(cc[u].z, aw, C2);
                D = fmaf(cc[u].w, aw, D);
                Tr = keep ? test_T : -fabsf(Tr);
                const bool acc = keep && alpha != 0.f;
                last = acc ? b0 + jj[u] + 1 : last;
            }
        }
#ifdef LGM_FWD_STAMPS
        fs_comp += sec_stamp() - fs_c;
#endif
    }
#ifdef LGM_FWD_STAMPS
    if (d.counters && tid == 0) {
        d.counters[8 + 8 * (size_t)tile + 2] = fs_head;  // (wave 0: termination count + staging + entry tests + barrier)
        d.counters[8 + 8 * (size_t)tile + 3] = fs_mid;   // (checkpoint stores + compaction)
        d.counters[8 + 8 * (size_t)tile + 4] = fs_comp;  // (the compositing loop)
        d.counters[8 + 8 * (size_t)tile + 5] = sec_stamp() - fs_t0;  // (the whole chunk loop)
    }
#endif
    if (zero_n16 > 0) {
        // this workgroup's slice of the backward's gradient accumulators (per-view and per-scene records, fp32 or
        // int64): zeroed here, at the end of the compositing, where the stores have the rest of the launch to drain,
        // instead of in the binning's critical path (pool / single scene -8 / -2 us, profiles/r04/ab_zf)
        const long long per = (zero_n16 + gridDim.x - 1) / gridDim.x, z0 = per * blockIdx.x;
        const long long z1 = min(zero_n16, z0 + per);
        for (long long q = z0 + tid; q < z1; q += TILE_PIX) zero_base[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (tid == 0) {
        if (ck_slot >= 0) cklist[ck_slot] = make_int2(-1, 0);  // reserved for a boundary never reached
        nck[tile] = ck_written;  // checkpoints c = 1 .. ck_written exist (a prefix: the counters only grow)
    }
    {  // the wave's largest last contributor (outside pixels: 0), for the backward's list bounds
        const int wl = wave_max_i32(last);
        if (lane == 0) wlast_out[4 * (size_t)tile + w] = wl;
    }
    if (d.counters) {
        // per-workgroup timeline (100 MHz s_memrealtime ticks): [8 + 8 tile] start, +1 end, +7 entries staged (low
        // 32 bits) and this wave's 4-entry steps (high 32 bits, wave 0). No aggregate atomics on shared words here:
        // 4 same-address atomics per wave over every tile serialise in L2 and stretched the forward's timeline ~7x.
        if (tid == 0) {
            // where it ran: HW_ID (SE / CU / SIMD / wave slot) in the high half of [+6] (the list length stays in the
            // low half), the XCD (XCC_ID) in the top byte of [+7]
            const unsigned hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);
            const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);
            d.counters[8 + 8 * (size_t)tile] = t_start;
            d.counters[8 + 8 * (size_t)tile + 1] = __builtin_amdgcn_s_memrealtime();
            d.counters[8 + 8 * (size_t)tile + 6] = (unsigned long long)(unsigned)n | ((unsigned long long)hw_id << 32);
            d.counters[8 + 8 * (size_t)tile + 7] = (unsigned long long)c_list | ((unsigned long long)c_iter << 32) |
                                                   ((unsigned long long)xcc << 56);
        }
    }
    float lsq_img = 0.f, lsq_a = 0.f;  // fused loss: this pixel's squared residuals
    if (inside) {
        Tr = fabsf(Tr);  // (the sign only marked saturation)
        const size_t P = (size_t)d.H * d.W;
        const size_t pid = (size_t)d.W * py + px;
        final_T[bv * P + pid] = Tr;
        n_contrib[bv * P + pid] = last;
        float *img = out_img + (size_t)bv * 3 * P;
        // explicit FMAs: the fused loss's backward recomputes these values bit for bit from cfin and final_T
        float c0 = fmaf(Tr, bg[0], C0), c1 = fmaf(Tr, bg[1], C1), c2 = fmaf(Tr, bg[2], C2);
        if (d.options & LGM_RENDER_CLAMP_IMAGE) {  // core/gs.py:87, gradient mask kept for the backward
            auto in01 = [](float v) { return (v >= 0.f && v <= 1.f) ? 1u : 0u; };
            cmask[bv * P + pid] = (unsigned char)(in01(c0) | (in01(c1) << 1) | (in01(c2) << 2));
            c0 = fminf(fmaxf(c0, 0.f), 1.f);
            c1 = fminf(fmaxf(c1, 0.f), 1.f);
            c2 = fminf(fmaxf(c2, 0.f), 1.f);
        }
        img[pid] = c0;
        img[P + pid] = c1;
        img[2 * P + pid] = c2;
        out_depth[bv * P + pid] = D;
        out_alpha[bv * P + pid] = 1 - Tr;
        cfin[bv * P + pid] = make_float4(C0, C1, C2, D);  // pre-background totals for the backward
        if (LOSS) {
            // core/models.py:145-148: gt composited over the background, squared residuals of image and alpha
            const float m = d.gt_mask[bv * P + pid];
            const float *gi = d.gt_img + (size_t)bv * 3 * P;
            const float r0 = c0 - (gi[pid] * m + bg[0] * (1.f - m));
            const float r1 = c1 - (gi[P + pid] * m + bg[1] * (1.f - m));
            const float r2 = c2 - (gi[2 * P + pid] * m + bg[2] * (1.f - m));
            const float ra = (1 - Tr) - m;
            lsq_img = r0 * r0 + r1 * r1 + r2 * r2;
            lsq_a = ra * ra;
        }
    }
    if (LOSS) {  // per-tile partial sums, fixed order
        __shared__ float sL[2][4];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            lsq_img += __shfl_xor(lsq_img, o, 64);
            lsq_a += __shfl_xor(lsq_a, o, 64);
        }
        if (lane == 0) { sL[0][w] = lsq_img; sL[1][w] = lsq_a; }
        __syncthreads();
        if (tid < 2) d.loss_part[2 * (size_t)tile + tid] = ((sL[tid][0] + sL[tid][1]) + sL[tid][2]) + sL[tid][3];
    }
}

// Fused loss, final reduction over the per-tile (image, alpha) partials, fixed order, one launch: workgroup g sums
// tiles [g * LR_TILES, +LR_TILES) (each thread LR_PER independent loads, then a fixed tree), writes its double2
// partial, and the workgroup that arrives last (a counter in the workspace, zeroed by the forward's memset and
// reset by that workgroup) sums the partials in workgroup order and writes
// out = (loss_mse, mse_image, mse_alpha, psnr) as core/models.py:148 (F.mse_loss twice) and :167 (psnr).
// (Was one workgroup looping over every tile: 38.8 us at cfg5's 26,624 tiles, now a few us.)
constexpr int LR_THREADS = 256, LR_PER = 8, LR_TILES = LR_THREADS * LR_PER;
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__global__ __launch_bounds__(LR_THREADS) void k_loss_reduce(int M, const float2 *__restrict__ part, double n_img,
                                                           double n_a, double2 *__restrict__ wg_part,
                                                           unsigned *__restrict__ counter, float *__restrict__ out) {
    __shared__ double s[2][LR_THREADS / 64];
    __shared__ bool s_last;
    const int t = threadIdx.x, w = t >> 6, lane = t & 63;
    const int k0 = blockIdx.x * LR_TILES + t;
    float2 v[LR_PER];
#pragma unroll
    for (int u = 0; u < LR_PER; u++) {
        const int k = k0 + u * LR_THREADS;
        v[u] = k < M ? part[k] : make_float2(0.f, 0.f);
    }
    double a = 0.0, b = 0.0;
#pragma unroll
    for (int u = 0; u < LR_PER; u++) {
        a += (double)v[u].x;
        b += (double)v[u].y;
    }
    a = wave_sum_f64(a);
    b = wave_sum_f64(b);
    if (lane == 0) { s[0][w] = a; s[1][w] = b; }
    __syncthreads();
    if (t == 0) {
        double2 r = make_double2(0.0, 0.0);
        for (int q = 0; q < LR_THREADS / 64; q++) { r.x += s[0][q]; r.y += s[1][q]; }
        wg_part[blockIdx.x] = r;
        __threadfence();  // the partial is visible device-wide before the arrival is counted
        s_last = atomicAdd(counter, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();  // acquire: the other workgroups' partials (written back from their XCDs' L2s)
    double2 r = make_double2(0.0, 0.0);  // the last workgroup: partials in workgroup order (lanes, then a tree)
    for (int g = t; g < (int)gridDim.x; g += LR_THREADS) {
        const double2 x = wg_part[g];
        r.x += x.x;
        r.y += x.y;
    }
    r.x = wave_sum_f64(r.x);
    r.y = wave_sum_f64(r.y);
    if (lane == 0) { s[0][w] = r.x; s[1][w] = r.y; }
    __syncthreads();
    if (t == 0) {
        double si = 0.0, sa = 0.0;
        for (int q = 0; q < LR_THREADS / 64; q++) { si += s[0][q]; sa += s[1][q]; }
        const float mi = (float)(si / n_img), ma = (float)(sa / n_a);
        out[0] = mi + ma;
        out[1] = mi;
        out[2] = ma;
        out[3] = -10.f * log10f(mi);
        *counter = 0u;  // ready for the next launch on this workspace
    }
}

// Sum over each 16-lane DPP row (quad_perm, row_half_mirror, row_mirror): every lane ends with its row's sum.
#define LGM_DPP_ADD(v, ctrl)                                                                                   \
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xf, 0xf, false))
__device__ __forceinline__ float row_sum16(float v) {
    LGM_DPP_ADD(v, 0xB1);   // quad_perm [1,0,3,2]
    LGM_DPP_ADD(v, 0x4E);   // quad_perm [2,3,0,1]
    LGM_DPP_ADD(v, 0x141);  // row_half_mirror
    LGM_DPP_ADD(v, 0x140);  // row_mirror
    return v;
}

// The per-pixel seeds of the backward: dL/dpixel (colour, depth, alpha) after the fused loss's MSE terms and the
// clamp's gradient mask, and the forward's pre-background totals. Shared by k_render_bwd and (deterministic mode)
// k_det_seed_max, so both see the same values.
struct PixelSeed {
    float dp0, dp1, dp2, dpd, dpa;
    float4 cf;
};
template <bool DEPTH, bool LOSS>
__device__ __forceinline__ void pixel_seed(const Dims &d, bool inside, int bv, size_t P, size_t pid, float T_final,
                                           const float *__restrict__ bg, const float4 *__restrict__ cfin,
                                           const float *__restrict__ d_img, const float *__restrict__ d_depth,
                                           const float *__restrict__ d_alpha, const unsigned char *__restrict__ cmask,
                                           PixelSeed &o) {
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f, dpd = 0.f, dpa = 0.f;
    float4 cf = make_float4(0.f, 0.f, 0.f, 0.f);
    if (inside) {
        cf = cfin[bv * P + pid];
        if (d_img) {
            const float *di = d_img + (size_t)bv * 3 * P;
            dp0 = di[pid];
            dp1 = di[P + pid];
            dp2 = di[2 * P + pid];
        }
        unsigned cm = 7u;
        float dd = 0.f, da = 0.f;
        if (d.options & LGM_RENDER_CLAMP_IMAGE) cm = cmask[bv * P + pid];
        if (DEPTH) dd = d_depth[bv * P + pid];
        if (d_alpha) da = d_alpha[bv * P + pid];
        if (LOSS) {
            // the MSE seeds (core/models.py:148): dL/dimage += 2 (image - gt) dL/dmse_image / numel, likewise alpha;
            // image recomputed from the forward's totals exactly as the forward formed it
            const float s_img = 2.f * d.d_loss[0] / (float)(3.0 * d.BV * (double)P);
            const float s_a = 2.f * d.d_loss[1] / (float)((double)d.BV * P);
            const float m = d.gt_mask[bv * P + pid];
            const float *gi = d.gt_img + (size_t)bv * 3 * P;
            float c0 = fmaf(T_final, bg[0], cf.x), c1 = fmaf(T_final, bg[1], cf.y), c2 = fmaf(T_final, bg[2], cf.z);
            if (d.options & LGM_RENDER_CLAMP_IMAGE) {
                c0 = fminf(fmaxf(c0, 0.f), 1.f);
                c1 = fminf(fmaxf(c1, 0.f), 1.f);
                c2 = fminf(fmaxf(c2, 0.f), 1.f);
            }
            dp0 += s_img * (c0 - (gi[pid] * m + bg[0] * (1.f - m)));
            dp1 += s_img * (c1 - (gi[P + pid] * m + bg[1] * (1.f - m)));
            dp2 += s_img * (c2 - (gi[2 * P + pid] * m + bg[2] * (1.f - m)));
            dpa = s_a * ((1 - T_final) - m);
        }
        // (the loads are all issued above, in the blocks that only load: each use waits for the one round trip
        // they share -- with the loads next to their uses, the clamp mask and d_alpha were two serial trips)
        if (d.options & LGM_RENDER_CLAMP_IMAGE) {  // torch clamp gradient: passes where 0 <= x <= 1
            dp0 = (cm & 1u) ? dp0 : 0.f;
            dp1 = (cm & 2u) ? dp1 : 0.f;
            dp2 = (cm & 4u) ? dp2 : 0.f;
        }
        if (DEPTH) dpd = dd;
        dpa += da;
    }
    o.dp0 = dp0; o.dp1 = dp1; o.dp2 = dp2; o.dpd = dpd; o.dpa = dpa;
    o.cf = cf;
}

// ---- Deterministic mode (LGM_RENDER_DETERMINISTIC): int64 fixed-point accumulators with scales that follow the
// data, so neither tiny nor huge gradients lose their meaning.
//  * a per-call scale 2^s with s = DET_BITS - exponent(max |dL/dpixel| over every seed): the accumulators' unit is
//    2^-DET_BITS of the largest per-pixel seed, whatever the loss normalisation (LGM's mean-MSE gives dL/dpixel
//    ~1e-9 at 8 x 8 views of 512^2: a fixed 2^-32 unit would leave its partials only tens of units);
//  * per (view, Gaussian) power-of-two normalisers of the view-dependent partials, from the compositing record (so
//    k_render_bwd and k_preproc_bwd derive bitwise the same exponents): dL/dmean2D by (W/2) sqrt(A) (resp. (H/2)
//    sqrt(C)) and dL/dconic by 1 / Sigma_xx, 1 / sqrt(Sigma_xx Sigma_yy), 1 / Sigma_yy (Sigma = conic^-1): with
//    alpha >= 1/255 only where q <= 2 ln 255, each normalised per-pixel term is bounded by a small constant times
//    |dL/dG|, so a large, elongated Gaussian's conic partials (pixel offsets of hundreds) cannot overflow int64 and a
//    small one's keep their resolution.
// Every power-of-two scaling is exact, so the only rounding is each flush's conversion to an integer (nearest).
constexpr int DET_BITS = 30;  // seed max -> 2^30 units: per flush |value| <= ~2^51, sums of 2^11 flushes < 2^63
__device__ __forceinline__ int f32_exp(float x) { return (int)((__float_as_uint(x) >> 23) & 0xffu) - 127; }
constexpr int DET_SLOTS = 64;  // k_det_seed_max spreads its atomics over this many words (same-address atomics serialise)
__device__ __forceinline__ int det_seed_shift(const unsigned *det_max) {  // s: the call's global scale exponent
    const uint4 *p = reinterpret_cast<const uint4 *>(det_max);
    unsigned mb = 0u;
#pragma unroll
    for (int i = 0; i < DET_SLOTS / 4; i++) {
        const uint4 v = p[i];
        mb = max(max(mb, max(v.x, v.y)), max(v.z, v.w));
    }
    const float m = __uint_as_float(mb);
    return (m > 0.f && m < 3.0e38f) ? DET_BITS - f32_exp(m) : 0;
}
struct DetNorm {
    int k[6];  // exponents of the view record's slots: mean2D x, y, conic A, B, C, depth
};
__device__ __forceinline__ DetNorm det_norm(float Ap, float Bp, float Cp, int W, int H) {
#pragma clang fp contract(off)
    DetNorm n;
    const float detp = Ap * Cp - 0.25f * (Bp * Bp);  // KQ^2 det(conic): the record holds -KQ A, -2 KQ B, -KQ C
    if (!(detp > 0.f) || !(detp < 3.0e38f) || !(Ap < 0.f) || !(Cp < 0.f)) {
        for (int q = 0; q < 6; q++) n.k[q] = 0;
        return n;
    }
    const int ea = f32_exp(-Ap), ec = f32_exp(-Cp), ed = f32_exp(detp);
    auto cl = [](int x) { return min(60, max(-60, x)); };
    n.k[0] = cl(-(f32_exp(0.5f * (float)W) + (ea >> 1)));
    n.k[1] = cl(-(f32_exp(0.5f * (float)H) + (ec >> 1)));
    n.k[2] = cl(ed - ec);              // 1 / Sigma_xx ~ det / C
    n.k[3] = cl(ed - ((ea + ec) >> 1));  // 1 / sqrt(Sigma_xx Sigma_yy)
    n.k[4] = cl(ed - ea);              // 1 / Sigma_yy ~ det / A
    n.k[5] = 0;
    return n;
}

// k_det_seed_max: grid (min(B*V*T, DET_MAX_WGS)), block 256, each workgroup striding over tiles: max |dL/dpixel|
// over every seed of the call -> det_max[DET_SLOTS] (float bits, atomicMax on the non-negative bit pattern, slot
// blockIdx % DET_SLOTS; zeroed by the caller; readers take the max of the slots). One atomic per workgroup, spread
// over 64 words: same-address atomics serialise (one per wave on one word over 12,288 tiles took 564 us).
constexpr int DET_MAX_WGS = 4096;
template <bool DEPTH, bool LOSS>
__global__ __launch_bounds__(256) void k_det_seed_max(Dims d, const float *__restrict__ final_T,
                                                      const float *__restrict__ bg, const float4 *__restrict__ cfin,
                                                      const float *__restrict__ d_img, const float *__restrict__ d_depth,
                                                      const float *__restrict__ d_alpha,
                                                      const unsigned char *__restrict__ cmask,
                                                      unsigned *__restrict__ det_max, unsigned *__restrict__ det_sat) {
    __shared__ unsigned s_m[4];
    // the call's overflow count starts at zero here, ahead of every k_render_bwd flush of the call (a repeated
    // backward of the same forward, LGM_RENDER_BACKWARD_AGAIN, must not inherit an earlier backward's count)
    if (blockIdx.x == 0 && threadIdx.x == 0) *det_sat = 0u;
    int lx, ly;
    tile_pixel(threadIdx.x, lx, ly);
    const size_t P = (size_t)d.H * d.W;
    float m = 0.f;
    for (int tile = blockIdx.x; tile < d.BV * d.T; tile += gridDim.x) {
        const int bv = tile / d.T, t = tile - bv * d.T;
        const int px = (t % d.gx) * BX + lx, py = (t / d.gx) * BY + ly;
        const bool inside = px < d.W && py < d.H;
        const size_t pid = inside ? (size_t)d.W * py + px : 0;
        PixelSeed sd;
        pixel_seed<DEPTH, LOSS>(d, inside, bv, P, pid, inside ? final_T[bv * P + pid] : 0.f, bg, cfin, d_img, d_depth,
                                d_alpha, cmask, sd);
        m = fmaxf(m, fmaxf(fmaxf(fabsf(sd.dp0), fabsf(sd.dp1)),
                           fmaxf(fmaxf(fabsf(sd.dp2), fabsf(sd.dpd)), fabsf(sd.dpa))));
    }
    unsigned mb = __float_as_uint(m);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o, 64));
    if ((threadIdx.x & 63) == 0) s_m[threadIdx.x >> 6] = mb;
    __syncthreads();
    if (threadIdx.x == 0) {
        mb = max(max(s_m[0], s_m[1]), max(s_m[2], s_m[3]));
        if (mb) atomicMax(det_max + blockIdx.x % DET_SLOTS, mb);
    }
}

// k_render_bwd: grid (B*V*T + CK slots), block 256. DEPTH: an upstream depth gradient is present (LGM passes none).
//
// The gradient pass walks each tile's list FRONT TO BACK, the forward's order. Upstream's reverse recurrence (suffix
// colour accumulators) is replaced by the equivalent prefix form: with T_i the transmittance in front of entry i,
// D_i = sum_{j <= i} alpha_j T_j (c_j . dL/dC) and the forward's per-pixel totals Dfin = C . dL/dC, T_final,
//     dL/dalpha_i = T_i (c_i . dL/dC) - (Dfin - K - D_i) / (1 - alpha_i),    K = (dL/dA - bg . dL/dC) T_final,
// so the per-pixel state is just (T, D). That state is what the forward checkpoints at each 256-entry chunk
// boundary it crosses (k_render_fwd: T and the prefix colour/depth sums; D = prefix . dL/dC), so the backward work
// item is one CHUNK, not one tile: workgroup g < B*V*T takes chunk 0 of LPT tile g, workgroup B*V*T + s takes the
// chunk of checkpoint slot s (cklist), and runs to the next checkpoint (or the tile's end if the pool ran out).
// Long tiles no longer bound the launch.
//
// Per-entry gradient sums over a wave's 64 pixels are pixel moments on the MFMA: w = G dL/dG and u = alpha T give
// sum_p w f(p) for f in {1, x, y, x^2, xy, y^2} (tile-centred pixel coordinates; the mean2D and conic partials
// follow from these and the Gaussian centre) and sum_p u dL/dC_c(p): a [features x pixels] . [pixels x entries]
// product: the wave walks its list MB = 8 entries per step (list padded with the sentinel), writes their w
// (columns 0..MB-1) and u (columns MB..) to a per-wave LDS image and sums them with v_mfma_f32_16x16x32_bf16 (the
// geometric features are exact in bf16; w, u and dL/dC as hi + lo bf16 pairs, ~2^-16 relative per product). Moments are combined over the tile's four waves in LDS, turned into gradient partials per
// entry and flushed once per (chunk, entry) to the per-view accumulators.
// Occupancy: at least 4 waves per SIMD for the register allocation (<= 128 VGPRs; the 64-entry chunks' LDS admits 4
// workgroups per CU); 2 for the depth-gradient instantiation, which LGM never runs.
template <bool DEPTH, bool LOSS, bool DET>  // DET: LGM_RENDER_DETERMINISTIC (int64 fixed-point flush)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEPTH ? 2 : 4))) void k_render_bwd(
    Dims d, long long slot_stride, const int *__restrict__ tile_start,
    const int *__restrict__ tile_count, const unsigned long long *__restrict__ pairs, const float4 *__restrict__ gP,
    const float4 *__restrict__ gQ, const float *__restrict__ gauss, const float *__restrict__ bg,
    const float *__restrict__ final_T, const int *__restrict__ n_contrib, const int *__restrict__ wlast_fwd,
    const float4 *__restrict__ cfin, const float *__restrict__ ck, const int2 *__restrict__ cklist,
    const int *__restrict__ nck,
    const unsigned *__restrict__ ckctr, int ck_region, const float *__restrict__ d_img,
    const float *__restrict__ d_depth, const float *__restrict__ d_alpha, const unsigned char *__restrict__ cmask,
    float *__restrict__ accum, const unsigned *__restrict__ det_max, unsigned *__restrict__ det_sat,
    long long item_stamps) {
    constexpr int NV = DEPTH ? NACC : NACC - 1;  // partials per (pixel, Gaussian): mean2D(2) conic(3) op rgb(3) [depth]
    // entries per staged chunk; LDS row stride of the moment slots: LS = 4 (mod 32) puts the rows a moment store
    // writes at once (4 qk + rr, qk = 0, 1 in a 32-lane store group: rows rr and rr + 4) 16 banks apart, so a batch's
    // 8 consecutive entry columns land on distinct banks (ds_write_b32 banks are (a / 4) mod 32)
    // (the depth-gradient instantiation keeps stride 65 and one shared junk row: its larger slots would not leave
    // room for a fourth workgroup per CU otherwise)
    constexpr int CH = BWD_CHUNK, LS = CH + 4;
    __shared__ StageBwd S;
    // per-wave moment slots (plain stores: each wave writes an entry's moments once; no LDS atomics), combined over
    // the entry's quadrant waves after the entries loop. Rows 0..5 geometric (w columns), then one row per colour
    // [+ depth] channel (u columns): the A operand holds each channel's dL/dpixel hi and lo bf16 parts in adjacent
    // rows (6 + 2c, 7 + 2c: one lane's accumulator pair), so a lane adds the pair before storing and the slot keeps
    // NC colour rows, not 2 NC. The MFMA results a lane does not keep go to a junk word after the rows (JB + lane +
    // the batch column; never read), so the stores need no exec-masked branches.
    constexpr int NC = DEPTH ? 4 : 3, NROW = 6 + NC, NROWA = 6 + 2 * NC;
    constexpr int JB = (LS * NROW + 3) & ~3;
    constexpr int SLOT = JB + 64 + CH + 4;        // junk words JB + lane + column; 16-B aligned slots
    constexpr int ZSLOT = JB;                     // the part zeroed per chunk (the junk words are never read)
    __shared__ __attribute__((aligned(16))) float sAccW[4][SLOT];
    __shared__ __attribute__((aligned(16))) float sWU[4][16 * WU_LD];  // read as float4: keep 16-B aligned
    // the chunk's gradient partials (rows q * LS + j; a needle's conic partials in rows NV .. NV + 2 for the fp64
    // flush) and its Gaussian ids, written by the conversion and read by the flush. Their own buffer (not a dead WU
    // image) lets a wave start the next chunk's quadrant tests and entries right after its share of the flush, while
    // other waves still flush: one barrier less per chunk
    __shared__ __attribute__((aligned(16))) float sO[(NV + 3) * LS];
    __shared__ unsigned sId[CH];
    __shared__ int s_ndl[2];  // chunk parity: the chunk holds a needle-like record (conic partials to the fp64 block)

    // ---- work item: (tile, chunk c, checkpoint slot)
    const int M = d.BV * d.T, Mp = round8(M);  // head items, then the checkpoint items (none in deterministic mode)
    int tile, c = 0, slot = -1;
    if ((int)blockIdx.x < M) {
        tile = xcd_item(blockIdx.x, M);
    } else {
        if ((int)blockIdx.x < Mp) return;  // padding: the checkpoint items start at a multiple of 8
        slot = (int)blockIdx.x - Mp;
        if ((int)(slot >> 3) >= (int)ckctr[slot & 7]) return;  // an unused slot of region slot & 7 (workgroup-uniform)
        const int2 e = cklist[slot];
        if (e.x < 0) return;  // reserved, never written
        tile = e.x;
        c = e.y;
    }
    const int bv = tile / d.T, t = tile - bv * d.T, b = bv / d.V;
    const int tx0 = (t % d.gx) * BX, ty0 = (t / d.gx) * BY;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    int lx, ly;
    tile_pixel(tid, lx, ly);
    const int px = tx0 + lx, py = ty0 + ly;
    const bool inside = px < d.W && py < d.H;
    const float pfx = (float)px, pfy = (float)py;
    long long base;
    int n;
    tile_range(tile, slot_stride, tile_start, tile_count, base, n);
    const unsigned *ids = reinterpret_cast<const unsigned *>(pairs + base);
    // the first chunk's ids and LDS DMA go out before the per-pixel state loads (bounded by the list length n, a
    // superset of [s0, s1): rows past s1 are staged but never listed or flushed), so their two dependent memory
    // round trips overlap the pixel loads instead of following them
    const bool stager = w == 0;  // (wave 3 staging, with waves 0-2 flushing and never waiting for their atomics, measured
                                 // slower: pool k_render_bwd 608 -> 620 us, profiles/r06/ab_bwd_w3)
    const int s0e = (c * TILE_PIX) << d.ck_shift;
    unsigned id_cur = stager && s0e + lane < n ? ids[s0e + lane] : 0u;
    if (stager && s0e + lane < n) stage_dma(S.buf[0], 0, id_cur, (size_t)bv * d.N, b, d.N, gP, gQ, gauss);
    unsigned id_next = stager && s0e + BWD_CHUNK + lane < n ? ids[s0e + BWD_CHUNK + lane] : 0u;
    const size_t P = (size_t)d.H * d.W;
    const size_t pid = inside ? (size_t)d.W * py + px : 0;
    const float T_final = inside ? final_T[bv * P + pid] : 0.f;
    const int last = inside ? n_contrib[bv * P + pid] : 0;
    // the checkpoint's loads go out before the seeds' (one shared round trip instead of a third serial one)
    float ckT = 1.0f, ck1 = 0.f, ck2 = 0.f, ck3 = 0.f, ck4 = 0.f;
    if (slot >= 0) {
        const float *cp = ck + (size_t)slot * 5 * TILE_PIX;
        ckT = cp[tid];
        ck1 = cp[TILE_PIX + tid];
        ck2 = cp[2 * TILE_PIX + tid];
        ck3 = cp[3 * TILE_PIX + tid];
        if (DEPTH) ck4 = cp[4 * TILE_PIX + tid];
    }
    PixelSeed sd;
    pixel_seed<DEPTH, LOSS>(d, inside, bv, P, pid, T_final, bg, cfin, d_img, d_depth, d_alpha, cmask, sd);
    const float dp0 = sd.dp0, dp1 = sd.dp1, dp2 = sd.dp2, dpd = sd.dpd, dpa = sd.dpa;
    const float4 cf = sd.cf;
    // per-pixel state entering the chunk: the forward's checkpoint (or the list head)
    float Tr = 1.0f, Dup = 0.f;
    if (slot >= 0) {
        Tr = ckT;
        Dup = fmaf(ck1, dp0, fmaf(ck2, dp1, ck3 * dp2));
        if (DEPTH) Dup = fmaf(ck4, dpd, Dup);
    }
    init_sentinel(S);  // (published by the first barrier of the chunk loop)
    // the forward's per-wave maxima of the last contributors: positions >= wlast touch no pixel of this wave, and
    // entries behind every pixel's last contributor are never visited
    const int4 wl4 = reinterpret_cast<const int4 *>(wlast_fwd)[tile];
    const int wlast = w == 0 ? wl4.x : w == 1 ? wl4.y : w == 2 ? wl4.z : wl4.w;
    const int nlist = min(n, max(max(wl4.x, wl4.y), max(wl4.z, wl4.w)));
    const int s0 = (c * TILE_PIX) << d.ck_shift;
    if (s0 >= nlist) {  // workgroup-uniform (the early DMA must land before the workgroup retires)
        vm_wait_all();
        return;
    }
    const int s1 = (c + 1 <= nck[tile]) ? min(nlist, s0 + (TILE_PIX << d.ck_shift)) : nlist;
    if (s0 >= s1) {  // (nothing to do; likewise)
        vm_wait_all();
        return;
    }
    const unsigned long long t_item = d.counters ? __builtin_amdgcn_s_memrealtime() : 0ull;
#ifdef LGM_BWD_STAMPS  // section cycles of this wave (diagnostic build; counters [0..7], scripts/diag_bwd_stamps.py)
    // [0] prologue, [1] chunk-top barrier, [2] chunk head (quadrant tests, compaction, next DMA issue), [3] entries
    // loop, [4] the post-entries barrier + moments -> partials, [5] the DMA wait (vmcnt 0), [6] the pre-flush
    // barrier, [7] the gradient atomics
    unsigned long long sec[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    SEC_T(ts_item);
#endif
    const float bg_dot = bg[0] * dp0 + bg[1] * dp1 + bg[2] * dp2;
    float cdpf = fmaf(cf.x, dp0, fmaf(cf.y, dp1, cf.z * dp2));
    if (DEPTH) cdpf = fmaf(cf.w, dpd, cdpf);
    const float DK = cdpf - (dpa - bg_dot) * T_final;  // Dfin - K
    float Erem = DK - Dup;  // Dfin - K - D_i, kept directly (one subtraction less per entry)
    const float ddelx_dx = 0.5f * d.W, ddely_dy = 0.5f * d.H;
    const int det_s = DET ? det_seed_shift(det_max) : 0;
    // per-flush bounds of the per-view and the per-scene records (render_common.h det_flush_limit_log2)
    const float det_lim_v = ldexpf(1.f, d.det_lim_log2 ? d.det_lim_log2 : det_flush_limit_log2(d.V, d.T, false));
    const float det_lim_s = ldexpf(1.f, d.det_lim_log2 ? d.det_lim_log2 : det_flush_limit_log2(d.V, d.T, true));
    const size_t gbase = (size_t)bv * d.N;
    // MFMA operands: A (features) lane (ql, qk) holds feature ql of wave pixels 32 t + 8 qk + j, j = 0..7
    const int ql = lane & 15, qk = lane >> 4;
    const float cxT = (float)tx0 + 7.5f, cyT = (float)ty0 + 7.5f;
    // the slot offset of this lane's r-th stored value: w columns (ql < MB) keep D rows 4 qk + r <= 5 (the geometric
    // moments); u columns keep the sums of the accumulator pairs (r = 0: D rows 4 qk, 4 qk + 1; r = 1: 4 qk + 2, + 3)
    // that are a colour channel's hi / lo rows 6 + 2c, 7 + 2c -> slot row 6 + c. Everything else: the junk word.
    int mrow[4];
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
        int row = -1;
        if (ql < MB) {
            if (4 * qk + rr <= 5) row = 4 * qk + rr;
        } else if (rr < 2) {
            const int a = 4 * qk + 2 * rr;  // the pair's first D row
            if (a >= 6 && a < NROWA) row = 6 + (a - 6) / 2;
        }
        mrow[rr] = row >= 0 ? row * LS : JB + lane;
    }
    float *myAcc = sAccW[w];
    float *myWU = sWU[w];
    const int lane_x = lane ^ 8;  // this lane's pixel in the swizzled image columns (wu_swz)
    myWU[lane] = dp0;
    myWU[64 + lane] = dp1;
    myWU[128 + lane] = dp2;
    myWU[192 + lane] = dpd;
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    // A operand: lane (ql, qk) holds row ql at the wave pixels p = 32 t2 + 8 qk + j, j = 0..7, i.e. tile-centred
    // fx = fx0 + j and fy = fy0 + 4 t2 + qk. Rows 0..5, the geometric features, are a + b j + c j^2 with per-lane
    // coefficients, exact in bf16 (small integers and halves); rows 6..6+NC-1 are dL/dpixel rounded to bf16 and rows
    // 6+NC.. the remainders, so A . (B_hi + B_lo) -- two MFMAs -- carries every product but lo x lo (~2^-16).
    bf16x8 Ah[2];
    {
        const float fx0 = (float)((w & 1) << 3) - 7.5f, fy0 = (float)((w >> 1) << 3) - 7.5f;
        const bool isdp = ql >= 6 && ql < NROWA, islo = isdp && ((ql - 6) & 1);
        const int qd = isdp ? (ql - 6) >> 1 : 0;  // the dL/dpixel channel of rows 6..NROWA-1 (hi, lo per channel)
#pragma unroll
        for (int t2 = 0; t2 < 2; t2++) {
            const float fy = fy0 + (float)(4 * t2 + qk);
            const float ca = ql == 0 ? 1.f : ql == 1 ? fx0 : ql == 2 ? fy : ql == 3 ? fx0 * fx0
                           : ql == 4 ? fx0 * fy : ql == 5 ? fy * fy : 0.f;
            const float cb = ql == 1 ? 1.f : ql == 3 ? 2.f * fx0 : ql == 4 ? fy : 0.f;
            const float cc2 = ql == 3 ? 1.f : 0.f;
            const float4 *src = reinterpret_cast<const float4 *>(myWU + qd * 64 + 32 * t2 + 8 * qk);
            const float4 d0 = src[0], d1 = src[1];
            const float dv[8] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w};
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const float geo = fmaf(fmaf(cc2, (float)j, cb), (float)j, ca);
                const __bf16 dh = (__bf16)dv[j];
                const float dlo = dv[j] - (float)dh;
                Ah[t2][j] = ql <= 5 ? (__bf16)geo : !isdp ? (__bf16)0.f : islo ? (__bf16)dlo : dh;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    int myj = 0;  // the chunk row of this lane's batch column (ql & 7)
    // Moment precision. On needle-like footprints (conic condition > ~1e3) the cov2D inverse amplifies any rounding
    // of the conic gradients into their scale / rotation gradients. A two-term split with a TRUNCATED hi part biases
    // every product's rounding one way (~2^-16, coherent over a tile's pixels): at 512^2 it left mean / scale / rot
    // at ~2x the fp32 oracle's own error vs fp64. A round-to-nearest hi part (same instruction count: <= 2^-17 per
    // product, unbiased) and an exact three-term split (+2 MFMAs and +40 VALU per 8-entry batch, k_render_bwd +7 %
    // on the pool) both put them at 0.5-0.8x the oracle's (profiles/r03/diag_float_spread), so the two-term
    // round-to-nearest split is used in both modes.
    // B operand of the current batch: lane (ql, qk) takes column ql at pixels 32 t + 8 qk + j (two 16-B reads per t)
    auto read_batch = [&](float (&xs)[2][8]) {
#pragma unroll
        for (int t2 = 0; t2 < 2; t2++) {
            const float *row = myWU + ql * WU_LD;
            const int p0 = 32 * t2 + 8 * qk, sw = wu_swz(ql);
            const float4 x0 = *reinterpret_cast<const float4 *>(row + (p0 ^ sw));
            const float4 x1 = *reinterpret_cast<const float4 *>(row + ((p0 + 4) ^ sw));
            xs[t2][0] = x0.x; xs[t2][1] = x0.y; xs[t2][2] = x0.z; xs[t2][3] = x0.w;
            xs[t2][4] = x1.x; xs[t2][5] = x1.y; xs[t2][6] = x1.z; xs[t2][7] = x1.w;
        }
    };
    // split hi + lo, the moment MFMAs, and the lane's (at most 4) live results into this wave's slots
    auto mfma_batch = [&](const float (&xs)[2][8], int col) {
        f32x4 a2[2];
#pragma unroll
        for (int t2 = 0; t2 < 2; t2++) {
            // hi = x rounded to bf16 (|x - hi| <= 2^-9 |x|), lo = the exact remainder rounded: <= 2^-17 |x| per
            // product (per pair: two packed conversions, the two hi halves back to fp32 by a shift and a mask, two
            // subtractions)
            bf16x8 bh, bl;
#pragma unroll
            for (int j = 0; j < 8; j += 2) {
                const bf16x2v hp = __builtin_convertvector((f32x2v){xs[t2][j], xs[t2][j + 1]}, bf16x2v);
                const unsigned hb = __builtin_bit_cast(unsigned, hp);
                const float h0 = __builtin_bit_cast(float, hb << 16), h1 = __builtin_bit_cast(float, hb & 0xffff0000u);
                const bf16x2v lp = __builtin_convertvector((f32x2v){xs[t2][j] - h0, xs[t2][j + 1] - h1}, bf16x2v);
                bh[j] = hp[0];
                bh[j + 1] = hp[1];
                bl[j] = lp[0];
                bl[j + 1] = lp[1];
            }
            f32x4 cacc = {0.f, 0.f, 0.f, 0.f};
            cacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah[t2], bh, cacc, 0, 0, 0);
            cacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ah[t2], bl, cacc, 0, 0, 0);
            a2[t2] = cacc;
        }
        const f32x4 acc = a2[0] + a2[1];
        // D[row = 4 qk + r][col = ql]: moments 0..5 in the w columns; in the u columns each colour channel's hi and lo
        // rows are one lane's pair (r, r + 1), added here (the same sum the conversion formed before: bitwise equal);
        // each lane stores its values at per-lane offsets fixed for the kernel (mrow; dead ones to its junk word)
        const bool ucol = ql >= MB;
        const float v0 = ucol ? acc[0] + acc[1] : acc[0], v1 = ucol ? acc[2] + acc[3] : acc[1];
        myAcc[mrow[0] + col] = v0;  // (sentinel columns: row CH, all zero)
        myAcc[mrow[1] + col] = v1;
        myAcc[mrow[2] + col] = acc[2];
        myAcc[mrow[3] + col] = acc[3];
    };

    // Staging pipeline (front to back over [s0, s1)): chunk b0 + CH streams into the other buffer by LDS DMA
    // during chunk b0's compositing and is complete (vm_wait_all) before chunk b0's gradient atomics are issued,
    // so no staging load queues behind them; the sorted ids run one chunk further ahead in a register.
    // Two barriers per chunk: P (after the entries loop: every wave's moments are in its slot) and F (before the
    // flush: the partials are in sO, and the stager's next chunk has landed). The chunk-top barrier of rounds 1-5 is
    // gone: a wave goes from its share of chunk c's flush straight into chunk c + 1's quadrant tests and entries
    // while the others still flush. That is safe because nothing the flush reads is written before the next P:
    // the partials and ids live in sO / sId (rewritten only by the next conversion, after P), the needle flag has one
    // word per chunk parity, and the next chunk's DMA overwrites the buffer of chunk c - 1, whose last reader (the
    // conversion of c - 1) finished before F of c - 1. Each wave zeroes its own moment slot at the top of a chunk,
    // after the conversion that read it (before F).
    vm_wait_all();
    __syncthreads();  // the first chunk's rows and the sentinel rows
    int cur = 0;
#ifdef LGM_BWD_STAMPS
    SEC_T(ts_loop);
    SEC_ADD(sec[0], ts_item, ts_loop);  // prologue: pixel state, seeds, MFMA operands, first staging
#endif
    for (int b0 = s0, ci = 0; b0 < s1; b0 += CH, cur ^= 1, ci++) {
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c0b);
#endif
        auto &B = S.buf[cur];
        // one row per lane: every wave tests all CH entries against its OWN quadrant (one ellipse test per lane
        // instead of four per staging thread) and the ballot is its compaction mask (no shared mask, no barrier)
        if (stager) reinterpret_cast<unsigned *>(&B.R[lane])[3] = id_cur;  // for the gradient flush
        if (!DET && tid == 0) s_ndl[ci & 1] = 0;  // (published by P; the flush of chunk ci - 2 read it before P of ci - 1)
        {  // every wave zeroes its own slot (an entry it skips, or never lists, adds nothing): wave-private, so the
           // entries loop follows the quadrant tests without a barrier (with the conversion over three waves below:
           // pool k_render_bwd 642 -> 635 us, bitwise equal, profiles/r04/ab_bwd_conv)
            float4 *z = reinterpret_cast<float4 *>(myAcc);
            for (int q = lane; q < ZSLOT / 4; q += 64) z[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        int cnt;
        {
            bool hit = false;
            if (b0 + lane < s1 && lane < wlast - b0) {  // positions < wlast only
                const float4 p = B.P[lane], q = B.Q[lane];
                const float qx = (float)(tx0 + ((w & 1) << 3)), qy = (float)(ty0 + ((w >> 1) << 3));
                hit = rec_hits_rect(p, q, qx, qx + 7.0f, qy, qy + 7.0f);
            }
            const unsigned long long bal = __ballot(hit);
            if (hit) S.list[w][__popcll(bal & lanemask_lt(lane))] = (unsigned short)lane;
            cnt = __popcll(bal);
            constexpr int PAD = (int)(sizeof(S.list[0]) / sizeof(S.list[0][0])) - CH;
            if (lane < PAD) S.list[w][cnt + lane] = (unsigned short)CH;
        }
        if (stager && b0 + lane + CH < s1) stage_dma(S.buf[cur ^ 1], 0, id_next, gbase, b, d.N, gP, gQ, gauss);
        id_cur = id_next;
        id_next = stager && b0 + lane + 2 * CH < s1 ? ids[b0 + lane + 2 * CH] : 0u;
        static_assert(MB == 8, "one batch = two 4-entry list words");
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c1);
        SEC_ADD(sec[2], ts_c0b, ts_c1);  // chunk head: quadrant tests + compaction, next DMA issue ([1]: unused)
#endif
        const int lastrel = last - b0;  // this pixel's last contributor, relative to the chunk
        uint2 lraw[2];  // the next step's list words, read one step ahead
        list_raw<MB>(S, w, 0, lraw);
        // one batch: MB list entries evaluated per pixel, their w and u written to this wave's WU image
        auto eval_batch = [&](int kk) {
            int jj8[MB];
            list_decode<MB>(lraw, jj8);
            myj = S.list[w][kk + (lane & (MB - 1))];  // the entry of this lane's batch column
            list_raw<MB>(S, w, kk + MB, lraw);        // in bounds: the list rows hold kRows + MB words
#pragma unroll
            for (int h = 0; h < 2; h++) {
                // a batch with <= 4 listed entries (often a chunk's last) skips its second half, all padding: the
                // stale w / u columns it leaves multiply into the sentinel column CH only (pool k_render_bwd 634 ->
                // 614 us, bitwise equal: profiles/r04/ab_session_f)
                if (h == 1 && kk + 4 >= cnt) break;  // (wave-uniform)
                float al[4], Gw[4];
                float4 cc[4], Pv[4], Qv[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {  // the LDS reads first, one wait (see k_render_fwd)
                    const int j = jj8[4 * h + u];
                    Pv[u] = B.P[j];
                    Qv[u] = B.Q[j];
                    const float4 Rj = B.R[j];
                    cc[u] = make_float4(Rj.x, Rj.y, Rj.z, 0.f);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const bool before_last = jj8[4 * h + u] < lastrel;  // position b0 + jj < last
                    const float4 Pj = Pv[u], Q = Qv[u];
                    cc[u].w = Q.w;
                    const float dx = Pj.x - pfx, dy = Pj.y - pfy;
                    const float lp = fmaf(Q.x * dy, dy, fmaf(fmaf(Pj.w, dy, Pj.z * dx), dx, Q.y));  // as k_render_fwd
                    const float e = __builtin_amdgcn_exp2f(lp);  // opacity G
                    const bool ok = before_last && lp <= Q.y && e >= 1.0f / 255.0f;
                    Gw[u] = ok ? e : 0.f;  // dL/dG = opacity dL/dalpha (0: the entry adds nothing here)
                    al[u] = alpha_cap(Gw[u]);  // (= ok ? alpha_cap(e) : 0, one select less: alpha_cap(0) = 0)
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {  // the prefix recurrences in list order
                    const float alpha = al[u];
                    const float4 cu = cc[u];
                    float cdp = fmaf(cu.x, dp0, fmaf(cu.y, dp1, cu.z * dp2));
                    if (DEPTH) cdp = fmaf(cu.w, dpd, cdp);
                    const float aT = alpha * Tr;
                    const float om = 1.f - alpha;
                    const float inv = __builtin_amdgcn_rcpf(om);  // 1 / (1 - alpha), 1 ulp
                    Erem = fmaf(-aT, cdp, Erem);
                    const float dL_dalpha = fmaf(Tr, cdp, -Erem * inv);
                    Tr = Tr - aT;
                    // w (columns 0..7) and u (8..15), pixel lane at lane ^ wu_swz(column): the swizzled
                    // columns 4..7 and 8..11 are h = 1 for w, h = 0 for u
                    myWU[(4 * h + u) * WU_LD + (h == 1 ? lane_x : lane)] = Gw[u] * dL_dalpha;
                    myWU[(MB + 4 * h + u) * WU_LD + (h == 0 ? lane_x : lane)] = aT;  // (dchannel_dcolor)
                }
            }
        };
        // software-pipelined: batch k's B operand is read from the WU image BEFORE batch k + 1 overwrites it (a
        // wave's LDS operations complete in issue order), so batch k's LDS round trip and moment MFMAs overlap batch
        // k + 1's evaluations instead of stalling the wave between batches
        if (cnt > 0) {
            eval_batch(0);
            for (int kk = 0; kk < cnt; kk += MB) {
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                float xs[2][8];
                read_batch(xs);
                const int col = myj;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // (the reads issue before the next writes)
                if (kk + MB < cnt) eval_batch(kk + MB);
                mfma_batch(xs, col);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        }
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c2);
        SEC_ADD(sec[3], ts_c1, ts_c2);  // the entries loop (evaluation, moments)
#endif
        __syncthreads();
        // moments -> gradient partials, an entry's three groups on three waves at once (thread 64 g + j, entry j):
        // g = 0 mean2D + opacity (moment rows 0..2) and the entry's Gaussian id, g = 1 conic (rows 0..5; a needle's go
        // to rows NV..NV+2 for the fp64 flush), g = 2 colour [+ depth] (the summed hi + lo rows). The partials go to
        // sO, rows q * LS + j.
        float *o = sO;
        if (w < 3 && b0 + lane < s1) {  // (w: wave-uniform)
            const int j = lane;
            auto msum = [&](int row) {
                float v = 0.f;
#pragma unroll
                for (int ww = 0; ww < 4; ww++) v += sAccW[ww][row * LS + j];
                return v;
            };
            if (w == 2) {
#pragma unroll
                for (int qq = 6; qq < NV; qq++) {
                    float v = 0.f;
#pragma unroll
                    for (int ww = 0; ww < 4; ww++) v += sAccW[ww][qq * LS + j];  // (each term: that wave's hi + lo)
                    o[qq * LS + j] = DET ? ldexpf(v, det_s) : v;
                }
            } else {
                const float4 Pj = B.P[j];
                const float4 Qj = B.Q[j];
                float cA, cB, cC, op;  // the upstream conic and opacity
                rec_conic(Pj, Qj, cA, cB, cC, op);
                const float xg = Pj.x - cxT, yg = Pj.y - cyT;
                const float q0 = msum(0), q1 = msum(1), q2 = msum(2);
                DetNorm nm;
                if (DET) nm = det_norm(Pj.z, Pj.w, Qj.x, d.W, d.H);
                if (w == 0) {
                    sId[j] = reinterpret_cast<const unsigned *>(&B.R[j])[3];
                    const float Sx = fmaf(xg, q0, -q1), Sy = fmaf(yg, q0, -q2);
                    float p0 = -ddelx_dx * (cA * Sx + cB * Sy);
                    float p1 = -ddely_dy * (cC * Sy + cB * Sx);
                    float p5 = op > 0.f ? q0 / op : 0.f;
                    if (DET) {
                        p0 = ldexpf(p0, det_s + nm.k[0]);
                        p1 = ldexpf(p1, det_s + nm.k[1]);
                        p5 = ldexpf(p5, det_s);
                    }
                    o[0 * LS + j] = p0;
                    o[1 * LS + j] = p1;
                    o[5 * LS + j] = p5;
                } else {
                    const float q3 = msum(3), q4 = msum(4), q5 = msum(5);
                    const float Sxx = fmaf(xg, fmaf(xg, q0, -2.f * q1), q3);
                    const float Sxy = fmaf(xg, fmaf(yg, q0, -q2), fmaf(-yg, q1, q4));
                    const float Syy = fmaf(yg, fmaf(yg, q0, -2.f * q2), q5);
                    float pc[3] = {-0.5f * Sxx, -0.5f * Sxy, -0.5f * Syy};
                    if (DET) {
#pragma unroll
                        for (int qq = 0; qq < 3; qq++) pc[qq] = ldexpf(pc[qq], det_s + nm.k[2 + qq]);
                    }
                    const bool ndl = !DET && rec_needle(Pj.z, Pj.w, Qj.x);
#pragma unroll
                    for (int qq = 0; qq < 3; qq++) {
                        o[(2 + qq) * LS + j] = ndl ? 0.f : pc[qq];
                        if (!DET) o[(NV + qq) * LS + j] = ndl ? pc[qq] : 0.f;
                    }
                    if (ndl) s_ndl[ci & 1] = 1;  // (benign race: every writer stores 1)
                }
            }
        }
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c3);
        SEC_ADD(sec[4], ts_c2, ts_c3);  // barrier + moments -> partials
#endif
        // the next chunk's DMA and ids have landed before the atomics below go out (they cannot delay it)
        vm_wait_all();
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c3a);
        SEC_ADD(sec[5], ts_c3, ts_c3a);  // DMA wait (and any earlier outstanding vector-memory op of this wave)
#endif
        __syncthreads();
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c3b);
        SEC_ADD(sec[6], ts_c3a, ts_c3b);  // pre-flush barrier
#endif
        // flush: lane -> (entry, value) flat, so one global-atomic wave-instruction covers ~6 contiguous 40-B
        // gradient records instead of 64 scattered rows
        constexpr int FT = 256, FQ = NACC;  // flushing threads; items per entry in the lane mapping
        {
        int ft = tid;
        // the lane's (entry, partial) indices recomputed per chunk: hoisted out of the chunk loop, their 64-bit
        // per-scene accumulator offsets were spilled, and each reload's vmcnt(0) waited for this flush's earlier atomics
        asm volatile("" : "+v"(ft));
#pragma unroll
        for (int it = 0; it < (CH * FQ + FT - 1) / FT; it++) {
            const int f = it * FT + ft;
            const int j = f / FQ, q = f - j * FQ;
            if (q < NV && j < CH && b0 + j < s1) {
                const float a = o[q * LS + j];
                const unsigned gid = sId[j];
                const size_t ai = acc_index(q, gbase + gid, (size_t)b * d.N + gid, (size_t)d.BV * d.N);
                if (a != 0.f) {
                    if (DET) {  // integer adds commute: order-independent sums (a is already in fixed-point units)
                        // (a per-view record takes at most T flushes, a per-scene one (q = 5..8) V * T: with |a|
                        // below the record's bound no sum reaches 2^62 whatever the flushes' signs; the design value
                        // is |a| <= ~2^51 per flush. A flush beyond the bound is counted and k_preproc_bwd then
                        // poisons the call's gradients with NaN instead of returning possibly wrapped sums)
                        if (!(fabsf(a) <= (q >= 5 && q < 9 ? det_lim_s : det_lim_v))) atomicAdd(det_sat, 1u);
                        atomicAdd(reinterpret_cast<unsigned long long *>(accum) + ai,
                                  (unsigned long long)__float2ll_rn(fminf(fmaxf(a, -9.0e18f), 9.0e18f)));
                    } else {
                        atomicAdd(accum + ai, a);
                    }
                }
            }
        }
        if (!DET && s_ndl[ci & 1]) {  // (workgroup-uniform) the chunk's needle conic partials, fp64
            int tt = tid;
            asm volatile("" : "+v"(tt));  // (recomputed here: lane indices hoisted out of the chunk loop spilled)
            for (; tt < 3 * CH; tt += FT) {  // (one pass)
                const int j = tt % CH, c3 = tt / CH;
                const float a = o[(NV + c3) * LS + j];
                if (a != 0.f && b0 + j < s1) {
                    const unsigned gid = sId[j];
                    // (the side block's offset recomputed here from the SGPR dims: a pointer hoisted out of the
                    // chunk loop was kept in VGPRs and spilled)
                    const size_t so = acc_side_offset(d.B, d.V, d.N) / 2;
                    atomicAdd(reinterpret_cast<double *>(accum) + so + (gbase + gid) * 3 + c3, (double)a);
                }
            }
        }
        }  // (flushing waves)
#ifdef LGM_BWD_STAMPS
        SEC_T(ts_c4);
        SEC_ADD(sec[7], ts_c3b, ts_c4);  // gradient atomics (issue)
#endif
    }
#ifdef LGM_BWD_STAMPS
    if (d.counters && lane == 0)
#pragma unroll
        for (int q = 0; q < 8; q++) atomicAdd(&d.counters[q], sec[q]);
#endif
    if (d.counters && tid == 0) {  // work-item timeline (lgm_diag.render_counters): start, end, (length | chunk | tile)
        unsigned long long *o = d.counters + item_stamps + 4 * (size_t)blockIdx.x;
        o[0] = t_item;
        o[1] = __builtin_amdgcn_s_memrealtime();
        o[2] = (unsigned long long)(s1 - s0) | ((unsigned long long)c << 20) | ((unsigned long long)tile << 40);
        o[3] = (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) |        // XCC_ID (the XCD)
               ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) << 8);  // HW_ID
    }
}

// The preprocess backward's recomputation of the forward's projection (make_proj / cov2d / the homogeneous
// divide): FP contraction on and 1-ulp v_rcp_f32 reciprocals. The forward keeps the oracle's bit-exact operation
// order because its integer outputs (radii, tile rects, sort keys) depend on it; here the values only feed
// gradients, and each IEEE division is ~10 VALU of a single thread's serial view chain (k_preproc_bwd 61.1 -> 55.5 us
// on the pool, gradients as accurate or more: profiles/r03/ab_preproc_fast).
__device__ __forceinline__ ProjCtx make_proj_bwd(const float *Vw, float mx, float my, float mz, float fx, float fy,
                                                 float tanx, float tany) {
    ProjCtx P;
    P.t[0] = Vw[0] * mx + Vw[4] * my + Vw[8] * mz + Vw[12];
    P.t[1] = Vw[1] * mx + Vw[5] * my + Vw[9] * mz + Vw[13];
    P.t[2] = Vw[2] * mx + Vw[6] * my + Vw[10] * mz + Vw[14];
    const float limx = 1.3f * tanx, limy = 1.3f * tany, rtz = __builtin_amdgcn_rcpf(P.t[2]);
    const float txtz = P.t[0] * rtz, tytz = P.t[1] * rtz;
    P.t[0] = fminf(limx, fmaxf(-limx, txtz)) * P.t[2];
    P.t[1] = fminf(limy, fmaxf(-limy, tytz)) * P.t[2];
    P.xmul = (txtz < -limx || txtz > limx) ? 0.f : 1.f;
    P.ymul = (tytz < -limy || tytz > limy) ? 0.f : 1.f;
    const float J00 = fx * rtz, J02 = -(fx * P.t[0]) * rtz * rtz;
    const float J11 = fy * rtz, J12 = -(fy * P.t[1]) * rtz * rtz;
#pragma unroll
    for (int r = 0; r < 3; r++) {
        P.T0[r] = Vw[4 * r + 0] * J00 + Vw[4 * r + 2] * J02;
        P.T1[r] = Vw[4 * r + 1] * J11 + Vw[4 * r + 2] * J12;
    }
    return P;
}
__device__ __forceinline__ void cov2d_bwd(const ProjCtx &P, const float c3[6], float &a, float &b, float &c) {
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

// k_preproc_bwd: grid (ceil(N/256), B), block 256. Sums over the scene's views in order (deterministic; the
// order must not depend on the launch's size: a batched pool equals its scenes rendered alone, bit for bit).
// LDSV (scenes of up to PRE_MAXV views): the view / projection matrices staged in LDS once per workgroup, the
// Gaussian, its first view's rect + accumulator row and its scene partials loaded before that staging, and view
// v + 1's rect + row loaded while view v is processed. Without it each view paid its global round trip and then two
// scalar-load round trips for the matrices, in series: pool 57.4 -> 52.3 us, one scene 16.5 -> 14.2 us, outputs
// bitwise equal (profiles/r05/ab_preproc_lds).
constexpr int PRE_MAXV = 32;
template <bool LDSV>
__global__ __launch_bounds__(256) void k_preproc_bwd(Dims d, const float *__restrict__ gauss,
                                                     const float *__restrict__ views,
                                                     const float *__restrict__ projs, const uint2 *__restrict__ rects,
                                                     float *__restrict__ accum, float *__restrict__ d_gauss,
                                                     float *__restrict__ d_means2D, const float4 *__restrict__ gP,
                                                     const float4 *__restrict__ gQ,
                                                     const unsigned *__restrict__ det_max,
                                                     const unsigned *__restrict__ det_sat) {
    const bool det = (d.options & LGM_RENDER_DETERMINISTIC) != 0;
    const int det_s = det ? det_seed_shift(det_max) : 0;
    const bool det_bad = det && *det_sat != 0u;  // a fixed-point flush overflowed (k_render_bwd): poison the call
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = blockIdx.y;
    // diagnostics: workgroup g's start / end in slots [2], [3] of per-tile record g (unused by the other kernels)
    const size_t g_diag = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    const bool stamp = d.counters && threadIdx.x == 0 && g_diag < (size_t)d.BV * d.T;
    if (stamp) d.counters[8 + 8 * g_diag + 2] = __builtin_amdgcn_s_memrealtime();
    const bool live = i < d.N;
    const float fx = d.fx, fy = d.fy, mod = d.mod;
    // float mode: the accumulator row is loaded beside the rect, not after it (one memory round trip per view
    // instead of two; an invisible view's row is uninitialised workspace, loaded and dropped); LDSV: view v + 1's
    // rect and row are loaded while view v is processed
    uint2 r_nx = make_uint2(0u, 0u);
    float2 acc_nx[NACC_V / 2];
    auto load_view = [&](int v) {
        const size_t k = ((size_t)b * d.V + v) * d.N + i;
        r_nx = rects[k];
        if (!det) {
            const float2 *acc2 = reinterpret_cast<const float2 *>(accum + k * NACC_V);
#pragma unroll
            for (int q = 0; q < NACC_V / 2; q++) acc_nx[q] = acc2[q];
        }
    };
    float g[14];
    const size_t ks = (size_t)d.BV * d.N * NACC_V + ((size_t)b * d.N + i) * NACC_S;  // view-independent partials
    float4 acc_s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (LDSV && live) {  // the Gaussian, its first view and its scene partials in flight during the staging
        load_gaussian(gauss + ((size_t)b * d.N + i) * 14, g);
        if (d.V > 0) load_view(0);
        if (!det) acc_s = *reinterpret_cast<const float4 *>(accum + ks);
    }
    // LDSV: the scene's view and projection matrices in LDS, loaded once by the workgroup, so the view loop's reads
    // of them are LDS round trips instead of scalar loads issued after each view's global loads
    __shared__ float s_vp[LDSV ? PRE_MAXV : 1][32];
    if constexpr (LDSV) {
        for (int t = threadIdx.x; t < 32 * d.V; t += blockDim.x) {
            const int v = t >> 5, e = t & 31, bv = b * d.V + v;
            s_vp[v][e] = e < 16 ? views[16 * bv + e] : projs[16 * bv + e - 16];
        }
        __syncthreads();
    }
    if (!live) return;
    if (!LDSV) load_gaussian(gauss + ((size_t)b * d.N + i) * 14, g);
    float R[3][3];
    const float q4[4] = {g[7], g[8], g[9], g[10]};
    quat_rot(q4, R);
    const float s[3] = {mod * g[4], mod * g[5], mod * g[6]};
    float c3[6];
    cov3d(s, R, c3);
    const float Sg[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
    float dmean[3] = {0, 0, 0}, dcov[6] = {0, 0, 0, 0, 0, 0}, dop = 0, dcol[3] = {0, 0, 0};
    for (int v = 0; v < d.V; v++) {
        const int bv = b * d.V + v;
        const size_t k = (size_t)bv * d.N + i;
        if (!LDSV) load_view(v);
        const uint2 r = r_nx;
        float2 acc_e[NACC_V / 2];
#pragma unroll
        for (int q = 0; q < NACC_V / 2; q++) acc_e[q] = acc_nx[q];
        if (LDSV && v + 1 < d.V) load_view(v + 1);
        const bool vis = (r.x & 0xffff) != (r.y & 0xffff);
        if (!vis) {
            if (d_means2D) { d_means2D[2 * k] = 0.f; d_means2D[2 * k + 1] = 0.f; }
            continue;
        }
        float acc[NACC_V];
        if (det) {  // back from fixed point: the same normalisers k_render_bwd derived from this record
            const longlong2 *acc2 = reinterpret_cast<const longlong2 *>(accum) + k * (NACC_V / 2);
            const float4 rp = gP[k];
            const DetNorm nm = det_norm(rp.z, rp.w, gQ[k].x, d.W, d.H);
#pragma unroll
            for (int q = 0; q < NACC_V / 2; q++) {
                const longlong2 a = acc2[q];
                acc[2 * q] = (float)ldexp((double)a.x, -(det_s + nm.k[2 * q]));
                acc[2 * q + 1] = (float)ldexp((double)a.y, -(det_s + nm.k[2 * q + 1]));
            }
        } else {  // (zeroed by the forward's epilogue; see LGM_RENDER_BACKWARD_AGAIN)
#pragma unroll
            for (int q = 0; q < NACC_V / 2; q++) {
                acc[2 * q] = acc_e[q].x;
                acc[2 * q + 1] = acc_e[q].y;
            }
        }
        if (!det && (r.y >> 31)) {  // a needle: its conic partials were summed in fp64
            const double *sd = reinterpret_cast<const double *>(accum + acc_side_offset(d.B, d.V, d.N)) + k * 3;
            acc[2] = (float)sd[0];
            acc[3] = (float)sd[1];
            acc[4] = (float)sd[2];
        }
        const float dm2x = acc[0], dm2y = acc[1];
        const float dcx = acc[2], dcy = acc[3], dcz = acc[4];
        const float ddep = acc[5];
        if (d_means2D) { d_means2D[2 * k] = dm2x; d_means2D[2 * k + 1] = dm2y; }
        const float *Vw = LDSV ? s_vp[v] : views + 16 * bv;
        const float *Pm = LDSV ? s_vp[v] + 16 : projs + 16 * bv;
        // ---- cov2D backward
        const ProjCtx Pc = make_proj_bwd(Vw, g[0], g[1], g[2], fx, fy, d.tanx, d.tany);
        float a, bb, c;
        cov2d_bwd(Pc, c3, a, bb, c);
        const float denom = a * c - bb * bb;
        const float denom2inv = __builtin_amdgcn_rcpf((denom * denom) + 0.0000001f);
        float dL_da = 0, dL_db = 0, dL_dc = 0;
        if (denom2inv != 0) {
            dL_da = denom2inv * (-c * c * dcx + 2 * bb * c * dcy + (denom - a * c) * dcz);
            dL_dc = denom2inv * (-a * a * dcz + 2 * a * bb * dcy + (denom - a * c) * dcx);
            dL_db = denom2inv * 2 * (bb * c * dcx - (denom + 2 * bb * bb) * dcy + a * bb * dcz);
            const float *t0 = Pc.T0, *t1 = Pc.T1;
            dcov[0] += (t0[0] * t0[0] * dL_da + t0[0] * t1[0] * dL_db + t1[0] * t1[0] * dL_dc);
            dcov[3] += (t0[1] * t0[1] * dL_da + t0[1] * t1[1] * dL_db + t1[1] * t1[1] * dL_dc);
            dcov[5] += (t0[2] * t0[2] * dL_da + t0[2] * t1[2] * dL_db + t1[2] * t1[2] * dL_dc);
            dcov[1] += 2 * t0[0] * t0[1] * dL_da + (t0[0] * t1[1] + t0[1] * t1[0]) * dL_db + 2 * t1[0] * t1[1] * dL_dc;
            dcov[2] += 2 * t0[0] * t0[2] * dL_da + (t0[0] * t1[2] + t0[2] * t1[0]) * dL_db + 2 * t1[0] * t1[2] * dL_dc;
            dcov[4] += 2 * t0[2] * t0[1] * dL_da + (t0[1] * t1[2] + t0[2] * t1[1]) * dL_db + 2 * t1[1] * t1[2] * dL_dc;
        }
        float dT0[3], dT1[3];
#pragma unroll
        for (int kk = 0; kk < 3; kk++) {
            const float s0 = Pc.T0[0] * Sg[kk][0] + Pc.T0[1] * Sg[kk][1] + Pc.T0[2] * Sg[kk][2];
            const float s1 = Pc.T1[0] * Sg[kk][0] + Pc.T1[1] * Sg[kk][1] + Pc.T1[2] * Sg[kk][2];
            dT0[kk] = 2 * s0 * dL_da + s1 * dL_db;
            dT1[kk] = 2 * s1 * dL_dc + s0 * dL_db;
        }
        const float dJ00 = Vw[0] * dT0[0] + Vw[4] * dT0[1] + Vw[8] * dT0[2];
        const float dJ02 = Vw[2] * dT0[0] + Vw[6] * dT0[1] + Vw[10] * dT0[2];
        const float dJ11 = Vw[1] * dT1[0] + Vw[5] * dT1[1] + Vw[9] * dT1[2];
        const float dJ12 = Vw[2] * dT1[0] + Vw[6] * dT1[1] + Vw[10] * dT1[2];
        const float tz = __builtin_amdgcn_rcpf(Pc.t[2]), tz2 = tz * tz, tz3 = tz2 * tz;
        const float dtx = Pc.xmul * -fx * tz2 * dJ02;
        const float dty = Pc.ymul * -fy * tz2 * dJ12;
        const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2 * fx * Pc.t[0]) * tz3 * dJ02 +
                          (2 * fy * Pc.t[1]) * tz3 * dJ12;
        dmean[0] += Vw[0] * dtx + Vw[1] * dty + Vw[2] * dtz;
        dmean[1] += Vw[4] * dtx + Vw[5] * dty + Vw[6] * dtz;
        dmean[2] += Vw[8] * dtx + Vw[9] * dty + Vw[10] * dtz;
        // ---- perspective-divide backward
        float hom[4];
        hom[0] = Pm[0] * g[0] + Pm[4] * g[1] + Pm[8] * g[2] + Pm[12];
        hom[1] = Pm[1] * g[0] + Pm[5] * g[1] + Pm[9] * g[2] + Pm[13];
        hom[3] = Pm[3] * g[0] + Pm[7] * g[1] + Pm[11] * g[2] + Pm[15];
        const float m_w = __builtin_amdgcn_rcpf(hom[3] + 0.0000001f);
        const float mul1 = hom[0] * m_w * m_w;
        const float mul2 = hom[1] * m_w * m_w;
        dmean[0] += (Pm[0] * m_w - Pm[3] * mul1) * dm2x + (Pm[1] * m_w - Pm[3] * mul2) * dm2y;
        dmean[1] += (Pm[4] * m_w - Pm[7] * mul1) * dm2x + (Pm[5] * m_w - Pm[7] * mul2) * dm2y;
        dmean[2] += (Pm[8] * m_w - Pm[11] * mul1) * dm2x + (Pm[9] * m_w - Pm[11] * mul2) * dm2y;
        // ---- depth backward (exact row 2 of the view matrix)
        dmean[0] += Vw[2] * ddep;
        dmean[1] += Vw[6] * ddep;
        dmean[2] += Vw[10] * ddep;
    }
    {  // the scene's view-independent partials (opacity, colour), summed over its views by the backward's atomics
        if (det) {
            const long long *a = reinterpret_cast<const long long *>(accum) + ks;
            dop = (float)ldexp((double)a[0], -det_s);
#pragma unroll
            for (int q = 0; q < 3; q++) dcol[q] = (float)ldexp((double)a[1 + q], -det_s);
        } else {
            const float4 a = LDSV ? acc_s : *reinterpret_cast<const float4 *>(accum + ks);
            dop = a.x;
            dcol[0] = a.y; dcol[1] = a.z; dcol[2] = a.w;
        }
    }
    // ---- cov3D backward, once on the view-summed dL/dcov3D (linear, so equal to the per-view sum)
    const float dS[3][3] = {{dcov[0], 0.5f * dcov[1], 0.5f * dcov[2]},
                            {0.5f * dcov[1], dcov[3], 0.5f * dcov[4]},
                            {0.5f * dcov[2], 0.5f * dcov[4], dcov[5]}};
    float dM[3][3];  // dM[c][r] = 2 s_r sum_k R[k][r] dS[c][k]   (glm M = S*R, M[k][r] = s_r R[k][r])
#pragma unroll
    for (int cc = 0; cc < 3; cc++)
#pragma unroll
        for (int rr = 0; rr < 3; rr++)
            dM[cc][rr] = 2.0f * s[rr] * (R[0][rr] * dS[cc][0] + R[1][rr] * dS[cc][1] + R[2][rr] * dS[cc][2]);
    float dscale[3], dd[3][3];
#pragma unroll
    for (int ii = 0; ii < 3; ii++) {
        dscale[ii] = (R[0][ii] * dM[0][ii] + R[1][ii] * dM[1][ii] + R[2][ii] * dM[2][ii]) * mod;
#pragma unroll
        for (int rr = 0; rr < 3; rr++) dd[ii][rr] = dM[rr][ii] * s[ii];  // dL_dMt[ii][rr] * s_ii
    }
    const float r_ = g[7], x = g[8], y = g[9], z = g[10];
    float dq[4];
    dq[0] = 2 * z * (dd[0][1] - dd[1][0]) + 2 * y * (dd[2][0] - dd[0][2]) + 2 * x * (dd[1][2] - dd[2][1]);
    dq[1] = 2 * y * (dd[1][0] + dd[0][1]) + 2 * z * (dd[2][0] + dd[0][2]) + 2 * r_ * (dd[1][2] - dd[2][1]) -
            4 * x * (dd[2][2] + dd[1][1]);
    dq[2] = 2 * x * (dd[1][0] + dd[0][1]) + 2 * r_ * (dd[2][0] - dd[0][2]) + 2 * z * (dd[1][2] + dd[2][1]) -
            4 * y * (dd[2][2] + dd[0][0]);
    dq[3] = 2 * r_ * (dd[0][1] - dd[1][0]) + 2 * x * (dd[2][0] + dd[0][2]) + 2 * y * (dd[1][2] + dd[2][1]) -
            4 * z * (dd[1][1] + dd[0][0]);
    float *o = d_gauss + ((size_t)b * d.N + i) * 14;
    const float out[14] = {dmean[0], dmean[1], dmean[2], dop, dscale[0], dscale[1], dscale[2],
                           dq[0], dq[1], dq[2], dq[3], dcol[0], dcol[1], dcol[2]};
    float2 *o2 = reinterpret_cast<float2 *>(o);
    const float qnan = __builtin_nanf("");
#pragma unroll
    for (int kk = 0; kk < 7; kk++)
        o2[kk] = det_bad ? make_float2(qnan, qnan) : make_float2(out[2 * kk], out[2 * kk + 1]);
    if (stamp) d.counters[8 + 8 * g_diag + 3] = __builtin_amdgcn_s_memrealtime();
}

}  // namespace

// ------------------------------------------------------------------------------------------------------------
int launch_render_fwd(const Dims &d, const float *gaussians, const float *bg, float *image, float *depth,
                      float *alpha, char *ws, const Layout &L, hipStream_t st) {
    const bool small = d.BV * d.T <= FWD_SMALL_TILES;
    auto fwd = (d.options & LGM_RENDER_FUSED_LOSS) ? (small ? k_render_fwd<true, 8> : k_render_fwd<true, FWD_FU>)
                                                   : (small ? k_render_fwd<false, 8> : k_render_fwd<false, FWD_FU>);
    LGM_LAUNCH("k_render_fwd", st, (fwd<<<(unsigned)(d.BV * d.T), 256, 0, st>>>(
                                       d, L.slot ? (long long)d.N : -1LL, (const int *)(ws + L.tile_start),
                                       (const int *)(ws + L.tile_count), (const unsigned long long *)(ws + L.pairs),
                                       (const float4 *)(ws + L.gP), (const float4 *)(ws + L.gQ), gaussians, bg,
                                       image, depth, alpha,
                                       (float *)(ws + L.final_T), (int *)(ws + L.n_contrib), (int *)(ws + L.wlast),
                                       (unsigned char *)(ws + L.cmask), (float4 *)(ws + L.cfin),
                                       (float *)(ws + L.ck), (int2 *)(ws + L.cklist), (int *)(ws + L.nck),
                                       (unsigned *)(ws + L.misc) + 4, L.ck_region, (float4 *)(ws + L.accum),
                                       // (rounded up to 16 B: the tail lands in the layout's
                                       // alignment padding, or on the fp64 side block's first entry, zeroed anyway)
                                       (long long)(((d.options & LGM_RENDER_DETERMINISTIC ? 8 : 4) * acc_elems(d.B, d.V, d.N) + 15) / 16))));
    return LGM_OK;
}

int launch_loss_reduce(const Dims &d, char *ws, const Layout &L, hipStream_t st) {
    const double P = (double)d.H * d.W;
    const int M = d.BV * d.T, G = (M + LR_TILES - 1) / LR_TILES;
    LGM_LAUNCH("k_loss_reduce", st, (k_loss_reduce<<<G, LR_THREADS, 0, st>>>(
                                        M, (const float2 *)(ws + L.lossp), 3.0 * d.BV * P, d.BV * P,
                                        (double2 *)(ws + L.lossw), (unsigned *)(ws + L.misc) + 12, d.loss_out)));
    return LGM_OK;
}

int launch_render_bwd(const Dims &d, const float *gaussians, const float *cam_view, const float *cam_view_proj,
                      const float *bg, const float *d_image, const float *d_depth, const float *d_alpha,
                      float *d_gaussians, float *d_means2D, char *ws, const Layout &L, hipStream_t st) {
    // the accumulators were zeroed by the forward (k_render_fwd's epilogue); a repeated backward of the same forward
    // clears what the previous one left
    if ((d.options & LGM_RENDER_BACKWARD_AGAIN) &&
        hipMemsetAsync(ws + L.accum, 0, (d.options & LGM_RENDER_DETERMINISTIC)
                                            ? acc_elems(d.B, d.V, d.N) * 8
                                            : acc_side_offset(d.B, d.V, d.N) * 4 + (size_t)d.BV * d.N * 24,
                       st) != hipSuccess) {
        set_error("hipMemsetAsync failed");
        return LGM_E_HIP;
    }
    const bool loss = (d.options & LGM_RENDER_FUSED_LOSS) != 0, det = (d.options & LGM_RENDER_DETERMINISTIC) != 0;
    unsigned *det_max = (unsigned *)(ws + L.detmax);
    if (det) {  // the call's fixed-point scale: max |dL/dpixel| over every seed (k_det_seed_max)
        if (hipMemsetAsync(det_max, 0, DET_SLOTS * 4, st) != hipSuccess) {
            set_error("hipMemsetAsync failed");
            return LGM_E_HIP;
        }
        auto smax = loss ? (d_depth ? k_det_seed_max<true, true> : k_det_seed_max<false, true>)
                         : (d_depth ? k_det_seed_max<true, false> : k_det_seed_max<false, false>);
        LGM_LAUNCH("k_det_seed_max", st, (smax<<<(unsigned)min(d.BV * d.T, DET_MAX_WGS), 256, 0, st>>>(
                                             d, (const float *)(ws + L.final_T), bg, (const float4 *)(ws + L.cfin),
                                             d_image, d_depth, d_alpha, (const unsigned char *)(ws + L.cmask),
                                             det_max, (unsigned *)(ws + L.misc) + 13)));
    }
    auto pick = [&](auto depth_tag) {
        constexpr bool DP = decltype(depth_tag)::value;
        return loss ? (det ? k_render_bwd<DP, true, true> : k_render_bwd<DP, true, false>)
                    : (det ? k_render_bwd<DP, false, true> : k_render_bwd<DP, false, false>);
    };
    auto bwd = d_depth ? pick(std::true_type{}) : pick(std::false_type{});
    // work items: chunk 0 of every tile, then one per checkpoint slot (unused slots exit at once)
    const int M = d.BV * d.T, Mp = round8(M);
    LGM_LAUNCH("k_render_bwd", st, (bwd<<<(unsigned)(Mp + L.ck_slots), 256, 0, st>>>(
                                       d, L.slot ? (long long)d.N : -1LL, (const int *)(ws + L.tile_start),
                                       (const int *)(ws + L.tile_count), (const unsigned long long *)(ws + L.pairs),
                                       (const float4 *)(ws + L.gP), (const float4 *)(ws + L.gQ), gaussians, bg,
                                       (const float *)(ws + L.final_T), (const int *)(ws + L.n_contrib),
                                       (const int *)(ws + L.wlast), (const float4 *)(ws + L.cfin), (const float *)(ws + L.ck),
                                       (const int2 *)(ws + L.cklist), (const int *)(ws + L.nck),
                                       (const unsigned *)(ws + L.misc) + 4, L.ck_region, d_image, d_depth, d_alpha,
                                       (const unsigned char *)(ws + L.cmask), (float *)(ws + L.accum), det_max,
                                       (unsigned *)(ws + L.misc) + 13,
                                       // (debug counters: after the per-tile and per-binning-workgroup records)
                                       8 + 8LL * d.BV * d.T + 8LL * d.BV * ((d.N + 511) / 512))));
    dim3 grid((d.N + 255) / 256, d.B);
    auto pre = d.V <= PRE_MAXV ? k_preproc_bwd<true> : k_preproc_bwd<false>;
    LGM_LAUNCH("k_preproc_bwd", st, (pre<<<grid, 256, 0, st>>>(d, gaussians, cam_view, cam_view_proj,
                                                                        (const uint2 *)(ws + L.rects),
                                                                        (float *)(ws + L.accum), d_gaussians,
                                                                        d_means2D, (const float4 *)(ws + L.gP),
                                                                        (const float4 *)(ws + L.gQ), det_max,
                                                                        (const unsigned *)(ws + L.misc) + 13)));
    return LGM_OK;
}

}  // namespace lgm
