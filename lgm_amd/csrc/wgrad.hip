// lgm_amd/csrc/wgrad.hip -- the weight-gradient GEMM of MVAttention's qkv / proj Linears (include/lgm_linear.h):
// dw = dy^T x and db = colsum(dy) over K = every token of the batch (core/attention.py:46,48 under bf16 autocast).
//
// The shape is what the library GEMM handles worst: a short, wide output (1,536 x 512 or 512 x 512) and a reduction
// over K = 32,768 tokens. hipBLASLt ran it on 55 / 57 workgroups of a 256-CU part at 240 / ~100 TFLOP/s
// (profiles/r05/final6/kernel_stats_by_grid.txt). Here:
//   * split-K over the whole chip: 128 x 128 output tiles, each K range split S ways so that tiles * S fills the 512
//     workgroup slots (2 per CU); each workgroup writes an fp32 partial, and k_wgrad_reduce sums the S partials of
//     every output in split order (deterministic) and scatters the tile into dw;
//   * both operands are K-major in memory (token rows), so both MFMA operands come from the hardware transposed LDS
//     read (ds_read_b64_tr_b16): a 32-row stage of dy and of x is copied into LDS by LDS DMA (global_load_lds, no
//     staging registers) as 256-B rows whose 32-B chunks are XOR-swizzled by the row (chunk c of row r at c ^ (r & 7)),
//     which puts the 8 rows of every 32-lane half of a transposed read on distinct banks;
//   * 64-row stages, double-buffered (the next stage's DMA in flight during the current one's MFMAs), one barrier per
//     stage (fragments of stage j + 1 read during stage j's MFMAs, software-pipelined at 210 VGPRs, measured slower
//     with 32-row stages: 59.7 -> 64-65 us per launch, profiles/r06/ab_wgrad_pipe);
//   * 4 waves per workgroup in 2 x 2, each a 64 x 64 block = 16 v_mfma_f32_16x16x32 per 32-row K step;
//   * db on the same MFMAs: the dy fragment times a ones operand gives the column sums; each workgroup adds the
//     stages whose index is congruent to its column tile (so the work is spread over the column tiles), and the
//     reduce kernel sums those partials in a fixed order too.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "lgm_attn.h"
#include "lgm_linear.h"

namespace lgm {
namespace wg {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef short s4v __attribute__((__vector_size__(8)));
typedef __attribute__((ext_vector_type(8))) short s8v;

constexpr int BM = 128, BN = 128;  // output tile (dw rows x columns) of one workgroup
// K rows per stage: two 32-row MFMA K steps per barrier, double-buffered (one stage in flight). Against 32-row stages in
// a 4-deep ring (three in flight): qkv 72.5 / 73.7 -> 65.7 / 65.8 us, proj (bias) 32.0 / 32.4 -> 29.4 / 30.2 us at the
// bench level (profiles/r06/ab_wgrad_bk64): half the barriers and waits per MFMA
constexpr int BK = 64;
constexpr int DPS = BK / 8;        // LDS-DMA pieces per wave per stage (both operands)
constexpr int RING = BK == 32 ? 4 : 2;  // LDS stages; RING - 1 in flight (with 32-row stages, 3 stages at 3 workgroups
                                        // per CU measured slower: k_wgrad 65 -> 68 us, profiles/r06/ab_wgrad_ring)
constexpr int THREADS = 256;
constexpr int IMG = BK * 256;      // bytes of one operand's stage image (BK rows x 128 16-bit columns)
constexpr int WPE = 2;             // workgroups (= waves per SIMD) per CU: 64 KB of LDS each
// workgroup slots the split targets (one round at 2 per CU). Targeting 256 (one per CU) or 1,024 (two rounds)
// measured slower at both Linears (bench level qkv 70.8 -> 111 / 72 us, proj 30 -> 41 / 34 us; profiles/r06/wgrad_split)
constexpr int SLOTS = 256 * WPE;
constexpr int FRAGS = 16;          // 16 x 16 accumulator blocks per wave
constexpr int DBT = 8;             // k_wgrad_reduce lanes per bias-gradient row

template <int DT> struct Op;
template <> struct Op<LGM_ATTN_BF16> { using V8 = bf16x8; static constexpr short ONE = 0x3f80; };
template <> struct Op<LGM_ATTN_F16> { using V8 = f16x8; static constexpr short ONE = 0x3c00; };

template <int DT> __device__ __forceinline__ f32x4 mfma(typename Op<DT>::V8 a, typename Op<DT>::V8 b, f32x4 c) {
    if constexpr (DT == LGM_ATTN_BF16) return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ unsigned lds_addr32(const void *p) {
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
// LDS DMA (global_load_lds_dwordx4: lane i's 16 B land at M0 + 16 i). Inline asm so that the compiler's waitcnt pass
// does not tie later LDS reads to the pending copy; completion is ordered by the counted vmcnt waits + a barrier.
__device__ __forceinline__ void lds_dma16(const void *src, unsigned lds_base) {
    const unsigned m = __builtin_amdgcn_readfirstlane(lds_base);
    unsigned saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(saved)
                 : "s"(m), "v"(src)
                 : "memory");
}
// s_waitcnt vmcnt(n) (n <= 15), leaving lgkmcnt / expcnt alone
template <int n> __device__ __forceinline__ void vm_wait() { __builtin_amdgcn_s_waitcnt(0x0F70 | n); }

// One operand's stage (rows k0 .. k0 + 31, columns col0 .. col0 + 127) into its swizzled image: wave w copies the
// pieces 2w and 2w + 1 (4 rows of 256 B each). Columns past ncols read the last 16 B of the row (finite; only outputs
// past M / N, which are never stored, see them). Rows past kend must be ZERO (they would add to valid outputs): the
// one stage that reaches past kend (the last of the last split) is staged through registers with zero fill instead.
template <bool TAIL>
__device__ __forceinline__ void stage(const uint16_t *__restrict__ src, long long ld, int k0, int kend, int col0,
                                      int ncols, unsigned char *img) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int q = 0; q < BK / 16; q++) {
        const int p = (BK / 16) * w + q, row = 4 * p + (lane >> 4), slot = lane & 15;
        const int lc = (slot >> 1) ^ (row & 7);                // logical 32-B chunk stored at physical chunk slot / 2
        const int col = min(col0 + 16 * lc + 8 * (slot & 1), ncols - 8);
        const uint16_t *s = src + (long long)(k0 + row) * ld + col;
        if (!TAIL) {
            lds_dma16(s, lds_addr32(img) + 1024u * p);
        } else {
            uint4 v = make_uint4(0u, 0u, 0u, 0u);
            if (k0 + row < kend) v = *reinterpret_cast<const uint4 *>(s);
            *reinterpret_cast<uint4 *>(img + 1024 * p + 16 * lane) = v;
        }
    }
}

// The 16x16x32 operand of 16 columns (logical chunk c) over the stage's 32 rows, by two transposed reads: lane
// (g, i) receives column 16 c + i at rows 4g .. 4g + 3 and 16 + 4g .. 16 + 4g + 3 (the same row order for both
// operands of a product, so the K sum is complete).
template <int DT>
__device__ __forceinline__ typename Op<DT>::V8 frag(const unsigned char *img, int c, int lane) {
    const int g = lane >> 4, i = lane & 15, r = 4 * g + (i >> 2);
    const unsigned char *p = img + r * 256 + ((c ^ (r & 7)) << 5) + 8 * (i & 3);  // (row r + 16: the same swizzle)
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(p + 16 * 256));
    const s8v v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(typename Op<DT>::V8, v);
}

// XCD-grouped work order (render_common.h xcd_item): the workgroups of one XCD take a contiguous range of the
// (split, tile) items, i.e. mostly every tile of one K range, so the tiles that read the same dy / x rows share an L2.
__device__ __forceinline__ int xcd_item(int b, int M) {
    const int q = M >> 3, r = M & 7, g = b & 7, i = b >> 3;
    return (g < r ? g * (q + 1) : r * (q + 1) + (g - r) * q) + i;
}

// k_wgrad: grid (tiles * S), block 256, 64 KB of LDS. Workgroup -> (split s, tile (mt, nt)); split s covers the
// stages [s q + min(s, r), ...) of the ceil(K / 32) stages (q, r = divmod(stages, S)).
template <int DT>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(WPE))) void k_wgrad(
    int K, int M, int N, const uint16_t *__restrict__ dy, long long ld_dy, const uint16_t *__restrict__ x,
    long long ld_x, int S, int NT, f32x4 *__restrict__ part, float *__restrict__ dbpart, int Mp) {
    __shared__ __attribute__((aligned(1024))) unsigned char sA[RING][IMG];
    __shared__ __attribute__((aligned(1024))) unsigned char sB[RING][IMG];
    const int tiles = gridDim.x / S;
    const int item = xcd_item(blockIdx.x, gridDim.x);
    const int s = item / tiles, tile = item - s * tiles, mt = tile / NT, nt = tile - mt * NT;
    const int m0 = mt * BM, n0 = nt * BN;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, wm = w >> 1, wn = w & 1;
    const int wn_u = __builtin_amdgcn_readfirstlane(w) & 1;  // (wave-uniform copy of wn: a scalar branch)
    const int nst_all = (K + BK - 1) / BK, q = nst_all / S, r = nst_all - q * S;
    const int st0 = s * q + min(s, r), nst = q + (s < r ? 1 : 0);
    const bool want_db = dbpart != nullptr;
    using V8 = typename Op<DT>::V8;
    const s8v ones_s = {Op<DT>::ONE, Op<DT>::ONE, Op<DT>::ONE, Op<DT>::ONE,
                        Op<DT>::ONE, Op<DT>::ONE, Op<DT>::ONE, Op<DT>::ONE};
    const V8 ones = __builtin_bit_cast(V8, ones_s);

    f32x4 acc[FRAGS], dbacc[2];
#pragma unroll
    for (int f = 0; f < FRAGS; f++) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
    dbacc[0] = dbacc[1] = f32x4{0.f, 0.f, 0.f, 0.f};

    // stage j of this split (rows k0 = (st0 + j) * BK ..) into ring slot j % RING; the stage that reaches past K is
    // the last one, staged through registers (its loads are waited for by the compiler before the LDS stores, which
    // also drains every earlier DMA: the counted waits below stay correct)
    auto issue = [&](int j) {
        const int k0 = (st0 + j) * BK, b = j % RING;
        if (k0 + BK <= K) {
            stage<false>(dy, ld_dy, k0, K, m0, M, sA[b]);
            stage<false>(x, ld_x, k0, K, n0, N, sB[b]);
        } else {
            stage<true>(dy, ld_dy, k0, K, m0, M, sA[b]);
            stage<true>(x, ld_x, k0, K, n0, N, sB[b]);
        }
    };
#pragma unroll
    for (int j = 0; j < RING - 1; j++)
        if (j < nst) issue(j);
    for (int j = 0; j < nst; j++) {
        // stage j has landed once at most the DMAs of the stages issued after it (4 per stage per wave) are pending
        const int ahead = min(nst - 1, j + RING - 2) - j;
        if (ahead >= 2) vm_wait<2 * DPS>();
        else if (ahead == 1) vm_wait<DPS>();
        else vm_wait<0>();
        __syncthreads();  // every wave's copies of stage j have landed; slot (j - 1) % RING is free
        if (j + RING - 1 < nst) issue(j + RING - 1);
#pragma unroll
        for (int kk = 0; kk < BK / 32; kk++) {  // the stage's 32-row K steps
            const unsigned char *a_img = sA[j % RING] + kk * 32 * 256, *b_img = sB[j % RING] + kk * 32 * 256;
            V8 fa[4], fb[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                fa[u] = frag<DT>(a_img, 4 * wm + u, lane);
                fb[u] = frag<DT>(b_img, 4 * wn + u, lane);
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int v = 0; v < 4; v++) acc[4 * u + v] = mfma<DT>(fa[u], fb[v], acc[4 * u + v]);
            // (static fragment indices under a wave-uniform branch: indexing fa by 2 * wn, a VGPR value to the
            // compiler, became a ~1,500-instruction select chain per stage and doubled the launch: 30 -> 60 us at the
            // proj level)
            if (want_db && ((st0 + j) * (BK / 32) + kk) % NT == nt) {
                if (wn_u == 0) {
                    dbacc[0] = mfma<DT>(fa[0], ones, dbacc[0]);
                    dbacc[1] = mfma<DT>(fa[1], ones, dbacc[1]);
                } else {
                    dbacc[0] = mfma<DT>(fa[2], ones, dbacc[0]);
                    dbacc[1] = mfma<DT>(fa[3], ones, dbacc[1]);
                }
            }
        }
    }
    // fp32 partials in fragment order: one float4 per lane per fragment, 1 KiB per wave-instruction
    f32x4 *pp = part + ((size_t)(s * tiles + tile) * 4 + w) * FRAGS * 64 + lane;
#pragma unroll
    for (int f = 0; f < FRAGS; f++) pp[f * 64] = acc[f];
    if (want_db && (lane & 15) == 0) {  // lane (g, 0) holds the sums of rows 4g .. 4g + 3 of each 16-row block
        float *dp = dbpart + (size_t)(nt * S + s) * Mp + m0 + 64 * wm + 4 * (lane >> 4);
#pragma unroll
        for (int h = 0; h < 2; h++) *reinterpret_cast<f32x4 *>(dp + 16 * (2 * wn + h)) = dbacc[h];
    }
}

// k_wgrad_reduce: grid (ceil(tiles * 4096 / 256) + [ceil(Mp / 256)]), block 256. One thread per (tile, wave,
// fragment, lane) float4 position: the S partials summed in split order (up to 16 loads in flight), the 4 values scattered to
// dw; then (db) DBT threads per row: the NT * S column-sum partials in a fixed order.
__global__ __launch_bounds__(256) void k_wgrad_reduce(int M, int N, int S, int NT, int tiles,
                                                      const f32x4 *__restrict__ part, const float *__restrict__ dbpart,
                                                      int Mp, float *__restrict__ dw, float *__restrict__ db) {
    const long long npos = (long long)tiles * 4 * FRAGS * 64;
    const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
    if (p < npos) {
        f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < S; s += 16) {  // up to 16 partials in flight per thread (S <= 16: one round trip)
            f32x4 v[16];
#pragma unroll
            for (int u = 0; u < 16; u++)
                v[u] = s + u < S ? part[(size_t)(s + u) * npos + p] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 16; u++)
                if (s + u < S) sum += v[u];  // (split order)
        }
        const int lane = (int)(p & 63), f = (int)((p >> 6) % FRAGS), w = (int)((p >> 10) & 3);
        const int tile = (int)(p >> 12), mt = tile / NT, nt = tile - mt * NT;
        const int a = f >> 2, b = f & 3, g = lane >> 4, j = lane & 15;
        const int m = mt * BM + 64 * (w >> 1) + 16 * a + 4 * g, n = nt * BN + 64 * (w & 1) + 16 * b + j;
        if (n < N) {
#pragma unroll
            for (int e = 0; e < 4; e++)
                if (m + e < M) dw[(size_t)(m + e) * N + n] = sum[e];
        }
        return;
    }
    if (!db) return;
    // db: DBT lanes per row (adjacent lanes), each summing a contiguous eighth of the NT * S partials in order (all
    // its loads in flight), then a fixed xor tree over the DBT lanes: deterministic. (One thread per row summing all
    // 128 partials of the bench's proj level one load at a time took 34 us.)
    const long long q = p - ((npos + 255) / 256) * 256;
    const int m = (int)(q / DBT), part8 = (int)(q % DBT);
    const int nq = NT * S, per = (nq + DBT - 1) / DBT, q0 = part8 * per, q1 = min(nq, q0 + per);
    float v = 0.f;
    if (m < M) {
        for (int qq = q0; qq < q1; qq += 16) {
            float t[16];
#pragma unroll
            for (int u = 0; u < 16; u++) t[u] = qq + u < q1 ? dbpart[(size_t)(qq + u) * Mp + m] : 0.f;
#pragma unroll
            for (int u = 0; u < 16; u++) v += t[u];
        }
    }
#pragma unroll
    for (int o = 1; o < DBT; o <<= 1) v += __shfl_xor(v, o, 64);  // (the same tree in every lane)
    if (m < M && part8 == 0) db[m] = v;
}

struct Plan {
    int MT, NT, tiles, S, Mp;
    size_t part_bytes, db_bytes;
};
inline Plan plan(int K, int M, int N, bool want_db) {
    Plan P;
    P.MT = (M + BM - 1) / BM;
    P.NT = (N + BN - 1) / BN;
    P.tiles = P.MT * P.NT;
    const int nst = (K + BK - 1) / BK;
    P.S = max(1, min(SLOTS / max(1, P.tiles), nst / 8));  // at least 8 stages per split
    P.Mp = P.MT * BM;
    P.part_bytes = (size_t)P.S * P.tiles * 4 * FRAGS * 64 * 16;
    P.db_bytes = want_db ? (size_t)P.NT * P.S * P.Mp * 4 : 0;
    return P;
}

}  // namespace wg
}  // namespace lgm

extern "C" size_t lgm_linear_wgrad_workspace_size(int K, int M, int N, int want_db) {
    if (K < 0 || M <= 0 || N <= 0) return 0;
    const lgm::wg::Plan P = lgm::wg::plan(K, M, N, want_db != 0);
    return ((P.part_bytes + 255) & ~(size_t)255) + P.db_bytes;
}

extern "C" int lgm_linear_wgrad(int dtype, int K, int M, int N, const void *dy, long long ld_dy, const void *x,
                                long long ld_x, float *dw, float *db, void *workspace, size_t workspace_bytes,
                                void *stream, const lgm_diag *diag) {
    using namespace lgm::wg;
    lgm::clear_error();
    lgm::DiagScope ds(diag);
    if (dtype != LGM_ATTN_BF16 && dtype != LGM_ATTN_F16) {
        lgm::set_error("lgm_linear_wgrad: dtype must be bf16 or fp16 (got %d)", dtype);
        return LGM_E_INVALID;
    }
    if (K < 0 || M <= 0 || N <= 0 || M % 8 || N % 8 || ld_dy < M || ld_x < N || ld_dy % 8 || ld_x % 8) {
        lgm::set_error("lgm_linear_wgrad: bad shape K=%d M=%d N=%d ld_dy=%lld ld_x=%lld (M, N, ld multiples of 8)", K,
                       M, N, ld_dy, ld_x);
        return LGM_E_INVALID;
    }
    if (!dw || (K > 0 && (!dy || !x)) || !workspace) {
        lgm::set_error("lgm_linear_wgrad: null pointer");
        return LGM_E_INVALID;
    }
    if (((uintptr_t)dy | (uintptr_t)x) & 15) {
        lgm::set_error("lgm_linear_wgrad: dy and x must be 16-byte aligned");
        return LGM_E_INVALID;
    }
    if (workspace_bytes < lgm_linear_wgrad_workspace_size(K, M, N, db != nullptr)) {
        lgm::set_error("lgm_linear_wgrad: workspace too small");
        return LGM_E_WORKSPACE;
    }
    const Plan P = plan(K, M, N, db != nullptr);
    hipStream_t st = (hipStream_t)stream;
    f32x4 *part = (f32x4 *)workspace;
    float *dbpart = db ? (float *)((char *)workspace + ((P.part_bytes + 255) & ~(size_t)255)) : nullptr;
    const int grid = P.tiles * P.S;
    if (dtype == LGM_ATTN_BF16)
        LGM_LAUNCH("k_wgrad", st, (k_wgrad<LGM_ATTN_BF16><<<grid, THREADS, 0, st>>>(
                                      K, M, N, (const uint16_t *)dy, ld_dy, (const uint16_t *)x, ld_x, P.S, P.NT, part,
                                      dbpart, P.Mp)));
    else
        LGM_LAUNCH("k_wgrad", st, (k_wgrad<LGM_ATTN_F16><<<grid, THREADS, 0, st>>>(
                                      K, M, N, (const uint16_t *)dy, ld_dy, (const uint16_t *)x, ld_x, P.S, P.NT, part,
                                      dbpart, P.Mp)));
    const long long npos = (long long)P.tiles * 4 * FRAGS * 64;
    const int rgrid = (int)((npos + 255) / 256) + (db ? (M * DBT + 255) / 256 : 0);
    LGM_LAUNCH("k_wgrad_reduce", st, (k_wgrad_reduce<<<rgrid, 256, 0, st>>>(M, N, P.S, P.NT, P.tiles, part, dbpart,
                                                                             P.Mp, dw, db)));
    return LGM_OK;
}
