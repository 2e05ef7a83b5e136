// apsp.hip -- all-pairs hop distances by blocked min-plus closure.
//
// For small dense fabrics (fat-tree k<=48, dragonfly) the all-pairs hop
// matrix fits in HBM many times over (V=2880: 16.6 MB of uint16) and the
// blocked Floyd-Warshall closure D <- min(D, D[:,K] (+) D[K,:]) over 64-wide
// pivot blocks is a tiled min-plus "GEMM".  min-plus is not a multiply-add,
// so it runs on the VALU (v_add/v_min), not MFMA: each thread owns a 4x4
// output micro-tile, pivot row/column tiles are staged in LDS and read as
// broadcasts.  Three phases per pivot block: (1) the pivot tile closes on
// itself, (2) pivot row and column tiles close against it, (3) every other
// tile takes one min-plus product.  Distances saturate at 0xFFFF (= no
// path), the same convention as the msbfs dist tables it cross-checks.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr int T = 64;            // tile edge
constexpr uint32_t INF = 0xFFFFu;

__device__ __forceinline__ uint32_t sat_add(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c > INF ? INF : c;
}

__global__ __launch_bounds__(256) void apsp_init_kernel(
    int V, int Vp, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, uint16_t *__restrict__ D)
{
    const size_t n = (size_t)Vp * Vp;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / Vp), c = (int)(i % Vp);
        D[i] = (r == c && r < V) ? 0 : (uint16_t)INF;
    }
}

__global__ __launch_bounds__(256) void apsp_edges_kernel(
    int V, int Vp, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, uint16_t *__restrict__ D)
{
    const int u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= V) return;
    for (int e = row_ptr[u]; e < row_ptr[u + 1]; ++e)
        if (col[e] != u) D[(size_t)u * Vp + col[e]] = 1;
}

// phase 1: the pivot tile, 64 sequential pivots inside LDS
__global__ __launch_bounds__(256) void apsp_phase1_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    __shared__ uint32_t t[T][T + 1];
    const int base = kb * T;
    for (int i = threadIdx.x; i < T * T; i += 256)
        t[i / T][i % T] = D[(size_t)(base + i / T) * Vp + base + i % T];
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        for (int i = threadIdx.x; i < T * T; i += 256) {
            const int r = i / T, c = i % T;
            const uint32_t v = sat_add(t[r][k], t[k][c]);
            if (v < t[r][c]) t[r][c] = v;
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < T * T; i += 256)
        D[(size_t)(base + i / T) * Vp + base + i % T] = (uint16_t)t[i / T][i % T];
}

// phase 2: blockIdx.y == 0 -> pivot row tile (kb, j), 1 -> column tile (j, kb)
__global__ __launch_bounds__(256) void apsp_phase2_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    int j = blockIdx.x;
    if (j >= kb) ++j;                       // skip the pivot tile itself
    const bool row = blockIdx.y == 0;
    __shared__ uint32_t piv[T][T + 1];
    __shared__ uint32_t t[T][T + 1];
    const int pb = kb * T;
    const int r0 = row ? pb : j * T;
    const int c0 = row ? j * T : pb;
    for (int i = threadIdx.x; i < T * T; i += 256) {
        piv[i / T][i % T] = D[(size_t)(pb + i / T) * Vp + pb + i % T];
        t[i / T][i % T] = D[(size_t)(r0 + i / T) * Vp + c0 + i % T];
    }
    __syncthreads();
    for (int k = 0; k < T; ++k) {
        for (int i = threadIdx.x; i < T * T; i += 256) {
            const int r = i / T, c = i % T;
            const uint32_t v = row ? sat_add(piv[r][k], t[k][c]) : sat_add(t[r][k], piv[k][c]);
            if (v < t[r][c]) t[r][c] = v;
        }
        __syncthreads();
    }
    for (int i = threadIdx.x; i < T * T; i += 256)
        D[(size_t)(r0 + i / T) * Vp + c0 + i % T] = (uint16_t)t[i / T][i % T];
}

// phase 3: tile (bi, bj) = min(tile, A(bi,kb) (+) B(kb,bj)); 4x4 per thread
__global__ __launch_bounds__(256) void apsp_phase3_kernel(int Vp, int kb, uint16_t *__restrict__ D)
{
    int bi = blockIdx.y, bj = blockIdx.x;
    if (bi >= kb) ++bi;
    if (bj >= kb) ++bj;
    __shared__ uint32_t A[T][T + 1];   // A[r][k]
    __shared__ uint32_t B[T][T + 1];   // B[k][c]
    const int pb = kb * T;
    for (int i = threadIdx.x; i < T * T; i += 256) {
        A[i / T][i % T] = D[(size_t)(bi * T + i / T) * Vp + pb + i % T];
        B[i / T][i % T] = D[(size_t)(pb + i / T) * Vp + bj * T + i % T];
    }
    __syncthreads();
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    uint32_t acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            acc[r][c] = D[(size_t)(bi * T + ty * 4 + r) * Vp + bj * T + tx * 4 + c];
#pragma unroll 8
    for (int k = 0; k < T; ++k) {
        uint32_t a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) a[r] = A[ty * 4 + r][k];
#pragma unroll
        for (int c = 0; c < 4; ++c) b[c] = B[k][tx * 4 + c];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = min(acc[r][c], a[r] + b[c]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            D[(size_t)(bi * T + ty * 4 + r) * Vp + bj * T + tx * 4 + c] =
                (uint16_t)(acc[r][c] > INF ? INF : acc[r][c]);
}

// ---------------------------------------------------------------------------
// Min-plus squaring: D <- min(D, D (x) D) in place, repeated until nothing
// changes.  Unlike the blocked Floyd-Warshall above (three dependent phases
// and 64 serial pivots per block step) every squaring is one fully parallel
// GEMM-shaped launch, and hop distances of a fabric with diameter d need
// ceil(log2 d) + 1 of them (k=48: 3).  In place is exact: every entry is
// always the length of some path (reading an already-improved value only
// speeds convergence), and a pass that improves nothing is the closure.
// The arithmetic is packed u16 on the VALU -- v_pk_add_u16 with clamp (0xFFFF
// saturates as "no path") and v_pk_min_u16 -- 2 (i, j) pairs per lane per
// instruction; each thread owns an 8 x 8 output block of a 128 x 128 tile,
// K staged through LDS in 32-wide slices, k-major so the 8 A values and the
// 8 B values of a step are one ds_read_b128 each.
// ---------------------------------------------------------------------------
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr int MT = 128;          // output tile edge
constexpr int KS = 32;           // K slice
constexpr int LDA = MT + 8;      // padded LDS row (u16)

__device__ __forceinline__ u16x2 as_pk(uint32_t x)
{
    return __builtin_bit_cast(u16x2, x);
}

__device__ __forceinline__ uint32_t as_u32(u16x2 x)
{
    return __builtin_bit_cast(uint32_t, x);
}

__global__ __launch_bounds__(256) void minplus_square_kernel(int Vp, uint16_t *__restrict__ D,
                                                             int *__restrict__ changed)
{
    __shared__ __attribute__((aligned(16))) uint16_t As[KS][LDA];   // As[k][i] = D[i0+i][k0+k]
    __shared__ __attribute__((aligned(16))) uint16_t Bs[KS][LDA];   // Bs[k][j] = D[k0+k][j0+j]
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int i0 = blockIdx.y * MT, j0 = blockIdx.x * MT;
    u16x2 acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint4 v = *reinterpret_cast<const uint4 *>(D + (size_t)(i0 + ty * 8 + r) * Vp + j0 + tx * 8);
        acc[r][0] = as_pk(v.x);
        acc[r][1] = as_pk(v.y);
        acc[r][2] = as_pk(v.z);
        acc[r][3] = as_pk(v.w);
    }

    // slices are staged register -> LDS: the next slice's global loads are in
    // flight while the current one is consumed
    uint4 ra[2], rb[2];
    auto load_slice = [&](int k0) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int L = threadIdx.x + 256 * h;
            ra[h] = *reinterpret_cast<const uint4 *>(D + (size_t)(i0 + (L >> 2)) * Vp + k0 +
                                                      (L & 3) * 8);
            rb[h] = *reinterpret_cast<const uint4 *>(D + (size_t)(k0 + (L >> 4)) * Vp + j0 +
                                                      (L & 15) * 8);
        }
    };
    auto store_slice = [&]() {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int L = threadIdx.x + 256 * h;
            const int i = L >> 2, kq = (L & 3) * 8;          // A: transpose into As[k][i]
            const uint32_t w[4] = {ra[h].x, ra[h].y, ra[h].z, ra[h].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                As[kq + 2 * e][i] = (uint16_t)(w[e] & 0xFFFFu);
                As[kq + 2 * e + 1][i] = (uint16_t)(w[e] >> 16);
            }
            *reinterpret_cast<uint4 *>(&Bs[L >> 4][(L & 15) * 8]) = rb[h];   // B: k-major already
        }
    };
    load_slice(0);
    for (int k0 = 0; k0 < Vp; k0 += KS) {
        store_slice();
        __syncthreads();
        if (k0 + KS < Vp) load_slice(k0 + KS);
#pragma unroll 4
        for (int k = 0; k < KS; ++k) {
            const uint4 av = *reinterpret_cast<const uint4 *>(&As[k][ty * 8]);
            const uint4 bv = *reinterpret_cast<const uint4 *>(&Bs[k][tx * 8]);
            const u16x2 b[4] = {as_pk(bv.x), as_pk(bv.y), as_pk(bv.z), as_pk(bv.w)};
            const uint32_t aw[4] = {av.x, av.y, av.z, av.w};
            // splat a row's value into both halves with one v_perm_b32, then
            // all 32 saturating adds before the 32 mins
            u16x2 t[8][4];
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const u16x2 as = as_pk(__builtin_amdgcn_perm(aw[r >> 1], aw[r >> 1],
                                                             (r & 1) ? 0x03020302u : 0x01000100u));
#pragma unroll
                for (int c = 0; c < 4; ++c) t[r][c] = __builtin_elementwise_add_sat(as, b[c]);
            }
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = __builtin_elementwise_min(acc[r][c], t[r][c]);
        }
        __syncthreads();
    }
    // only this block writes its tile, so the old values can be re-read here
    // instead of being held in registers through the K loop
    bool any = false;
    uint32_t mx = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        uint16_t *p = D + (size_t)(i0 + ty * 8 + r) * Vp + j0 + tx * 8;
        const uint4 o = *reinterpret_cast<const uint4 *>(p);
        uint4 v;
        v.x = as_u32(acc[r][0]);
        v.y = as_u32(acc[r][1]);
        v.z = as_u32(acc[r][2]);
        v.w = as_u32(acc[r][3]);
        any |= (v.x != o.x) | (v.y != o.y) | (v.z != o.z) | (v.w != o.w);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t w = as_u32(acc[r][c]);
            const uint32_t lo = w & 0xFFFFu, hi = w >> 16;
            mx = max(mx, lo == 0xFFFFu ? 0u : lo);
            mx = max(mx, hi == 0xFFFFu ? 0u : hi);
        }
        *reinterpret_cast<uint4 *>(p) = v;
    }
    if (__ballot(any) && lane_id() == 0) atomicOr(changed, 1);
    // largest finite distance (wave max, one atomic per wave)
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane_id() == 0) atomicMax(reinterpret_cast<unsigned *>(changed) + 1, mx);
}


// Same pass on 64 x 64 output tiles, 128 threads (each 4 rows x 8 columns):
// 4x the workgroups of the 128 x 128 tiling, so they spread evenly over the
// CUs (k=48: 2,025 two-wave groups, <= 8 per CU, vs 529 four-wave groups of
// which 17 CUs got a third -- the last CUs set the pass time), and V needs
// padding only to a multiple of 64 (k=48: none).  Per k step a thread reads
// 4 A values (ds_read_b64) and 8 B values (ds_read_b128): 4 splats, 16 adds,
// 16 mins for 32 outputs -- the 128-tile kernel's VALU per output.
constexpr int MT64 = 64;
constexpr int LDA64 = MT64 + 8;

__global__ __launch_bounds__(128) void minplus_square64_kernel(int Vp, uint16_t *__restrict__ D,
                                                               int *__restrict__ changed)
{
    __shared__ __attribute__((aligned(16))) uint16_t As[KS][LDA64];   // As[k][i] = D[i0+i][k0+k]
    __shared__ __attribute__((aligned(16))) uint16_t Bs[KS][LDA64];   // Bs[k][j] = D[k0+k][j0+j]
    const int tx = threadIdx.x & 7, ty = threadIdx.x >> 3;
    const int i0 = blockIdx.y * MT64, j0 = blockIdx.x * MT64;
    u16x2 acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint4 v = *reinterpret_cast<const uint4 *>(D + (size_t)(i0 + ty * 4 + r) * Vp + j0 + tx * 8);
        acc[r][0] = as_pk(v.x);
        acc[r][1] = as_pk(v.y);
        acc[r][2] = as_pk(v.z);
        acc[r][3] = as_pk(v.w);
    }
    uint4 ra0, ra1, rb0, rb1;
    auto load_slice = [&](int k0) {
        const int L0 = threadIdx.x, L1 = threadIdx.x + 128;
        ra0 = *reinterpret_cast<const uint4 *>(D + (size_t)(i0 + (L0 >> 2)) * Vp + k0 + (L0 & 3) * 8);
        ra1 = *reinterpret_cast<const uint4 *>(D + (size_t)(i0 + (L1 >> 2)) * Vp + k0 + (L1 & 3) * 8);
        rb0 = *reinterpret_cast<const uint4 *>(D + (size_t)(k0 + (L0 >> 3)) * Vp + j0 + (L0 & 7) * 8);
        rb1 = *reinterpret_cast<const uint4 *>(D + (size_t)(k0 + (L1 >> 3)) * Vp + j0 + (L1 & 7) * 8);
    };
    auto store_a = [&](int L, const uint4 &v) {         // transpose into As[k][i]
        const int i = L >> 2, kq = (L & 3) * 8;
        As[kq + 0][i] = (uint16_t)(v.x & 0xFFFFu);
        As[kq + 1][i] = (uint16_t)(v.x >> 16);
        As[kq + 2][i] = (uint16_t)(v.y & 0xFFFFu);
        As[kq + 3][i] = (uint16_t)(v.y >> 16);
        As[kq + 4][i] = (uint16_t)(v.z & 0xFFFFu);
        As[kq + 5][i] = (uint16_t)(v.z >> 16);
        As[kq + 6][i] = (uint16_t)(v.w & 0xFFFFu);
        As[kq + 7][i] = (uint16_t)(v.w >> 16);
    };
    load_slice(0);
    for (int k0 = 0; k0 < Vp; k0 += KS) {
        store_a(threadIdx.x, ra0);
        store_a(threadIdx.x + 128, ra1);
        *reinterpret_cast<uint4 *>(&Bs[threadIdx.x >> 3][(threadIdx.x & 7) * 8]) = rb0;
        *reinterpret_cast<uint4 *>(&Bs[(threadIdx.x + 128) >> 3][(threadIdx.x & 7) * 8]) = rb1;
        __syncthreads();
        if (k0 + KS < Vp) load_slice(k0 + KS);
#pragma unroll 8
        for (int k = 0; k < KS; ++k) {
            const uint2 av = *reinterpret_cast<const uint2 *>(&As[k][ty * 4]);
            const uint4 bv = *reinterpret_cast<const uint4 *>(&Bs[k][tx * 8]);
            const u16x2 b[4] = {as_pk(bv.x), as_pk(bv.y), as_pk(bv.z), as_pk(bv.w)};
            const uint32_t aw[2] = {av.x, av.y};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const u16x2 as = as_pk(__builtin_amdgcn_perm(aw[r >> 1], aw[r >> 1],
                                                             (r & 1) ? 0x03020302u : 0x01000100u));
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    acc[r][c] = __builtin_elementwise_min(acc[r][c],
                                                          __builtin_elementwise_add_sat(as, b[c]));
            }
        }
        __syncthreads();
    }
    bool any = false;
    uint32_t mx = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        uint16_t *p = D + (size_t)(i0 + ty * 4 + r) * Vp + j0 + tx * 8;
        const uint4 o = *reinterpret_cast<const uint4 *>(p);
        uint4 v;
        v.x = as_u32(acc[r][0]);
        v.y = as_u32(acc[r][1]);
        v.z = as_u32(acc[r][2]);
        v.w = as_u32(acc[r][3]);
        any |= (v.x != o.x) | (v.y != o.y) | (v.z != o.z) | (v.w != o.w);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t w = as_u32(acc[r][c]);
            const uint32_t lo = w & 0xFFFFu, hi = w >> 16;
            mx = max(mx, lo == 0xFFFFu ? 0u : lo);
            mx = max(mx, hi == 0xFFFFu ? 0u : hi);
        }
        *reinterpret_cast<uint4 *>(p) = v;
    }
    if (__ballot(any) && lane_id() == 0) atomicOr(changed, 1);
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (lane_id() == 0) atomicMax(reinterpret_cast<unsigned *>(changed) + 1, mx);
}

// Bellman-Ford sweeps, 8 rows at a time: row i of D holds upper bounds of
// the hop distances from i (every entry is the length of a real path), and
// D[i][j] <- min(D[i][j], min over in-neighbours k of j of D[i][k] + 1)
// keeps that true while extending the exact horizon by at least one hop per
// sweep; a sweep that changes nothing proves the row exact (D[i][i] = 0 and
// the edge inequalities hold everywhere: by induction on path length).  The
// rows of one source depend on nothing else, so a block iterates its 8 rows
// to that fixpoint (or `cap` sweeps) in LDS with no grid-wide step, and
// writes them back.  Rows staged TRANSPOSED (column j -> its 8 row values,
// one 16-byte entry): one ds_read_b128 per in-neighbour k serves all 8
// rows, the relaxation is 4 v_pk_add_u16 (clamp) + 4 v_pk_min_u16; sweeps
// update in place (any interleaving keeps valid upper bounds).  Small-
// diameter sparse fabrics (k=48: diameter 4) converge here in a handful of
// V^2 x in-degree sweeps, where each squaring pass costs V^3.
// changed[0]: some block did not reach its fixpoint within cap sweeps;
// changed[1]: the most sweeps any block ran.
// column k's 16-B entry lives at lsw(k): the 16 entries of each aligned
// group of 16 (one 256-B LDS bank row) permuted by the group number, so
// columns a multiple of 16 apart -- a fat-tree aggregation switch's core
// neighbours are 24 apart -- fall in different bank slots of a ds_read_b128
__device__ __forceinline__ int lsw(int k) { return k ^ ((k >> 4) & 15); }

// NQ: u32 words of an in-row that hold entries (in-degree <= 2 NQ), a
// template so the row loads are whole 16-B loads and the relaxation loop
// has no branch (a runtime bound put a scalar branch around every load and
// every LDS read pair: 2.3x slower per sweep)
template <int NQ>
__global__ __launch_bounds__(1024) void apsp_relax8_kernel(int V, int Vp,
                                                          const uint16_t *__restrict__ radj,
                                                          const uint16_t *__restrict__ adj,
                                                          uint16_t *__restrict__ D,
                                                          int *__restrict__ changed, int cap,
                                                          int fresh)
{
    static_assert(NQ % 4 == 0 && NQ <= 32, "whole 16-B in-row loads");
    // L[j] = D[i0..i0+7][j] as 8 u16; L[V] = all INF: the in-rows' padding
    // (sentinel V) relaxes against it to no effect, so the inner loop has no
    // per-lane branch and its LDS reads issue back to back
    extern __shared__ uint4 L[];
    const int i0 = blockIdx.x * 8;
    if (fresh) {
        // D not initialised: the block's 8 rows start as 0 on the diagonal,
        // 1 on each out-link (the rows' u16 out-rows, 64 lanes per row), INF
        // elsewhere -- what apsp_init_kernel + apsp_edges_kernel write, built
        // here in LDS instead of 2 x V^2 x 2 bytes through HBM
        uint16_t *L16 = reinterpret_cast<uint16_t *>(L);
        for (int j = threadIdx.x; j <= V; j += blockDim.x) {
            uint32_t w[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ra = i0 + 2 * q, rb = ra + 1;
                const uint32_t a = ra >= V ? 0u : (ra == j ? 0u : 0xFFFFu);
                const uint32_t b = rb >= V ? 0u : (rb == j ? 0u : 0xFFFFu);
                w[q] = a | (b << 16);
            }
            L[lsw(j)] = make_uint4(w[0], w[1], w[2], w[3]);
        }
        __syncthreads();
        for (int t = threadIdx.x; t < 8 * 64; t += blockDim.x) {
            const int r = t >> 6, i = i0 + r;
            if (i < V) {
                const int x = (int)adj[(size_t)i * 64 + (t & 63)];
                if (x < V && x != i) L16[(size_t)lsw(x) * 8 + r] = 1;
            }
        }
    }
    for (int j = threadIdx.x; j <= V && !fresh; j += blockDim.x) {
        uint32_t w[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ra = i0 + 2 * q, rb = ra + 1;
            // rows past V (the last block) hold 0: they never change and
            // never hold the early exit below back; real rows' L[V] is INF
            const uint32_t a = ra >= V ? 0u : (j < V ? D[(size_t)ra * Vp + j] : 0xFFFFu);
            const uint32_t b = rb >= V ? 0u : (j < V ? D[(size_t)rb * Vp + j] : 0xFFFFu);
            w[q] = a | (b << 16);
        }
        L[lsw(j)] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    __syncthreads();
    const u16x2 one = {1, 1};
    bool any = false, ch = true;
    int sweeps = 0;
    while (ch && sweeps < cap) {
        ch = false;
        ++sweeps;
        u16x2 mx = {0, 0};                      // largest entry this thread saw
        for (int j = threadIdx.x; j < V; j += blockDim.x) {
            const uint4 *rr = reinterpret_cast<const uint4 *>(radj + (size_t)j * 64);
            uint32_t nb[NQ];                     // in-row of j, sentinel V
#pragma unroll
            for (int q = 0; q < NQ / 4; ++q) {
                const uint4 t = rr[q];
                nb[4 * q] = t.x;
                nb[4 * q + 1] = t.y;
                nb[4 * q + 2] = t.z;
                nb[4 * q + 3] = t.w;
            }
            const uint4 c = L[lsw(j)];
            u16x2 cur[4], best[4], alt[4];
            cur[0] = __builtin_bit_cast(u16x2, c.x);
            cur[1] = __builtin_bit_cast(u16x2, c.y);
            cur[2] = __builtin_bit_cast(u16x2, c.z);
            cur[3] = __builtin_bit_cast(u16x2, c.w);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                best[r] = cur[r];
                alt[r] = cur[r];
            }
            // 8 LDS reads in flight per batch (4 in-row words), two
            // independent min chains (even / odd halves of each word)
#pragma unroll
            for (int q0 = 0; q0 < NQ; q0 += 4) {
                uint4 x[8];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    x[2 * t] = L[lsw((int)(nb[q0 + t] & 0xFFFFu))];
                    x[2 * t + 1] = L[lsw((int)(nb[q0 + t] >> 16))];
                }
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    u16x2 *acc = (t & 1) ? alt : best;
                    acc[0] = __builtin_elementwise_min(
                        acc[0], __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, x[t].x), one));
                    acc[1] = __builtin_elementwise_min(
                        acc[1], __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, x[t].y), one));
                    acc[2] = __builtin_elementwise_min(
                        acc[2], __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, x[t].z), one));
                    acc[3] = __builtin_elementwise_min(
                        acc[3], __builtin_elementwise_add_sat(__builtin_bit_cast(u16x2, x[t].w), one));
                }
            }
            bool d = false;                      // INF + 1 saturates: never below INF
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                best[r] = __builtin_elementwise_min(best[r], alt[r]);
                d |= __builtin_bit_cast(uint32_t, best[r]) != __builtin_bit_cast(uint32_t, cur[r]);
                mx = __builtin_elementwise_max(mx, best[r]);
            }
            if (d) {
                L[lsw(j)] = make_uint4(__builtin_bit_cast(uint32_t, best[0]),
                                  __builtin_bit_cast(uint32_t, best[1]),
                                  __builtin_bit_cast(uint32_t, best[2]),
                                  __builtin_bit_cast(uint32_t, best[3]));
                ch = true;
            }
        }
        // exact without a confirming sweep: after s in-place sweeps every
        // distance <= s + 1 is exact (each sweep extends the exact horizon
        // by at least one hop), and an entry is an upper bound of its true
        // distance, so once every entry of the block is finite and <= s + 1
        // each one equals its true distance
        const uint32_t m = mx.x > mx.y ? mx.x : mx.y;
        const bool far = m > (uint32_t)(sweeps + 1);   // INF (0xFFFF) included
        ch = __syncthreads_or(ch);
        any |= ch;
        if (!__syncthreads_or(far)) ch = false;
    }
    if (any || fresh) {                          // write the improved (or new) rows back
        for (int j = threadIdx.x; j < V; j += blockDim.x) {
            const uint4 c = L[lsw(j)];
            const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int ra = i0 + 2 * q, rb = ra + 1;
                if (ra < V) D[(size_t)ra * Vp + j] = (uint16_t)(w[q] & 0xFFFFu);
                if (rb < V) D[(size_t)rb * Vp + j] = (uint16_t)(w[q] >> 16);
            }
        }
    }
    if (threadIdx.x == 0) {
        if (ch) atomicOr(changed, 1);            // cap reached before the fixpoint
        atomicMax(changed + 1, sweeps);
    }
}

}  // namespace

static int launch_apsp_squaring(sdnr_ctx *ctx, uint16_t *D, int V, int Vp, int mt)
{
    int rc = sdnr_reserve(&ctx->scratch2, &ctx->scratch2_bytes, 256);
    if (rc) return rc;
    int *changed = static_cast<int *>(ctx->scratch2);
    // Squaring passes double the exact horizon for V^3 each; Bellman-Ford
    // sweeps (apsp_relax8_kernel) extend it by one hop for V^2 x in-degree
    // each and stop by themselves at the fixpoint.  So: sweep to the
    // fixpoint, capped at about one squaring pass's worth of sweeps; only a
    // graph whose diameter outruns the cap gets a squaring pass (horizon x2)
    // and sweeps again.  SDNROUTE_APSP_RELAX=0: squaring only, stopping when
    // a pass changes nothing, or when after s squarings (exact for every
    // distance <= 2^s) the largest finite distance M is < 2^s.
    const int nt = Vp / mt;
    const char *rf = getenv("SDNROUTE_APSP_RELAX");
    // the transposed 8-row block must fit LDS (16 B per vertex + the INF
    // column: V < 10,240)
    const bool relax = ctx->radj16 && ctx->max_indeg <= 64 &&
                       (((size_t)V + 1 + 15) & ~(size_t)15) * 16 <= 160 * 1024 &&
                       !(rf && !strcmp(rf, "0"));
    // sweeps per squaring pass of cost: V^3 / (V E) = V / avg degree, /4
    // for the sweeps' lower op rate (measured k=48: 46 us per sweep of all
    // rows vs 0.95 ms per squaring pass)
    long long capl = ctx->E > 0 ? ((long long)V * V) / (4ll * ctx->E) : 4;
    const int cap = capl < 4 ? 4 : (capl > 64 ? 64 : (int)capl);
    ctx->last_launches = 0;
    ctx->last_sweeps = 0;
    // in-row words per column, rounded to whole 16-B loads
    const int nq = ((ctx->max_indeg + 1) / 2 + 3) & ~3;
    auto relax_kernel = nq <= 4 ? apsp_relax8_kernel<4>
                      : nq <= 8 ? apsp_relax8_kernel<8>
                      : nq <= 12 ? apsp_relax8_kernel<12>
                      : nq <= 16 ? apsp_relax8_kernel<16>
                      : nq <= 24 ? apsp_relax8_kernel<24> : apsp_relax8_kernel<32>;
    // V + 1 entries (the INF column), whole groups of 16 (the swizzle lsw)
    const size_t lbytes = (((size_t)V + 1 + 15) & ~(size_t)15) * 16;
    if (relax) sdnr_allow_lds(reinterpret_cast<const void *>(relax_kernel), lbytes);
    // the first sweep launch builds its rows from the out-rows itself (no
    // init / edge passes over V^2); the padding of a Vp > V matrix, which
    // the squaring passes read, still comes from the init pass
    const bool fused = relax && ctx->adj16;
    if (!fused || Vp != V)
        hipLaunchKernelGGL(apsp_init_kernel, dim3(1024), dim3(256), 0, ctx->stream, V, Vp,
                           ctx->row_ptr, ctx->col, D);
    if (!fused)
        hipLaunchKernelGGL(apsp_edges_kernel, dim3((V + 255) / 256), dim3(256), 0, ctx->stream,
                           V, Vp, ctx->row_ptr, ctx->col, D);
    for (int it = 1; it <= 40; ++it) {         // 2^40 >> any hop distance
        if (relax) {
            SDNR_HIP(hipMemsetAsync(changed, 0, 2 * sizeof(int), ctx->stream));
            hipLaunchKernelGGL(relax_kernel, dim3((V + 7) / 8), dim3(1024), lbytes, ctx->stream,
                               V, Vp, ctx->radj16, ctx->adj16, D, changed, cap,
                               (int)(fused && it == 1));
            SDNR_HIP(hipGetLastError());
            int h[2] = {1, 0};
            int rc = sdnr_fetch_ints(ctx, changed, 2, h);
            if (rc) return rc;
            ctx->last_sweeps += h[1];
            if (!h[0]) break;                  // every row at its fixpoint: exact
        }
        ctx->last_launches = it;
        SDNR_HIP(hipMemsetAsync(changed, 0, 2 * sizeof(int), ctx->stream));
        if (mt == MT64)
            hipLaunchKernelGGL(minplus_square64_kernel, dim3(nt, nt), dim3(128), 0, ctx->stream,
                               Vp, D, changed);
        else
            hipLaunchKernelGGL(minplus_square_kernel, dim3(nt, nt), dim3(256), 0, ctx->stream, Vp,
                               D, changed);
        SDNR_HIP(hipGetLastError());
        int h[2] = {0, 0};
        int rc = sdnr_fetch_ints(ctx, changed, 2, h);
        if (rc) return rc;
        if (!relax && (!h[0] || (it < 31 && (long long)h[1] < (1ll << it)))) break;
        if (relax && !h[0]) break;             // nothing improved: exact
    }
    return SDNR_OK;
}

int sdnr_launch_apsp(sdnr_ctx *ctx, uint16_t *d_dist)
{
    const int V = ctx->V;
    if (V == 0) return SDNR_OK;
    if (V > 16384) return sdnr_fail(SDNR_ERR_INVAL, "apsp: V=%d > 16384", V);
    // SDNROUTE_APSP=fw selects the blocked Floyd-Warshall, =sq128 the
    // 128 x 128-tile squaring (A/B, tests); default: 64 x 64-tile squaring
    const char *f = getenv("SDNROUTE_APSP");
    const bool fw = f && !strcmp(f, "fw");
    const int mt = f && !strcmp(f, "sq128") ? MT : MT64;
    const int nb = (V + (fw ? T : mt) - 1) / (fw ? T : mt);
    const int Vp = nb * (fw ? T : mt);
    const size_t bytes = (size_t)Vp * Vp * sizeof(uint16_t);
    uint16_t *D = d_dist;
    if (Vp != V) {
        int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes, bytes);
        if (rc) return rc;
        D = static_cast<uint16_t *>(ctx->scratch);
    }
    if (!fw) {
        ctx->last_kernel = mt == MT64 ? "minplus_square64_kernel" : "minplus_square_kernel";
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
        int rc = launch_apsp_squaring(ctx, D, V, Vp, mt);
        if (rc) return rc;
        if (ctx->last_launches == 0 && ctx->last_sweeps > 0)
            ctx->last_kernel = "apsp_relax8_kernel";   // converged by sweeps alone
        if (D != d_dist)
            SDNR_HIP(hipMemcpy2DAsync(d_dist, (size_t)V * 2, D, (size_t)Vp * 2, (size_t)V * 2, V,
                                      hipMemcpyDeviceToDevice, ctx->stream));
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    ctx->last_kernel = "apsp_phase{1,2,3}_kernel";
    ctx->last_sweeps = 0;
    ctx->last_launches = nb;
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipLaunchKernelGGL(apsp_init_kernel, dim3(1024), dim3(256), 0, ctx->stream, V, Vp,
                       ctx->row_ptr, ctx->col, D);
    hipLaunchKernelGGL(apsp_edges_kernel, dim3((V + 255) / 256), dim3(256), 0, ctx->stream,
                       V, Vp, ctx->row_ptr, ctx->col, D);
    for (int kb = 0; kb < nb; ++kb) {
        hipLaunchKernelGGL(apsp_phase1_kernel, dim3(1), dim3(256), 0, ctx->stream, Vp, kb, D);
        if (nb > 1) {
            hipLaunchKernelGGL(apsp_phase2_kernel, dim3(nb - 1, 2), dim3(256), 0, ctx->stream,
                               Vp, kb, D);
            hipLaunchKernelGGL(apsp_phase3_kernel, dim3(nb - 1, nb - 1), dim3(256), 0,
                               ctx->stream, Vp, kb, D);
        }
    }
    SDNR_HIP(hipGetLastError());
    if (D != d_dist)
        SDNR_HIP(hipMemcpy2DAsync(d_dist, (size_t)V * 2, D, (size_t)Vp * 2, (size_t)V * 2, V,
                                  hipMemcpyDeviceToDevice, ctx->stream));
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
