// ecmp.hip -- the shortest-route (ECMP) sets of find_route(..., multiple=True).
//
// SURVEY.md 8(f) 3.  _find_routes_bfs (sdnmpi/util/topology_db.py:86-122)
// enumerates every simple path FIFO and keeps the shortest, which is every
// path of the shortest-path DAG toward d in lexicographic dpid order (FIFO
// over ascending neighbours, :106) -- exponential in the reference (fat-tree
// k=6 runs out of memory).  Here the set is counted and unranked instead:
//
//  * ecmp_count_kernel: per destination row, paths[x] = number of shortest
//    x -> d routes = sum of paths[n] over out-neighbours n one hop closer,
//    computed level by level (levels from the dist table) with the row's
//    distances and counts in LDS; saturating at UINT64_MAX.
//    ecmp_count_rows_kernel is the same DP over the 64-wide u16 rows -- the
//    form used whenever those rows exist.
//  * ecmp_unrank_kernel: route r of (x, d) in lexicographic order: at each
//    vertex take the ascending out-neighbours one hop closer and descend
//    into the one whose count range holds r (r -= paths[n] for the ones
//    skipped).  One thread per route; the vertex sequence is written to a
//    fixed-stride slot.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr uint64_t kSat = ~0ull;

__device__ __forceinline__ uint64_t sat_add(uint64_t a, uint64_t b)
{
    const uint64_t c = a + b;
    return c < a ? kSat : c;
}

__global__ __launch_bounds__(1024) void ecmp_count_kernel(
    int V, int ndst, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const uint16_t *__restrict__ dist, uint64_t *__restrict__ paths)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lcnt[];
    uint16_t *ld = reinterpret_cast<uint16_t *>(lcnt + V);
    __shared__ int maxd;
    for (int row = blockIdx.x; row < ndst; row += gridDim.x) {
        const uint16_t *drow = dist + (size_t)row * V;
        uint64_t *prow = paths + (size_t)row * V;
        if (threadIdx.x == 0) maxd = 0;
        __syncthreads();
        int mymax = 0;
        for (int x = threadIdx.x; x < V; x += blockDim.x) {
            const uint16_t dx = drow[x];
            ld[x] = dx;
            lcnt[x] = dx == 0 ? 1ull : 0ull;
            if (dx != 0xFFFFu && dx > mymax) mymax = dx;
        }
        atomicMax(&maxd, mymax);
        __syncthreads();
        const int top = maxd;
        for (int L = 1; L <= top; ++L) {
            for (int x = threadIdx.x; x < V; x += blockDim.x) {
                if (ld[x] != (uint16_t)L) continue;
                uint64_t c = 0;
                const int re = row_ptr[x + 1];
                for (int e = row_ptr[x]; e < re; ++e) {
                    const int n = col[e];
                    if (ld[n] == (uint16_t)(L - 1)) c = sat_add(c, lcnt[n]);
                }
                lcnt[x] = c;
            }
            __syncthreads();
        }
        for (int x = threadIdx.x; x < V; x += blockDim.x) prow[x] = lcnt[x];
        __syncthreads();
    }
}

// Thread-per-vertex form over the 64-wide u16 out-rows (adj16, sentinel V,
// out-degrees deg32): a vertex of level L reads its row with 16-byte loads
// and sums its out-neighbours' counts from LDS.  Out-neighbours of a level-L
// vertex have level >= L-1, and with STAGE the counts of level L are held
// back (stage[], by list position) until every level-L vertex has read its
// neighbours, so at read time only level L-1 (and d) hold non-zero counts:
// the sum needs no level test.  Without STAGE (V too large for the staging
// buffer) each neighbour's level is checked in LDS instead.  Level L's
// vertices are collected first (ballot scan over per-wave slices).
// LDS: counts u64 [V+1] | STAGE: stage u64 [V] | levels u16 [V+1] |
// level list u16 [V] | NW words.
__host__ __device__ inline size_t ecmp_wave_lds(int V, int NW, bool stage)
{
    const size_t Vp = (size_t)((V + 1 + 3) & ~3);
    return Vp * (stage ? 20 : 12) + (size_t)NW * 4;
}

template <int NW, bool STAGE>
__global__ __launch_bounds__(NW * 64) void ecmp_count_rows_kernel(
    int V, int ndst, const uint16_t *__restrict__ adj, const uint32_t *__restrict__ deg,
    const uint16_t *__restrict__ dist, uint64_t *__restrict__ paths)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lcnt[];
    const int Vp = (V + 1 + 3) & ~3;
    uint64_t *stage = lcnt + Vp;                              // STAGE only
    uint16_t *ld = reinterpret_cast<uint16_t *>(lcnt + (STAGE ? 2 * Vp : Vp));
    uint16_t *list = ld + Vp;
    int *ctl = reinterpret_cast<int *>(list + Vp);
    __shared__ int maxd;
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    const int slice = ((V + NW * 64 - 1) / (NW * 64)) * 64;
    for (int row = blockIdx.x; row < ndst; row += gridDim.x) {
        const uint16_t *drow = dist + (size_t)row * V;
        uint64_t *prow = paths + (size_t)row * V;
        if (threadIdx.x == 0) maxd = 0;
        __syncthreads();
        int mymax = 0;
        for (int x = threadIdx.x; x <= V; x += blockDim.x) {
            const uint16_t dx = x < V ? drow[x] : (uint16_t)0xFFFEu;   // sentinel: no level
            ld[x] = dx;
            lcnt[x] = dx == 0 ? 1ull : 0ull;
            if (dx < 0xFFFEu && dx > mymax) mymax = dx;
        }
        atomicMax(&maxd, mymax);
        __syncthreads();
        const int top = maxd;
        const int s0 = w * slice, s1 = min(V, s0 + slice);
        for (int L = 1; L <= top; ++L) {
            int cnt = 0;
            for (int x0 = s0; x0 < s1; x0 += 64) {
                const int x = x0 + lane;
                cnt += __popcll(__ballot(x < s1 && ld[x] == (uint16_t)L));
            }
            if (lane == 0) ctl[w] = cnt;
            __syncthreads();
            int at = 0, total = 0;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const int c = ctl[k];
                at += k < w ? c : 0;
                total += c;
            }
            for (int x0 = s0; x0 < s1; x0 += 64) {
                const int x = x0 + lane;
                const bool hit = x < s1 && ld[x] == (uint16_t)L;
                const uint64_t m = __ballot(hit);
                if (hit) list[at + lanes_below(m)] = (uint16_t)x;
                at += __popcll(m);
            }
            __syncthreads();                     // list complete
            for (int i = threadIdx.x; i < total; i += blockDim.x) {
                const int x = list[i];
                const int dx = (int)deg[x];
                const uint4 *rp = reinterpret_cast<const uint4 *>(adj + (size_t)x * 64);
                uint64_t c = 0;
                for (int k = 0; k < dx; k += 8) {
                    const uint4 v = rp[k >> 3];
                    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int n = (int)((wd[j >> 1] >> ((j & 1) * 16)) & 0xFFFFu);
                        // padding slots hold V: count 0, level 0xFFFE
                        if (STAGE) {
                            c = sat_add(c, lcnt[n]);
                        } else if (ld[n] == (uint16_t)(L - 1)) {
                            c = sat_add(c, lcnt[n]);
                        }
                    }
                }
                if (STAGE) stage[i] = c;
                else lcnt[x] = c;
            }
            if (STAGE) {
                __syncthreads();                 // every level-L row read
                for (int i = threadIdx.x; i < total; i += blockDim.x) lcnt[list[i]] = stage[i];
            }
            __syncthreads();                     // level L counted, list free
        }
        for (int x = threadIdx.x; x < V; x += blockDim.x) prow[x] = lcnt[x];
        __syncthreads();
    }
}

// Graphs whose row state does not fit one workgroup's LDS (torus 32^3,
// Jellyfish 100k): the same level DP with the counts kept in the output row
// itself (global memory) and the levels read from the dist row.  Level L's
// vertices are found by a sweep of the dist row; each one sums its CSR
// out-neighbours one level closer.  Only this workgroup touches the row, so
// a barrier (workgroup-scope release/acquire, same CU) orders the levels.
__global__ __launch_bounds__(1024) void ecmp_count_global_kernel(
    int V, int ndst, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const uint16_t *__restrict__ dist, uint64_t *__restrict__ paths)
{
    __shared__ int maxd;
    for (int row = blockIdx.x; row < ndst; row += gridDim.x) {
        const uint16_t *drow = dist + (size_t)row * V;
        uint64_t *prow = paths + (size_t)row * V;
        if (threadIdx.x == 0) maxd = 0;
        __syncthreads();
        int mymax = 0;
        for (int x = threadIdx.x; x < V; x += blockDim.x) {
            const uint16_t dx = drow[x];
            prow[x] = dx == 0 ? 1ull : 0ull;
            if (dx != 0xFFFFu && dx > mymax) mymax = dx;
        }
        atomicMax(&maxd, mymax);
        __syncthreads();
        const int top = maxd;
        for (int L = 1; L <= top; ++L) {
            for (int x = threadIdx.x; x < V; x += blockDim.x) {
                if (drow[x] != (uint16_t)L) continue;
                uint64_t c = 0;
                const int re = row_ptr[x + 1];
                for (int e = row_ptr[x]; e < re; ++e) {
                    const int n = col[e];
                    if (drow[n] == (uint16_t)(L - 1)) c = sat_add(c, prow[n]);
                }
                prow[x] = c;
            }
            __syncthreads();
        }
    }
}

__global__ __launch_bounds__(256) void ecmp_unrank_kernel(
    int V, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const uint16_t *__restrict__ dist, const uint64_t *__restrict__ paths,
    const int32_t *__restrict__ rows, const int32_t *__restrict__ srcs,
    const uint64_t *__restrict__ ranks, int nroutes, int max_len, int32_t *__restrict__ out)
{
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nroutes; k += gridDim.x * blockDim.x) {
        int32_t *o = out + (size_t)k * max_len;
        const size_t rb = (size_t)rows[k] * V;
        int x = srcs[k];
        uint64_t r = ranks[k];
        int len = 0;
        uint32_t dx = dist[rb + x];
        if (dx == 0xFFFFu || r >= paths[rb + x] || (int)dx + 1 > max_len) {
            for (int j = 0; j < max_len; ++j) o[j] = -1;      // no such route
            continue;
        }
        o[len++] = x;
        while (dx > 0) {
            int nxt = -1;
            const int re = row_ptr[x + 1];
            for (int e = row_ptr[x]; e < re; ++e) {
                const int n = col[e];
                if ((uint32_t)dist[rb + n] + 1u != dx) continue;
                const uint64_t c = paths[rb + n];
                if (r < c) {
                    nxt = n;
                    break;
                }
                r -= c;
            }
            if (nxt < 0) break;                               // saturated counts only
            x = nxt;
            --dx;
            o[len++] = x;
        }
        for (int j = len; j < max_len; ++j) o[j] = -1;
    }
}

}  // namespace

int sdnr_launch_ecmp_counts(sdnr_ctx *ctx, const uint16_t *d_dist, int32_t ndst,
                            uint64_t *d_paths)
{
    const int V = ctx->V;
    if (ndst == 0 || V == 0) return SDNR_OK;
    // thread-per-vertex kernel over the 64-wide rows when they exist
    constexpr int NW = 4;
    const size_t cap = SDNR_MAX_LDS_PER_BLOCK - 1024;
    // SDNROUTE_ECMP=global forces the global-memory DP (tests)
    const char *ef = getenv("SDNROUTE_ECMP");
    const bool force_global = ef && !strcmp(ef, "global");
    const bool rows_ok = !force_global && ctx->adj16 != nullptr && ctx->deg32 != nullptr &&
                         V < 65534 && ecmp_wave_lds(V, NW, false) <= cap;
    if (rows_ok) {
        const bool stage = ecmp_wave_lds(V, NW, true) <= cap;
        const size_t wlds = ecmp_wave_lds(V, NW, stage);
        int grid = ctx->num_cus * 8;
        if (grid > ndst) grid = ndst;
        auto k = stage ? ecmp_count_rows_kernel<NW, true> : ecmp_count_rows_kernel<NW, false>;
        sdnr_allow_lds(reinterpret_cast<const void *>(k), wlds);
        ctx->last_kernel = stage ? "ecmp_count_rows_kernel<stage>" : "ecmp_count_rows_kernel";
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
        hipLaunchKernelGGL(k, dim3(grid), dim3(NW * 64), wlds, ctx->stream, V, ndst, ctx->adj16,
                           ctx->deg32, d_dist, d_paths);
        SDNR_HIP(hipGetLastError());
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    const size_t lds = (size_t)V * 10;
    if (force_global || lds > SDNR_MAX_LDS_PER_BLOCK - 1024) {
        // row state in global memory (the output row); one workgroup per row
        int grid = ctx->num_cus * 4;
        if (grid > ndst) grid = ndst;
        ctx->last_kernel = "ecmp_count_global_kernel";
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
        hipLaunchKernelGGL(ecmp_count_global_kernel, dim3(grid), dim3(1024), 0, ctx->stream, V,
                           ndst, ctx->row_ptr, ctx->col, d_dist, d_paths);
        SDNR_HIP(hipGetLastError());
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    int grid = ctx->num_cus * 2;
    if (grid > ndst) grid = ndst;
    sdnr_allow_lds(reinterpret_cast<const void *>(ecmp_count_kernel), lds);
    ctx->last_kernel = "ecmp_count_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipLaunchKernelGGL(ecmp_count_kernel, dim3(grid), dim3(1024), lds, ctx->stream, V, ndst,
                       ctx->row_ptr, ctx->col, d_dist, d_paths);
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}

int sdnr_launch_ecmp_unrank(sdnr_ctx *ctx, const uint16_t *d_dist, const uint64_t *d_paths,
                            const int32_t *d_rows, const int32_t *d_srcs, const uint64_t *d_ranks,
                            int32_t nroutes, int32_t max_len, int32_t *d_out)
{
    if (nroutes == 0) return SDNR_OK;
    int g = (nroutes + 255) / 256;
    if (g > ctx->num_cus * 16) g = ctx->num_cus * 16;
    ctx->last_kernel = "ecmp_unrank_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipLaunchKernelGGL(ecmp_unrank_kernel, dim3(g), dim3(256), 0, ctx->stream, ctx->V, ctx->row_ptr,
                       ctx->col, d_dist, d_paths, d_rows, d_srcs, d_ranks, nroutes, max_len, d_out);
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
