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
//  * ecmp_unrank_kernel: route r of (x, d) in lexicographic order: at each
//    vertex take the ascending out-neighbours one hop closer and descend
//    into the one whose count range holds r (r -= paths[n] for the ones
//    skipped).  One thread per route; the vertex sequence is written to a
//    fixed-stride slot.
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
    const size_t lds = (size_t)V * 10;
    if (lds > SDNR_MAX_LDS_PER_BLOCK - 1024)
        return sdnr_fail(SDNR_ERR_INVAL, "ecmp counts: V=%d too large for one workgroup", V);
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
