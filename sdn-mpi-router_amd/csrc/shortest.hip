// shortest.hip -- shortest-route tables (find_route(..., multiple=True)).
//
// Reference: TopologyDB._find_routes_bfs (sdnmpi/util/topology_db.py:86-122)
// enumerates all simple paths FIFO and keeps the shortest; FIFO order with
// ascending neighbours (:106) is lexicographic order of the dpid sequence,
// so routes[0] is the lexicographically smallest shortest path: from x the
// next hop toward d is the SMALLEST out-neighbour n with
// dist(n, d) == dist(x, d) - 1, and the full ECMP set is the shortest-path
// DAG walked in ascending order.  Both need dist(., d), computed here:
//
//  * msbfs: multi-source BFS, 64 destinations per 64-bit mask word.  Pull
//    step on the forward CSR (x joins level L+1 of destination b if one of
//    its out-neighbours is in level L of b): next[x] = OR(front[n]) & ~vis[x].
//    For V <= 6400 one 1024-thread workgroup keeps vis/front/next for its 64
//    destinations in LDS (24 B per vertex) and runs every level behind
//    workgroup barriers; larger graphs run one launch per level over all
//    batches with the masks in HBM.
//  * nexthop: per (destination, vertex) the first (= smallest dense id =
//    smallest dpid) out-neighbour one hop closer; the destination's dist row
//    is staged in LDS, one thread per vertex scans its sorted row.
#include "common.h"

namespace {

constexpr int kBfsThreads = 1024;

__device__ __forceinline__ void write_levels(uint64_t nw, int b0, int ndst,
                                             int V, int x, uint16_t lvl,
                                             uint16_t *__restrict__ dist)
{
    while (nw) {
        const int b = __ffsll((unsigned long long)nw) - 1;
        nw &= nw - 1;
        if (b0 + b < ndst) dist[(size_t)(b0 + b) * V + x] = lvl;
    }
}

__global__ __launch_bounds__(kBfsThreads) void msbfs_lds_kernel(
    int V, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ dst, int ndst, uint16_t *__restrict__ dist)
{
    extern __shared__ __attribute__((aligned(16))) uint64_t lmask[];
    uint64_t *vis = lmask;
    uint64_t *front = vis + V;
    uint64_t *next = front + V;
    const int b0 = blockIdx.x * 64;
    const int nb = min(64, ndst - b0);
    for (int x = threadIdx.x; x < V; x += blockDim.x) {
        vis[x] = 0;
        front[x] = 0;
    }
    __syncthreads();
    if (threadIdx.x < nb) {
        const int d = dst[b0 + threadIdx.x];
        if (d >= 0 && d < V) {
            atomicOr((unsigned long long *)&vis[d], 1ull << threadIdx.x);
            atomicOr((unsigned long long *)&front[d], 1ull << threadIdx.x);
            dist[(size_t)(b0 + threadIdx.x) * V + d] = 0;
        }
    }
    __syncthreads();
    for (int lvl = 1; lvl < 0xFFFF; ++lvl) {
        int any = 0;
        for (int x = threadIdx.x; x < V; x += blockDim.x) {
            uint64_t acc = 0;
            const int re = row_ptr[x + 1];
            for (int e = row_ptr[x]; e < re; ++e) acc |= front[col[e]];
            const uint64_t nw = acc & ~vis[x];
            next[x] = nw;
            if (nw) {
                any = 1;
                vis[x] |= nw;
                write_levels(nw, b0, ndst, V, x, (uint16_t)lvl, dist);
            }
        }
        if (!__syncthreads_or(any)) break;
        uint64_t *t = front;
        front = next;
        next = t;
    }
}

// one BFS level for every batch; masks [nbatch][V] in global memory
__global__ __launch_bounds__(256) void msbfs_level_kernel(
    int V, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    int ndst, int lvl, const uint64_t *__restrict__ front,
    uint64_t *__restrict__ next, uint64_t *__restrict__ vis,
    uint16_t *__restrict__ dist, int *__restrict__ changed)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int batch = blockIdx.y;
    if (x >= V) return;
    const size_t off = (size_t)batch * V;
    uint64_t acc = 0;
    const int re = row_ptr[x + 1];
    for (int e = row_ptr[x]; e < re; ++e) acc |= front[off + col[e]];
    const uint64_t nw = acc & ~vis[off + x];
    next[off + x] = nw;
    if (nw) {
        vis[off + x] |= nw;
        write_levels(nw, batch * 64, ndst, V, x, (uint16_t)lvl, dist);
        *changed = 1;
    }
}

__global__ __launch_bounds__(256) void msbfs_seed_kernel(
    int V, const int32_t *__restrict__ dst, int ndst, uint64_t *__restrict__ front,
    uint64_t *__restrict__ vis, uint16_t *__restrict__ dist)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ndst) return;
    const int d = dst[i];
    if (d < 0 || d >= V) return;
    const size_t off = (size_t)(i >> 6) * V + d;
    atomicOr((unsigned long long *)&front[off], 1ull << (i & 63));
    atomicOr((unsigned long long *)&vis[off], 1ull << (i & 63));
    dist[(size_t)i * V + d] = 0;
}

// nh/nh_port for destination blockIdx.y, vertices in blockIdx.x's range
__global__ __launch_bounds__(256) void nexthop_kernel(
    int V, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ port, const uint16_t *__restrict__ dist,
    int32_t *__restrict__ nh, int32_t *__restrict__ nh_port, int stage)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t ldist[];
    const size_t row = (size_t)blockIdx.y * V;
    const uint16_t *drow = dist + row;
    if (stage) {
        for (int x = threadIdx.x; x < V; x += blockDim.x) ldist[x] = drow[x];
        __syncthreads();
        drow = ldist;
    }
    const int per = (V + gridDim.x - 1) / gridDim.x;
    const int lo = blockIdx.x * per;
    const int hi = min(V, lo + per);
    for (int x = lo + threadIdx.x; x < hi; x += blockDim.x) {
        const uint32_t dx = drow[x];
        int best = -1, bport = -1;
        if (dx != 0xFFFFu && dx != 0u) {
            const int re = row_ptr[x + 1];
            for (int e = row_ptr[x]; e < re; ++e) {
                const int n = col[e];
                if ((uint32_t)drow[n] + 1u == dx) {
                    best = n;
                    bport = port[e];
                    break;
                }
            }
        }
        nh[row + x] = best;
        nh_port[row + x] = bport;
    }
}

}  // namespace

int sdnr_launch_shortest(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst,
                         uint16_t *d_dist, int32_t *d_nh, int32_t *d_nh_port)
{
    const int V = ctx->V;
    if (ndst == 0 || V == 0) return SDNR_OK;
    const int nbatch = (ndst + 63) / 64;
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    SDNR_HIP(hipMemsetAsync(d_dist, 0xFF, (size_t)ndst * V * sizeof(uint16_t), ctx->stream));
    const size_t lds = (size_t)V * 3 * sizeof(uint64_t);
    ctx->last_kernel = lds <= 150 * 1024 ? "msbfs_lds_kernel+nexthop_kernel"
                                         : "msbfs_level_kernel+nexthop_kernel";
    if (lds <= 150 * 1024) {
        auto k = msbfs_lds_kernel;
        if (lds > 64 * 1024) sdnr_allow_lds(reinterpret_cast<const void *>(k), lds);
        hipLaunchKernelGGL(k, dim3(nbatch), dim3(kBfsThreads), lds, ctx->stream, V,
                           ctx->row_ptr, ctx->col, d_dst, ndst, d_dist);
        SDNR_HIP(hipGetLastError());
    } else {
        const size_t mbytes = (size_t)nbatch * V * sizeof(uint64_t);
        int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes, 3 * mbytes + 256);
        if (rc) return rc;
        char *base = static_cast<char *>(ctx->scratch);
        uint64_t *front = reinterpret_cast<uint64_t *>(base);
        uint64_t *next = reinterpret_cast<uint64_t *>(base + mbytes);
        uint64_t *vis = reinterpret_cast<uint64_t *>(base + 2 * mbytes);
        int *changed = reinterpret_cast<int *>(base + 3 * mbytes);
        SDNR_HIP(hipMemsetAsync(base, 0, 3 * mbytes + 256, ctx->stream));
        hipLaunchKernelGGL(msbfs_seed_kernel, dim3((ndst + 255) / 256), dim3(256), 0,
                           ctx->stream, V, d_dst, ndst, front, vis, d_dist);
        SDNR_HIP(hipGetLastError());
        int h_changed = 1;
        for (int lvl = 1; lvl < 0xFFFF && h_changed; ++lvl) {
            SDNR_HIP(hipMemsetAsync(changed, 0, sizeof(int), ctx->stream));
            hipLaunchKernelGGL(msbfs_level_kernel, dim3((V + 255) / 256, nbatch), dim3(256),
                               0, ctx->stream, V, ctx->row_ptr, ctx->col, ndst, lvl,
                               front, next, vis, d_dist, changed);
            SDNR_HIP(hipGetLastError());
            SDNR_HIP(hipMemcpyAsync(&h_changed, changed, sizeof(int), hipMemcpyDeviceToHost,
                                    ctx->stream));
            SDNR_HIP(hipStreamSynchronize(ctx->stream));
            uint64_t *t = front;
            front = next;
            next = t;
        }
    }
    if (d_nh && d_nh_port) {
        const int stage = (size_t)V * 2 <= 64 * 1024;
        int gx = (V + 1023) / 1024;
        if (gx < 1) gx = 1;
        hipLaunchKernelGGL(nexthop_kernel, dim3(gx, ndst), dim3(256),
                           stage ? (size_t)V * 2 : 0, ctx->stream, V, ctx->row_ptr,
                           ctx->col, ctx->port, d_dist, d_nh, d_nh_port, stage);
        SDNR_HIP(hipGetLastError());
    }
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
