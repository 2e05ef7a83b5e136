// incremental.hip -- which cached default-route rows a link change alters.
//
// Ryu's EventLinkAdd / EventLinkDelete reach TopologyDB.
// add_link / delete_link (reference sdnmpi/topology.py:192-198,
// sdnmpi/util/topology_db.py:30-42).  A cached tree row (the tree of first
// pushes of _find_route_dfs, topology_db.py:59-84, from source s) changes iff
//  * removed or re-ported link (u, v): it is the tree edge into v,
//    parent_s[v] == u (the search looks at (u, v) only when it pops u and
//    pushes v only if v is unvisited then);
//  * added link (u, v), u != v, v != s: u is reached and v is still unvisited
//    when u is popped -- v unreached, or v pushed (by p = parent_s[v]) in a pop
//    that comes after u's.  Pops follow the tree's preorder with children in
//    DESCENDING id order (LIFO over ascending pushes), so "after" is decided
//    from the two root paths: an ancestor pops first; otherwise, below the
//    lowest common ancestor, the branch of the larger child pops first.
// One thread per (row, link) climbs the two tree paths with dependent loads
// of the row's own tree words and depths (the pool's compact rows, decoded
// in place); round 4 did the same climb as one torch op and one host sync per
// tree level (incremental.py), 40-180 ms per add_link on k=48.
#include "common.h"

namespace {

struct TreeRows {
    const uint32_t *tree;     // [rows][V]: port16 / slot words, or int32 parents
    const void *depth;        // [rows][V]: u16 (0xFFFF unreached) or int32 (-1)
    int layout;               // SDNR_TREE_INT32 / SDNR_TREE_PORT16 / SDNR_TREE_SLOT
    int depth_bytes;          // 2 or 4
};

__device__ __forceinline__ int parent_of(const TreeRows &t, size_t rb, int x)
{
    const uint32_t w = t.tree[rb + x];
    if (t.layout == SDNR_TREE_PORT16) {
        const int p = (int)(w & 0xFFFFu);
        return p == 0xFFFF ? -1 : p;
    }
    if (t.layout == SDNR_TREE_SLOT) return w == 0xFFFFFFFFu ? -1 : (int)(w & 0x3FFFFFFu);
    return (int)w;
}

__device__ __forceinline__ int depth_of(const TreeRows &t, size_t rb, int x)
{
    if (t.depth_bytes == 2) {
        const uint16_t d = static_cast<const uint16_t *>(t.depth)[rb + x];
        return d == 0xFFFF ? -1 : (int)d;
    }
    return static_cast<const int32_t *>(t.depth)[rb + x];
}

// a popped before b in the traversal of row rb (both reached, a != b);
// false + *bad when the tree is inconsistent (a climb longer than V steps)
__device__ bool popped_before(const TreeRows &t, size_t rb, int V, int a, int b, bool *bad)
{
    int x = a, y = b;
    int hx = depth_of(t, rb, x), hy = depth_of(t, rb, y);
    const bool b_deeper = hy > hx;
    int steps = 0;
    while (hx > hy && x >= 0) {                  // lift the deeper one
        x = parent_of(t, rb, x);
        --hx;
        if (++steps > V) break;
    }
    while (hy > hx && y >= 0) {
        y = parent_of(t, rb, y);
        --hy;
        if (++steps > V) break;
    }
    if (x < 0 || y < 0 || steps > V) {
        *bad = true;
        return false;
    }
    if (x == y) return b_deeper;                  // one is the other's ancestor
    for (;;) {                                    // climb together to the LCA's children
        const int px = parent_of(t, rb, x), py = parent_of(t, rb, y);
        if (px == py) return x > y;               // the larger child's branch pops first
        if (px < 0 || py < 0 || ++steps > V) {
            *bad = true;
            return false;
        }
        x = px;
        y = py;
    }
}

// thread (row r, link k): links [0, nrm) removed / re-ported, [nrm, nrm +
// nadd) added; affected[r] |= 1 when the link alters row r
__global__ __launch_bounds__(256) void dfs_rows_affected_kernel(
    TreeRows t, int V, int nrows, const int32_t *__restrict__ row_src,
    const int32_t *__restrict__ links, int nrm, int nadd, uint8_t *__restrict__ affected,
    int *__restrict__ err)
{
    const int nl = nrm + nadd;
    const int64_t total = (int64_t)nrows * nl;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int r = (int)(i / nl), k = (int)(i % nl);
        const int s = row_src[r];
        if (s < 0) continue;                      // a free pool slot
        if (*reinterpret_cast<volatile const uint8_t *>(&affected[r]))
            continue;                             // another link already flagged it
        const int u = links[2 * k], v = links[2 * k + 1];
        if (u < 0 || u >= V || v < 0 || v >= V) continue;
        const size_t rb = (size_t)r * V;
        bool hit;
        if (k < nrm) {
            hit = parent_of(t, rb, v) == u && v != s;
        } else {
            if (u == v || v == s || parent_of(t, rb, u) < 0) continue;   // u unreached: never popped
            const int pv = parent_of(t, rb, v);
            if (pv < 0) {
                hit = true;                       // v unreached: u's pop now pushes it
            } else {
                bool bad = false;
                hit = !popped_before(t, rb, V, pv, u, &bad);
                if (bad) atomicOr(err, kErrTreeClimb);
            }
        }
        if (hit) affected[r] = 1;
    }
}

}  // namespace

int sdnr_launch_dfs_rows_affected(sdnr_ctx *ctx, const uint32_t *d_tree, const void *d_depth,
                                  int32_t layout, int32_t depth_bytes, int32_t nrows,
                                  const int32_t *d_row_src, const int32_t *d_links, int32_t nrm,
                                  int32_t nadd, uint8_t *d_affected)
{
    SDNR_HIP(hipMemsetAsync(d_affected, 0, (size_t)nrows, ctx->stream));
    const int64_t total = (int64_t)nrows * (nrm + nadd);
    if (total == 0) return SDNR_OK;
    int64_t g = (total + 255) / 256;
    if (g > (int64_t)ctx->num_cus * 16) g = (int64_t)ctx->num_cus * 16;
    ctx->last_kernel = "dfs_rows_affected_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    TreeRows t{d_tree, d_depth, layout, depth_bytes};
    hipLaunchKernelGGL(dfs_rows_affected_kernel, dim3((unsigned)g), dim3(256), 0, ctx->stream, t,
                       ctx->V, nrows, d_row_src, d_links, nrm, nadd, d_affected, ctx->d_err);
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
