// dfs.hip -- reference-exact default-route tables on gfx950.
//
// Reference: TopologyDB._find_route_dfs (sdnmpi/util/topology_db.py:59-84):
// a LIFO stack search where a switch is marked visited when it is PUSHED
// (:78-82) and neighbours are pushed in ascending dpid order (:76).  The
// parent of v is fixed by the pop that first pushes it, and stopping at the
// destination (:70-71) happens after that push, so one full traversal from
// s answers find_route(s, d) for EVERY d: the route is the path from s to d
// in the tree of first pushes.  That traversal is serial pop after pop, so
// the kernels run one source per wavefront and make the pop chain short:
//
//  * one pop = one coalesced load of u's adjacency row (ELL rows of width
//    W <= 64 are addressed as u*W: no row_ptr load on the chain), a gather of
//    the visited bits from LDS, __ballot over the row, mbcnt ranks for the
//    ascending push order, and ds_or to mark;
//  * the largest freshly pushed child is the next pop (LIFO), so it stays in
//    an SGPR instead of going through the stack;
//  * dfs_lds_kernel (V < 65536, small graphs): visited bits, stack, parent,
//    slot and depth live in LDS (10 B per vertex) and the tables are written
//    once, coalesced, after the traversal -- no global store on the chain;
//  * dfs_global_kernel (large graphs): visited bits and a 1024-entry stack
//    ring in LDS, spilled to / refilled from global scratch in halves;
//    table entries are stored as vertices are pushed.
//
// Sources are independent: persistent grid, one 64-thread workgroup per
// source, grid-stride over sources.
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int kRing = 1024;   // LDS stack ring entries (global mode)

template <bool ELL, bool HOPS>
__global__ __launch_bounds__(64) void dfs_lds_wide_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;                       // visited bits
    uint32_t *stk = vis + VWp;                 // stack: v | depth << 16
    uint32_t *ps = stk + V;                    // parent | row slot << 16
    uint16_t *dep = reinterpret_cast<uint16_t *>(ps + V);
    const int lane = lane_id();

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {                 // unknown source: empty row
            for (int v = lane; v < V; v += SDNR_WAVE) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int w = lane; w < VW; w += SDNR_WAVE) vis[w] = 0u;
        __syncthreads();
        if (lane == 0) {
            vis[s >> 5] = 1u << (s & 31);
            ps[s] = (uint32_t)s;
            dep[s] = 0;
        }
        __syncthreads();

        int sp = 0, u = s, du = 0;
        for (;;) {
            int rs, re;
            if (ELL) {
                rs = u * W;
                re = rs + W;
            } else {
                rs = row_ptr[u];
                re = row_ptr[u + 1];
            }
            int nxt = -1;
            for (int base = rs; base < re; base += SDNR_WAVE) {
                const int e = base + lane;
                int v = -1;
                if (e < re) v = col[e];
                bool unv = false;
                if (v >= 0) unv = ((vis[v >> 5] >> (v & 31)) & 1u) == 0u;
                const uint64_t m = __ballot(unv);
                if (m == 0) continue;
                const int cnt = __popcll(m);
                const int rank = lanes_below(m);
                const uint32_t dtag = (uint32_t)(du + 1) << 16;
                if (nxt >= 0) {                // previous chunk's top goes below
                    if (lane == 0) stk[sp] = (uint32_t)nxt | dtag;
                    sp += 1;
                }
                if (unv) {
                    atomicOr(&vis[v >> 5], 1u << (v & 31));
                    ps[v] = (uint32_t)u | ((uint32_t)(e - rs) << 16);
                    if (HOPS) dep[v] = (uint16_t)(du + 1);
                    if (rank < cnt - 1) stk[sp + rank] = (uint32_t)v | dtag;
                }
                sp += cnt - 1;
                nxt = read_lane(v, highest_lane(m));
            }
            if (nxt >= 0) {
                u = nxt;
                du += 1;
            } else {
                if (sp == 0) break;
                sp -= 1;
                const uint32_t ent = (uint32_t)uniform((int)stk[sp]);
                u = (int)(ent & 0xFFFFu);
                du = (int)(ent >> 16);
            }
        }
        __syncthreads();

        for (int v = lane; v < V; v += SDNR_WAVE) {
            int p = -1, pt = -1, h = -1;
            if ((vis[v >> 5] >> (v & 31)) & 1u) {
                const uint32_t x = ps[v];
                p = (int)(x & 0xFFFFu);
                if (v == s) {
                    h = 0;
                } else {
                    const int slot = (int)(x >> 16);
                    pt = ELL ? port[(size_t)p * W + slot] : port[row_ptr[p] + slot];
                    h = HOPS ? (int)dep[v] : 0;
                }
            }
            prow[v] = p;
            trow[v] = pt;
            if (HOPS) hrow[v] = h;
        }
        __syncthreads();
    }
}

template <bool ELL, bool HOPS>
__global__ __launch_bounds__(64) void dfs_global_wide_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops,
    uint2 *__restrict__ spill_all)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;
    uint2 *ring = reinterpret_cast<uint2 *>(vis + VWp);   // (v, depth)
    uint2 *spill = spill_all + (size_t)blockIdx.x * (size_t)V;
    const int lane = lane_id();

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = lane; v < V; v += SDNR_WAVE) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int w = lane; w < VW; w += SDNR_WAVE) vis[w] = 0u;
        __syncthreads();
        if (lane == 0) {
            vis[s >> 5] = 1u << (s & 31);
            prow[s] = s;
            trow[s] = -1;
            if (HOPS) hrow[s] = 0;
        }
        __syncthreads();

        int lsp = 0, bot = 0, gsp = 0;        // ring depth, ring bottom, spilled
        int u = s, du = 0;
        for (;;) {
            int rs, re;
            if (ELL) {
                rs = u * W;
                re = rs + W;
            } else {
                rs = row_ptr[u];
                re = row_ptr[u + 1];
            }
            int nxt = -1;
            for (int base = rs; base < re; base += SDNR_WAVE) {
                const int e = base + lane;
                int v = -1, pt = -1;
                if (e < re) {
                    v = col[e];
                    pt = port[e];
                }
                bool unv = false;
                if (v >= 0) unv = ((vis[v >> 5] >> (v & 31)) & 1u) == 0u;
                const uint64_t m = __ballot(unv);
                if (m == 0) continue;
                const int cnt = __popcll(m);
                const int rank = lanes_below(m);
                if (unv) {
                    atomicOr(&vis[v >> 5], 1u << (v & 31));
                    prow[v] = u;
                    trow[v] = pt;
                    if (HOPS) hrow[v] = du + 1;
                }
                if (lsp + cnt > kRing) {       // spill the oldest half
                    for (int i = lane; i < kRing / 2; i += SDNR_WAVE)
                        spill[gsp + i] = ring[(bot + i) & (kRing - 1)];
                    gsp += kRing / 2;
                    bot = (bot + kRing / 2) & (kRing - 1);
                    lsp -= kRing / 2;
                }
                const uint32_t dn = (uint32_t)(du + 1);
                if (nxt >= 0) {
                    if (lane == 0) ring[(bot + lsp) & (kRing - 1)] = make_uint2((uint32_t)nxt, dn);
                    lsp += 1;
                }
                if (unv && rank < cnt - 1)
                    ring[(bot + lsp + rank) & (kRing - 1)] = make_uint2((uint32_t)v, dn);
                lsp += cnt - 1;
                nxt = read_lane(v, highest_lane(m));
            }
            if (nxt >= 0) {
                u = nxt;
                du += 1;
                continue;
            }
            if (lsp == 0) {
                if (gsp == 0) break;
                const int n = gsp < kRing / 2 ? gsp : kRing / 2;
                // the spill was written by this wave: wait for the stores and
                // drop this CU's L1 copy before reading it back
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                bot = (bot - n) & (kRing - 1);
                for (int i = lane; i < n; i += SDNR_WAVE)
                    ring[(bot + i) & (kRing - 1)] = spill[gsp - n + i];
                gsp -= n;
                lsp = n;
            }
            lsp -= 1;
            const uint2 ent = ring[(bot + lsp) & (kRing - 1)];
            u = uniform((int)ent.x);
            du = uniform((int)ent.y);
        }
        __syncthreads();
        for (int v = lane; v < V; v += SDNR_WAVE) {
            if (((vis[v >> 5] >> (v & 31)) & 1u) == 0u) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Batched pops.  A pop that finds no unvisited neighbour (a "leaf" pop)
// changes nothing -- no mark, no push -- so a run of leaf pops can be checked
// against the same visited set in any order.  The batched kernels read the
// top K stack entries, issue the K row loads and then the K visited gathers
// back to back (one memory latency for K pops instead of K), and take the
// first entry from the top that has an unvisited neighbour: everything above
// it was a leaf pop, it is processed exactly as the sequential search would,
// and everything below stays on the stack for the next batch (its check is
// stale).  On the k=48 fat-tree 96% of pops are leaves.
//
// Rows must fit one wavefront (max out-degree <= 64): ELL rows at u*W, or
// CSR rows (row_ptr loads issued with the batch).  Adjacency arrays carry 64
// padding entries so every lane may load unconditionally (a guarded load per
// batch slot makes hipcc wait vmcnt(0) per slot).
// ---------------------------------------------------------------------------

template <bool ELL, int K>
__device__ __forceinline__ void batch_rows(int kk, const int (&uu)[K], int W,
                                           const int32_t *__restrict__ row_ptr,
                                           const int32_t *__restrict__ col,
                                           int (&rs)[K], int (&v)[K])
{
    // every slot loads unconditionally (addresses stay inside the padded
    // arrays); validity is applied afterwards with bit masks, never with a
    // branch, so the K loads are all in flight together
    const int lane = lane_id();
    int x[K], b[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const int u = uu[i];
        if (ELL) {
            rs[i] = u * W;
            b[i] = rs[i] + W;
        } else {
            rs[i] = row_ptr[u];
            b[i] = row_ptr[u + 1];
        }
        x[i] = col[rs[i] + lane];
    }
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const int ok = -(int)((i < kk) & (rs[i] + lane < b[i]));   // 0 or -1
        v[i] = (x[i] & ok) | ~ok;
    }
}

// visited test of K candidate rows: K independent LDS gathers, then ballots
template <int K>
__device__ __forceinline__ void batch_unvisited(const uint32_t *vis, const int (&v)[K],
                                                uint64_t (&m)[K])
{
    uint32_t w[K];
#pragma unroll
    for (int i = 0; i < K; ++i) w[i] = vis[(v[i] & 0x7FFFFFFF) >> 5 & ((v[i] >> 31) ^ -1)];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const bool fresh = (v[i] >= 0) & (((w[i] >> (v[i] & 31)) & 1u) == 0u);
        m[i] = __ballot(fresh);
    }
}

template <int K>
__device__ __forceinline__ int first_live(const uint64_t (&m)[K])
{
    int istar = K;
#pragma unroll
    for (int i = K - 1; i >= 0; --i)
        if (m[i] != 0) istar = i;
    return istar;
}

// small graphs (V < 65536): all per-source state in LDS, tables flushed once
template <bool ELL, bool HOPS, int K>
__global__ __launch_bounds__(64) void dfs_lds_batch_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;                       // visited bits
    uint32_t *stk = vis + VWp;                 // stack: v | depth << 16
    uint32_t *ps = stk + V;                    // parent | row slot << 16
    uint16_t *dep = reinterpret_cast<uint16_t *>(ps + V);
    const int lane = lane_id();

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = lane; v < V; v += SDNR_WAVE) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int w = lane; w < VW; w += SDNR_WAVE) vis[w] = 0u;
        __syncthreads();
        if (lane == 0) {
            vis[s >> 5] = 1u << (s & 31);
            ps[s] = (uint32_t)s;
            dep[s] = 0;
            stk[0] = (uint32_t)s;
        }
        __syncthreads();

        int sp = 1;
        while (sp > 0) {
            const int kk = sp < K ? sp : K;
            const int slot = sp - 1 - lane;
            uint32_t mine = stk[slot < 0 ? 0 : slot];
            mine = lane < kk ? mine : 0u;            // slots past the stack: vertex 0
            uint32_t ent[K];
            int uu[K];
#pragma unroll
            for (int i = 0; i < K; ++i) {
                ent[i] = (uint32_t)read_lane((int)mine, i);
                uu[i] = (int)(ent[i] & 0xFFFFu);
            }
            int rs[K], v[K];
            batch_rows<ELL, K>(kk, uu, W, row_ptr, col, rs, v);
            uint64_t m[K];
            batch_unvisited<K>(vis, v, m);
            const int istar = first_live<K>(m);
            if (istar == K) {                      // kk leaf pops
                sp -= kk;
                continue;
            }
            sp -= istar + 1;
            uint64_t mm = 0;
            int vv = -1;
            uint32_t eu = 0;
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i == istar) {
                    mm = m[i];
                    vv = v[i];
                    eu = ent[i];
                }
            const int u = (int)(eu & 0xFFFFu);
            const int du = (int)(eu >> 16);
            if ((mm >> lane) & 1ull) {
                const int rank = lanes_below(mm);
                atomicOr(&vis[vv >> 5], 1u << (vv & 31));
                ps[vv] = (uint32_t)u | ((uint32_t)lane << 16);
                if (HOPS) dep[vv] = (uint16_t)(du + 1);
                stk[sp + rank] = (uint32_t)vv | ((uint32_t)(du + 1) << 16);
            }
            sp += __popcll(mm);
        }
        __syncthreads();

        for (int v = lane; v < V; v += SDNR_WAVE) {
            int p = -1, pt = -1, h = -1;
            if ((vis[v >> 5] >> (v & 31)) & 1u) {
                const uint32_t x = ps[v];
                p = (int)(x & 0xFFFFu);
                if (v == s) {
                    h = 0;
                } else {
                    const int slot = (int)(x >> 16);
                    pt = ELL ? port[(size_t)p * W + slot] : port[row_ptr[p] + slot];
                    h = HOPS ? (int)dep[v] : 0;
                }
            }
            prow[v] = p;
            trow[v] = pt;
            if (HOPS) hrow[v] = h;
        }
        __syncthreads();
    }
}

// large graphs: visited bits + a stack ring in LDS (spilled to HBM in
// halves), table entries stored as vertices are pushed
template <bool ELL, bool HOPS, int K>
__global__ __launch_bounds__(64) void dfs_global_batch_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops,
    uint2 *__restrict__ spill_all)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;
    uint2 *ring = reinterpret_cast<uint2 *>(vis + VWp);   // (v, depth)
    uint2 *spill = spill_all + (size_t)blockIdx.x * (size_t)V;
    const int lane = lane_id();

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = lane; v < V; v += SDNR_WAVE) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int w = lane; w < VW; w += SDNR_WAVE) vis[w] = 0u;
        __syncthreads();
        if (lane == 0) {
            vis[s >> 5] = 1u << (s & 31);
            prow[s] = s;
            trow[s] = -1;
            if (HOPS) hrow[s] = 0;
            ring[0] = make_uint2((uint32_t)s, 0u);
        }
        __syncthreads();

        int lsp = 1, bot = 0, gsp = 0;        // ring depth, ring bottom, spilled
        for (;;) {
            if (lsp == 0) {
                if (gsp == 0) break;
                const int n = gsp < kRing / 2 ? gsp : kRing / 2;
                // the spill was written by this wave: wait for the stores and
                // drop this CU's L1 copy before reading it back
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                bot = (bot - n) & (kRing - 1);
                for (int i = lane; i < n; i += SDNR_WAVE)
                    ring[(bot + i) & (kRing - 1)] = spill[gsp - n + i];
                gsp -= n;
                lsp = n;
            }
            const int kk = lsp < K ? lsp : K;
            uint2 me = ring[(bot + lsp - 1 - lane) & (kRing - 1)];
            me.x = lane < kk ? me.x : 0u;            // slots past the stack: vertex 0
            me.y = lane < kk ? me.y : 0u;
            uint32_t ent[K], edep[K];
#pragma unroll
            for (int i = 0; i < K; ++i) {
                ent[i] = (uint32_t)read_lane((int)me.x, i);
                edep[i] = (uint32_t)read_lane((int)me.y, i);
            }
            int uu[K];
#pragma unroll
            for (int i = 0; i < K; ++i) uu[i] = (int)ent[i];
            int rs[K], v[K];
            batch_rows<ELL, K>(kk, uu, W, row_ptr, col, rs, v);
            uint64_t m[K];
            batch_unvisited<K>(vis, v, m);
            const int istar = first_live<K>(m);
            if (istar == K) {
                lsp -= kk;
                continue;
            }
            lsp -= istar + 1;
            uint64_t mm = 0;
            int vv = -1, r0 = 0;
            uint32_t eu = 0, ed = 0;
#pragma unroll
            for (int i = 0; i < K; ++i)
                if (i == istar) {
                    mm = m[i];
                    vv = v[i];
                    eu = ent[i];
                    ed = edep[i];
                    r0 = rs[i];
                }
            const int cnt = __popcll(mm);
            if (lsp + cnt > kRing) {               // spill the oldest half
                for (int i = lane; i < kRing / 2; i += SDNR_WAVE)
                    spill[gsp + i] = ring[(bot + i) & (kRing - 1)];
                gsp += kRing / 2;
                bot = (bot + kRing / 2) & (kRing - 1);
                lsp -= kRing / 2;
            }
            if ((mm >> lane) & 1ull) {
                const int rank = lanes_below(mm);
                atomicOr(&vis[vv >> 5], 1u << (vv & 31));
                prow[vv] = (int)eu;
                trow[vv] = port[r0 + lane];
                if (HOPS) hrow[vv] = (int)ed + 1;
                ring[(bot + lsp + rank) & (kRing - 1)] = make_uint2((uint32_t)vv, ed + 1u);
            }
            lsp += cnt;
        }
        __syncthreads();
        for (int v = lane; v < V; v += SDNR_WAVE) {
            if (((vis[v >> 5] >> (v & 31)) & 1u) == 0u) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Cooperative batched pops (small graphs, the k=48 headline path).
//
// With one wavefront per source the batched loop is instruction-issue bound
// (one wave per SIMD pays >= 4 cycles per instruction on the chain).  Here a
// workgroup of NW waves owns one source: each wave checks KW of the K = NW*KW
// top stack entries (row load + visited gather + ballot), publishes one flag
// word per wave, and after one barrier every wave derives the same first
// live slot; the owning wave pushes, and a second barrier publishes the push
// (skipped when all K entries were leaf pops).  Rows are u16 with stride 64
// (one 128-byte line each) padded with a sentinel vertex V whose visited bit
// is always set, and row V is all sentinel: no lane or slot needs a validity
// mask.  Every wave keeps its own copy of the stack depth; all copies follow
// the same deterministic updates.
// ---------------------------------------------------------------------------
template <int NW, int KW, bool HOPS>
__global__ __launch_bounds__(NW * 64) void dfs_coop_kernel(
    int V, const uint16_t *__restrict__ adj, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ port, const int32_t *__restrict__ src, int nsrc,
    int32_t *__restrict__ out_parent, int32_t *__restrict__ out_port,
    int32_t *__restrict__ out_hops)
{
    constexpr int K = NW * KW;
    static_assert(K <= 64, "one flag bit per slot");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 1 + 31) >> 5;            // + sentinel bit V
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;
    uint32_t *stk = vis + VWp;                   // v | depth << 16
    uint32_t *ps = stk + V;                      // parent | row slot << 16
    uint16_t *dep = reinterpret_cast<uint16_t *>(ps + V);
    uint32_t *xch = ps + V + ((V + 1) >> 1);     // flags[2][NW], count[2]
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int i = threadIdx.x; i < VW; i += blockDim.x) vis[i] = 0u;
        __syncthreads();
        if (threadIdx.x == 0) {
            vis[s >> 5] |= 1u << (s & 31);
            vis[V >> 5] |= 1u << (V & 31);
            ps[s] = (uint32_t)s;
            dep[s] = 0;
            stk[0] = (uint32_t)s;
        }
        __syncthreads();

        int sp = 1, par = 0;
        while (sp > 0) {
            const int kk = sp < K ? sp : K;
            const int slot = w * KW + lane;
            const int at = sp - 1 - slot;
            uint32_t mine = stk[at < 0 ? 0 : at];
            mine = slot < kk ? mine : (uint32_t)V;          // past the stack: sentinel row
            uint32_t ent[KW];
            int x[KW];
#pragma unroll
            for (int j = 0; j < KW; ++j) ent[j] = (uint32_t)read_lane((int)mine, j);
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                const uint16_t *row = adj + (size_t)(ent[j] & 0xFFFFu) * 64;
                x[j] = row[lane];
            }
            uint32_t wd[KW];
#pragma unroll
            for (int j = 0; j < KW; ++j) wd[j] = vis[x[j] >> 5];
            uint64_t m[KW];
            uint32_t fl = 0;
#pragma unroll
            for (int j = 0; j < KW; ++j) {
                m[j] = __ballot(((wd[j] >> (x[j] & 31)) & 1u) == 0u);
                fl |= (m[j] != 0 ? 1u : 0u) << j;
            }
            if (lane == 0) xch[par * NW + w] = fl;
            __syncthreads();
            const uint32_t fw = xch[par * NW + (lane < NW ? lane : 0)];
            uint64_t gm = 0;
#pragma unroll
            for (int q = 0; q < NW; ++q) gm |= (uint64_t)(uint32_t)read_lane((int)fw, q) << (q * KW);
            if (gm == 0) {                               // K leaf pops
                sp -= kk;
                par ^= 1;
                continue;
            }
            const int istar = __ffsll((unsigned long long)gm) - 1;
            sp -= istar + 1;
            if (w == istar / KW) {
                const int js = istar % KW;
                uint64_t mm = 0;
                int xv = 0;
                uint32_t eu = 0;
#pragma unroll
                for (int j = 0; j < KW; ++j)
                    if (j == js) {
                        mm = m[j];
                        xv = x[j];
                        eu = ent[j];
                    }
                const int u = (int)(eu & 0xFFFFu);
                const uint32_t dn = (eu >> 16) + 1u;
                if ((mm >> lane) & 1ull) {
                    atomicOr(&vis[xv >> 5], 1u << (xv & 31));
                    ps[xv] = (uint32_t)u | ((uint32_t)lane << 16);
                    if (HOPS) dep[xv] = (uint16_t)dn;
                    stk[sp + lanes_below(mm)] = (uint32_t)xv | (dn << 16);
                }
                if (lane == 0) xch[2 * NW + par] = (uint32_t)__popcll(mm);
            }
            __syncthreads();
            sp += (int)xch[2 * NW + par];
            par ^= 1;
        }
        __syncthreads();

        for (int v = threadIdx.x; v < V; v += blockDim.x) {
            int p = -1, pt = -1, h = -1;
            if ((vis[v >> 5] >> (v & 31)) & 1u) {
                const uint32_t xx = ps[v];
                p = (int)(xx & 0xFFFFu);
                if (v == s) {
                    h = 0;
                } else {
                    pt = port[row_ptr[p] + (int)(xx >> 16)];
                    h = HOPS ? (int)dep[v] : 0;
                }
            }
            prow[v] = p;
            trow[v] = pt;
            if (HOPS) hrow[v] = h;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Counted pops (small graphs with in/out-degree <= 64): the k=48 headline.
//
// cnt[u] = number of out-neighbours of u not yet visited.  A pop is a leaf
// pop exactly when cnt[u] == 0, so runs of leaf pops are skipped 64 stack
// entries at a time: one LDS read of the stack slots, one gather of their
// counts, one ballot -- no adjacency row is touched.  The price is moved to
// push time, where it is parallel: a vertex v that becomes visited
// decrements cnt[x] for every in-neighbour x (its reverse row, loaded with
// the other children's rows in flight together, then ds_sub_u32 on packed
// u16 pairs -- a count never drops below zero, so no borrow crosses halves).
// Only the non-leaf pops (~4% on the k=48 fat-tree) load a forward row and
// gather visited bits.  A workgroup of NW waves owns one source: every wave
// runs the skip and the row check redundantly (same LDS state, same result,
// no exchange), wave 0 writes marks/stack/tree, the children's decrements
// are split round-robin over the waves; barrier A separates the visited
// gathers from the marks, barrier B publishes the push.
// ---------------------------------------------------------------------------
#ifdef SDNR_STAMPS
// diagnostic build only: cycles per phase of the counted-pop loop, summed
// over every source by wave 0 of each workgroup (never in the real kernel)
__device__ unsigned long long g_stamp[16];
#define SDNR_STAMP(t) \
    do { __builtin_amdgcn_sched_barrier(0); \
         asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); \
         __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define SDNR_STAMP(t) do { (void)(t); } while (0)
#endif

template <int NW, bool HOPS>
__global__ __launch_bounds__(NW * 64) void dfs_count_kernel(
    int V, const uint16_t *__restrict__ adj, const uint16_t *__restrict__ radj,
    const uint32_t *__restrict__ deg, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ port, const int32_t *__restrict__ src, int nsrc,
    int32_t *__restrict__ out_parent, int32_t *__restrict__ out_port,
    int32_t *__restrict__ out_hops)
{
    constexpr int G = 8;                         // child rows in flight per wave
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 1 + 31) >> 5;            // + sentinel bit V
    const int VWp = (VW + 3) & ~3;
    const int CWp = (V + 1 + 3) & ~3;            // u32 counts of 0..V
    const int SWp = (((V + 1) >> 1) + 3) & ~3;   // u16 stack
    uint32_t *vis = lds;
    uint32_t *cnt = vis + VWp;
    uint16_t *stk = reinterpret_cast<uint16_t *>(cnt + CWp);
    uint32_t *ps = cnt + CWp + SWp;              // parent | row slot << 16
    uint16_t *dep = reinterpret_cast<uint16_t *>(ps + V);
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    unsigned long long t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0, t5 = 0;   // stamps (diag)
#ifdef SDNR_STAMPS
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
#endif

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int i = threadIdx.x; i < VW; i += blockDim.x) vis[i] = 0u;
        for (int i = threadIdx.x; i <= V; i += blockDim.x) cnt[i] = deg[i];
        __syncthreads();
        if (threadIdx.x == 0) {
            vis[s >> 5] |= 1u << (s & 31);
            vis[V >> 5] |= 1u << (V & 31);
            ps[s] = (uint32_t)s;
            if (HOPS) dep[s] = 0;
            stk[0] = (uint16_t)s;
        }
        if (w == 0) {                            // s is visited: its in-neighbours lose one
            const int r = radj[(size_t)s * 64 + lane];
            if (r != V) atomicSub(&cnt[r], 1u);
        }
        __syncthreads();

        int sp = 1;
        int pu = -1, xpre = V;                   // speculatively loaded row of pu
        for (;;) {
            SDNR_STAMP(t0);
            // ---- skip leaf pops, 64 stack slots per step
            uint64_t m = 0;
            int e = V;
            while (sp > 0) {
                const int kk = sp < 64 ? sp : 64;
                const int at = sp - 1 - lane;
                e = stk[at < 0 ? 0 : at];
                e = lane < kk ? e : V;
                m = __ballot(cnt[e] != 0u);
                if (m) break;
                sp -= kk;
            }
            if (!m) break;
            const int first = __ffsll((unsigned long long)m) - 1;
            const int u = read_lane(e, first);
            sp -= first + 1;
            SDNR_STAMP(t1);
            // ---- the non-leaf pop: forward row (usually prefetched: the
            // top of the stack is the previous push's largest child), visited gather
            const int x = (u == pu) ? xpre : (int)adj[(size_t)u * 64 + lane];
            const uint32_t wv = vis[x >> 5];
            const bool fresh = ((wv >> (x & 31)) & 1u) == 0u;
            const uint64_t mm = __ballot(fresh);
            const int rank = lanes_below(mm);
            pu = read_lane(x, highest_lane(mm));     // cnt[u] != 0 -> mm != 0
            xpre = adj[(size_t)pu * 64 + lane];
            int du = 0;
            if (HOPS) du = uniform((int)dep[u]);
            SDNR_STAMP(t2);
            __syncthreads();                     // A: gathers before marks
            SDNR_STAMP(t3);
            if (w == 0 && fresh) {
                atomicOr(&vis[x >> 5], 1u << (x & 31));
                ps[x] = (uint32_t)u | ((uint32_t)lane << 16);
                if (HOPS) dep[x] = (uint16_t)(du + 1);
                stk[sp + rank] = (uint16_t)x;
            }
            // ---- children decrement their in-neighbours' counts; child j
            // (ascending) belongs to wave j % NW, up to G rows in flight
            uint64_t mine = __ballot(fresh && (rank % NW) == w);
            int n = __popcll(mine);
            while (n > 0) {
                int r[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    int v = V;                   // past n: the all-sentinel row
                    if (g < n) {
                        v = read_lane(x, __ffsll((unsigned long long)mine) - 1);
                        mine &= mine - 1;
                    }
                    r[g] = radj[(size_t)v * 64 + lane];
                }
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (g < n && r[g] != V) atomicSub(&cnt[r[g]], 1u);
                n -= G;
            }
            sp += __popcll(mm);
            SDNR_STAMP(t4);
            __syncthreads();                     // B: publish the push
            SDNR_STAMP(t5);
#ifdef SDNR_STAMPS
            acc[0] += t1 - t0;
            acc[1] += t2 - t1;
            acc[2] += t3 - t2;
            acc[3] += t4 - t3;
            acc[4] += t5 - t4;
            acc[5] += 1;
#endif
        }
        __syncthreads();

        for (int v = threadIdx.x; v < V; v += blockDim.x) {
            int p = -1, pt = -1, h = -1;
            if ((vis[v >> 5] >> (v & 31)) & 1u) {
                const uint32_t xx = ps[v];
                p = (int)(xx & 0xFFFFu);
                if (v == s) {
                    h = 0;
                } else {
                    pt = port[row_ptr[p] + (int)(xx >> 16)];
                    h = HOPS ? (int)dep[v] : 0;
                }
            }
            prow[v] = p;
            trow[v] = pt;
            if (HOPS) hrow[v] = h;
        }
        __syncthreads();
    }
#ifdef SDNR_STAMPS
    if (threadIdx.x == 0)
        for (int k = 0; k < 6; ++k) atomicAdd(&g_stamp[k], acc[k]);
#endif
}

// ---------------------------------------------------------------------------
// Lane-packed batched pops for large, low-degree graphs (torus 32^3: 6,
// Jellyfish: 16).  A row needs only LPR >= W lanes, so one wave instruction
// checks R = 64/LPR stack entries (lane l -> slot l/LPR, row position l%LPR)
// and J instructions check K = R*J entries: R times fewer loads, gathers and
// ballots per pop than one-row-per-wavefront.  Same exact semantics as
// dfs_global_batch_kernel (first live entry from the top is processed).
// ---------------------------------------------------------------------------
template <int LPR, int J, bool HOPS, int RING>
__global__ __launch_bounds__(64) void dfs_global_packed_kernel(
    int V, int W, const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops,
    uint2 *__restrict__ spill_all)
{
    constexpr int R = 64 / LPR;
    constexpr int K = R * J;
    static_assert(K <= 64, "one stack slot per lane");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    uint32_t *vis = lds;
    uint2 *ring = reinterpret_cast<uint2 *>(vis + VWp);   // (v, depth)
    uint2 *spill = spill_all + (size_t)blockIdx.x * (size_t)V;
    const int lane = lane_id();
    const int pos = lane % LPR;
    const int sub = lane / LPR;
    const uint64_t lowmask = (LPR == 64) ? ~0ull : ((1ull << LPR) - 1ull);

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = out_port + (size_t)si * V;
        int32_t *hrow = HOPS ? out_hops + (size_t)si * V : nullptr;
        if (s < 0 || s >= V) {
            for (int v = lane; v < V; v += SDNR_WAVE) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
            continue;
        }
        for (int w = lane; w < VW; w += SDNR_WAVE) vis[w] = 0u;
        __syncthreads();
        if (lane == 0) {
            vis[s >> 5] = 1u << (s & 31);
            prow[s] = s;
            trow[s] = -1;
            if (HOPS) hrow[s] = 0;
            ring[0] = make_uint2((uint32_t)s, 0u);
        }
        __syncthreads();

        int lsp = 1, bot = 0, gsp = 0;
        for (;;) {
            if (lsp == 0) {
                if (gsp == 0) break;
                const int n = gsp < RING / 2 ? gsp : RING / 2;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                bot = (bot - n) & (RING - 1);
                for (int i = lane; i < n; i += SDNR_WAVE)
                    ring[(bot + i) & (RING - 1)] = spill[gsp - n + i];
                gsp -= n;
                lsp = n;
            }
            const int kk = lsp < K ? lsp : K;
            uint2 me = ring[(bot + lsp - 1 - lane) & (RING - 1)];
            me.x = lane < kk ? me.x : 0u;
            me.y = lane < kk ? me.y : 0u;
            int x[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int slot = j * R + sub;
                const int u = __shfl((int)me.x, slot);             // slot >= kk: vertex 0
                x[j] = col[u * W + pos];
            }
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int ok = -(int)(((j * R + sub) < kk) & (pos < W));
                x[j] = (x[j] & ok) | ~ok;
            }
            uint64_t m[J];
#pragma unroll
            for (int j = 0; j < J; ++j) {
                const int xi = x[j] & 0x7FFFFFFF;
                const uint32_t w = vis[(xi >> 5) & ((x[j] >> 31) ^ -1)];
                m[j] = __ballot((x[j] >= 0) & (((w >> (xi & 31)) & 1u) == 0u));
            }
            int jstar = J;
#pragma unroll
            for (int j = J - 1; j >= 0; --j)
                if (m[j] != 0) jstar = j;
            if (jstar == J) {
                lsp -= kk;
                continue;
            }
            uint64_t mj = 0;
            int vv = -1;
#pragma unroll
            for (int j = 0; j < J; ++j)
                if (j == jstar) {
                    mj = m[j];
                    vv = x[j];
                }
            const int sstar = (__ffsll((unsigned long long)mj) - 1) / LPR;   // sub-slot
            const int istar = jstar * R + sstar;
            const uint64_t mm = mj & (lowmask << (sstar * LPR));
            const int eu = read_lane((int)me.x, istar);
            const uint32_t ed = (uint32_t)read_lane((int)me.y, istar);
            lsp -= istar + 1;
            const int cnt = __popcll(mm);
            if (lsp + cnt > RING) {
                for (int i = lane; i < RING / 2; i += SDNR_WAVE)
                    spill[gsp + i] = ring[(bot + i) & (RING - 1)];
                gsp += RING / 2;
                bot = (bot + RING / 2) & (RING - 1);
                lsp -= RING / 2;
            }
            if ((mm >> lane) & 1ull) {
                const int rank = lanes_below(mm);
                atomicOr(&vis[vv >> 5], 1u << (vv & 31));
                prow[vv] = eu;
                trow[vv] = port[eu * W + pos];
                if (HOPS) hrow[vv] = (int)ed + 1;
                ring[(bot + lsp + rank) & (RING - 1)] = make_uint2((uint32_t)vv, ed + 1u);
            }
            lsp += cnt;
        }
        __syncthreads();
        for (int v = lane; v < V; v += SDNR_WAVE) {
            if (((vis[v >> 5] >> (v & 31)) & 1u) == 0u) {
                prow[v] = -1;
                trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Search / writer split for large graphs (torus 32^3, Jellyfish 100k).
//
// rocprofv3 on dfs_global_packed_kernel (profiles/r02_torus_dfs_*,
// r02_jf_dfs_*): 84% / 64% of wave cycles waiting.  That kernel stores the
// table entries (parent, port) from the search wave at every push, and a
// wave's vector-memory counter is in order: the next row load's wait also
// waits for every table store issued before it -- a write acknowledgement on
// each step of the serial chain -- and the port lookup sits on the chain
// too.  Here NS search waves of a workgroup (one source each) never store on
// the chain: a push appends (vertex, parent, row slot[, depth]) records to
// the wave's LDS queue and a writer wave drains the NS queues, loads the
// ports and issues the table stores (parent | port << 16 directly when the
// packed layout is asked for).  Rows are read in the narrowest format the
// vertex count allows -- u16 ids below 65,535 vertices; 16 low bits plus a
// per-row mask of the 17th bit below 131,071 (the 100k Jellyfish ELL drops
// from 6.4 MB to 3.6 MB, inside an XCD's 4 MB L2).  The search itself is the
// batched pop of dfs_global_packed_kernel (first live entry from the top).
// ---------------------------------------------------------------------------
constexpr int kRow32 = 0, kRow16 = 1, kRow17 = 2;
// dictionary rows (split kernel, rows of <= 8 slots): row u = u + D[p(u)],
// the pattern ids and D staged in LDS (capi.hip upload_dict)
constexpr int kRowDict = 3;
constexpr int kSplitQ = 64;                    // queued records per search wave
// SDNROUTE_DFS_FLAGS (tuning): search waves at raised issue priority,
// non-temporal table stores, or (diagnostic) no table stores at all / port
// slot instead of the port
// (diagnostic) no port lookups in the writer
constexpr int kFlagPrio = 1, kFlagNT = 2, kFlagNoStore = 4, kFlagNoPort = 8;
// dfs_async_kernel: the worker rows are pre-swizzled count indices (radjw)
constexpr int kFlagPreSwz = 16;
// hop counts written as u16 (0xFFFF unreached) instead of int32: the depth
// plane of the drop-in's table pool (sdnr_dfs_tables_tree)
constexpr int kFlagHops16 = 32;
// split kernel: sources taken from the CU's own contiguous chunk (see
// split_next_source) instead of the static blockIdx-strided order
constexpr int kFlagCuMap = 64;
// async kernel: when every fresh child of a candidate is a leaf, the next
// candidate comes off the stack -- read its window, counts and row before
// the push instead of after it
constexpr int kFlagSpecPop = 128;

// s_getreg encodings: (size - 1) << 11 | offset << 6 | register id
constexpr int kHwIdReg = (31 << 11) | 4;      // HW_REG_HW_ID: cu [11:8], sh [12], se [14:13]
constexpr int kXccIdReg = (15 << 11) | 20;    // HW_REG_XCC_ID: the XCD

// Number of this wave's CU, 0, 1, 2, ... in order of first arrival (wq:
// [nch] chunk cursors | arrivals counter | 1,024-entry CU table, -1 = not
// numbered yet, -2 = being numbered).  Lane 0 works; the result is uniform.
__device__ int split_cu_number(int *wq, int nch, int lane, int *err)
{
    const uint32_t hw = __builtin_amdgcn_s_getreg(kHwIdReg);
    const uint32_t xcc = __builtin_amdgcn_s_getreg(kXccIdReg) & 7u;
    const int key = (int)((((xcc * 4u + ((hw >> 13) & 3u)) * 2u + ((hw >> 12) & 1u)) * 16u) +
                          ((hw >> 8) & 15u));
    int *tab = wq + nch + 1;
    int n = 0;
    if (lane == 0) {
        int v = atomicCAS(&tab[key], -1, -2);
        if (v == -1) {
            n = atomicAdd(&wq[nch], 1);
            __hip_atomic_store(&tab[key], n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            for (unsigned spin = 0; v < 0; ++spin) {
                if (spin > (1u << 22)) {
                    atomicOr(err, 32);
                    v = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                v = __hip_atomic_load(&tab[key], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            }
            n = v;
        }
    }
    return uniform(read_lane(n, 0)) % nch;
}

// The next source of a search wave under kFlagCuMap: the sources are cut
// into nch contiguous chunks, one per CU (by arrival number); a wave takes
// the next source of its chunk, so the ~28 search waves co-resident on a CU
// walk neighbouring sources at the same time (on the torus their traversals
// read neighbouring rows, which the CU's L1 then serves).  A
// wave whose chunk is exhausted looks 64 chunks at a time for one with
// sources left (cursor loads at agent scope) and takes from it.  Returns
// nsrc when no chunk has work.  Bounded: every failed claim exhausts a chunk.
__device__ int split_next_source(int *wq, int nch, int nsrc, int *chunk, int lane)
{
    for (int guard = 0; guard <= 2 * nch + 2; ++guard) {
        const int c = *chunk;
        const int lo = (int)((int64_t)c * nsrc / nch), hi = (int)((int64_t)(c + 1) * nsrc / nch);
        int t = 0;
        if (lane == 0) t = atomicAdd(&wq[c], 1);
        t = uniform(read_lane(t, 0));
        if (lo + t < hi) return lo + t;
        int found = -1;
        for (int base = 0; base < nch && found < 0; base += SDNR_WAVE) {
            const int k = base + lane;
            bool has = false;
            int cc = 0;
            if (k < nch) {
                cc = c + 1 + k < nch ? c + 1 + k : c + 1 + k - nch;
                const int l2 = (int)((int64_t)cc * nsrc / nch);
                const int h2 = (int)((int64_t)(cc + 1) * nsrc / nch);
                has = l2 + __hip_atomic_load(&wq[cc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < h2;
            }
            const uint64_t m = __ballot(has);
            if (m) found = read_lane(cc, __ffsll((unsigned long long)m) - 1);
        }
        if (found < 0) return nsrc;
        *chunk = found;
    }
    return nsrc;
}

// hop count of entry e of an [rows][V] hop table, int32 or u16 (kFlagHops16)
__device__ __forceinline__ void put_hop(int32_t *__restrict__ hops, size_t e, int h, int flags)
{
    if (flags & kFlagHops16) reinterpret_cast<uint16_t *>(hops)[e] = (uint16_t)h;
    else hops[e] = h;
}

template <int FMT>
__device__ __forceinline__ int split_row(const void *__restrict__ rows,
                                         const uint32_t *__restrict__ rhi, int V, int W, int u,
                                         int pos)
{
    const size_t e = (size_t)u * W + pos;
    int x;
    if (FMT == kRow32) {
        x = static_cast<const int32_t *>(rows)[e];
    } else {
        x = (int)static_cast<const uint16_t *>(rows)[e];
        if (FMT == kRow17) x |= (int)((rhi[u] >> pos) & 1u) << 16;
    }
    return x < V ? x : -1;                     // padding (-1, 0xFFFF, 0x1FFFF)
}

// visited-bit word w lives at w ^ ((w >> 5) & 31): words 32 apart (ids 1,024
// apart -- a 32^3 torus's z neighbours) fall in different LDS banks
__device__ __forceinline__ int vsw(int w) { return w ^ ((w >> 5) & 31); }

// stack ring entries: (vertex, depth), or the vertex alone (half the LDS:
// more sources per CU on the 100k Jellyfish, 10 instead of 9; measured 13 %
// slower on the torus, which keeps the pair)
template <bool HOPS> struct SplitRing;
template <> struct SplitRing<true> {
    using T = uint2;
    static __device__ __forceinline__ uint2 get(T e) { return e; }
    static __device__ __forceinline__ T put(uint32_t v, uint32_t d) { return make_uint2(v, d); }
};
template <> struct SplitRing<false> {
    using T = uint32_t;
    static __device__ __forceinline__ uint2 get(T e) { return make_uint2(e, 0u); }
    static __device__ __forceinline__ T put(uint32_t v, uint32_t) { return v; }
};

// dictionary rows without hop counts: one u32 per entry, vertex | pattern
// << 16 (V <= 65535) -- the narrow ring keeps the 32^3 torus at 4 workgroups
// per CU with the dictionary's LDS added
struct SplitRingDict {
    using T = uint32_t;
    static __device__ __forceinline__ uint2 get(T e) { return make_uint2(e & 0xFFFFu, e >> 16); }
    static __device__ __forceinline__ T put(uint32_t v, uint32_t y) { return v | (y << 16); }
};

__host__ __device__ constexpr bool split_wide_ring(int lpr, bool hops, bool dict = false)
{
    return hops || (lpr == 8 && !dict);
}

__host__ __device__ inline size_t split_lds_words(int V, int ring, int ns, bool hops, int lpr,
                                                  bool dict = false)
{
    const size_t VWp = (size_t)((((V + 31) >> 5) + 31) & ~31);
    return (size_t)ns * (VWp + (split_wide_ring(lpr, hops, dict) ? 2 : 1) * (size_t)ring) +
           (size_t)ns * kSplitQ * (hops ? 3 : 2) +
           ((3 * (size_t)ns + 3) & ~(size_t)3);
}

// tree layouts of the split kernel: int32 parent/port tables, parent | port
// << 16 (sdnr_dfs_tables_packed), parent | slot << 26 (sdnr_dfs_tables_slots)
constexpr int kTreeInt32 = 0, kTreePort16 = 1, kTreeSlot = 2;

// The writer wave of the split kernels: drains the NS search waves' record
// queues (vertex | slot << 26, parent[, depth]) into the table rows, loading
// the port of each tree edge off the search chain.  One round takes the
// records of ALL queues at once, packed into the 64 lanes (queue k's pending
// records after queue k-1's), so a round is one LDS read -> port load ->
// store chain however many queues have records (round 5 drained the queues
// one after the other: NS dependent port-load round trips per round, and
// with dictionary rows -- a search twice as fast -- the search waves then
// waited 929 cycles per push for queue room; stamps).
template <int NS, bool HOPS, int PK>
__device__ __forceinline__ void split_writer(int V, int W, const int32_t *__restrict__ ell_port,
                                             const uint2 *qrec, const uint32_t *qdep, int *ctl,
                                             int lane, int32_t *__restrict__ out_parent,
                                             int32_t *__restrict__ out_port,
                                             int32_t *__restrict__ out_hops, int *__restrict__ err,
                                             int flags)
{
    static_assert(NS <= 32, "one lane per queue");
    constexpr unsigned kIdle = 1u << 26;
    constexpr bool PACKED = PK != kTreeInt32;
    int consd = 0;                     // lane k < NS: records of queue k consumed
    unsigned idle = 0;
    for (;;) {
        // records first, then the row: a source's row is announced before
        // its first record, and changes only after the writer consumed all
        // of the previous source's records
        int P = 0, row = -1;
        if (lane < NS) {
            P = __hip_atomic_load(&ctl[lane], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            row = __hip_atomic_load(&ctl[2 * NS + lane], __ATOMIC_ACQUIRE,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const int avail = lane < NS ? P - consd : 0;
        // exclusive prefix of the queues' pending records over lanes 0..NS-1
        int incl = avail;
#pragma unroll
        for (int d = 1; d < NS; d <<= 1) {
            const int t = __shfl_up(incl, d);
            if (lane >= d) incl += t;
        }
        const int excl = incl - avail;
        const int total = read_lane(incl, NS - 1);
        if (total > 0) {
            // lane l serves record l of the packed list: queue k with
            // excl_k <= l < excl_k + avail_k (a uniform scan over the queues)
            int k = -1, idx = 0, crow = 0, cbase = 0;
#pragma unroll
            for (int q = 0; q < NS; ++q) {
                const int e = read_lane(excl, q), a = read_lane(avail, q);
                if (lane >= e && lane < e + a) {
                    k = q;
                    idx = lane - e;
                    crow = read_lane(row, q);
                    cbase = read_lane(consd, q);
                }
            }
            if (k >= 0) {
                const int at = k * kSplitQ + ((cbase + idx) & (kSplitQ - 1));
                const uint2 r = qrec[at];
                const int v = (int)(r.x & 0x3FFFFFFu), slot = (int)(r.x >> 26);
                const int par = (int)r.y;
                const size_t e = (size_t)crow * V + v;
                if (PK == kTreeSlot) {         // no port lookup: the slot names it
                    const int32_t tv = (int32_t)((uint32_t)par | ((uint32_t)slot << 26));
                    if (flags & kFlagNT) __builtin_nontemporal_store(tv, &out_parent[e]);
                    else if (!(flags & kFlagNoStore)) out_parent[e] = tv;
                    if (HOPS && !(flags & kFlagNoStore)) put_hop(out_hops, e, (int)qdep[at], flags);
                } else {
                    const int pt = (flags & kFlagNoPort) ? slot : ell_port[(size_t)par * W + slot];
                    if (flags & kFlagNoStore) {
                        // diagnostic: records consumed, no table stores
                    } else if (flags & kFlagNT) {
                        if (PACKED) {
                            __builtin_nontemporal_store(
                                (int32_t)(((uint32_t)par & 0xFFFFu) | ((uint32_t)pt << 16)),
                                &out_parent[e]);
                        } else {
                            __builtin_nontemporal_store(par, &out_parent[e]);
                            __builtin_nontemporal_store(pt, &out_port[e]);
                        }
                        if (HOPS) {
                            if (flags & kFlagHops16)
                                __builtin_nontemporal_store(
                                    (uint16_t)qdep[at], reinterpret_cast<uint16_t *>(out_hops) + e);
                            else
                                __builtin_nontemporal_store((int)qdep[at], &out_hops[e]);
                        }
                    } else {
                        if (PACKED) {
                            out_parent[e] = (int32_t)(((uint32_t)par & 0xFFFFu) |
                                                      ((uint32_t)pt << 16));
                        } else {
                            out_parent[e] = par;
                            out_port[e] = pt;
                        }
                        if (HOPS) put_hop(out_hops, e, (int)qdep[at], flags);
                    }
                }
            }
            // queue k's share of this round (the list is cut at 64 lanes)
            const int took = lane < NS ? max(0, min(avail, SDNR_WAVE - excl)) : 0;
            consd += took;
            // the record reads above are done (LDS ops in order)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (took > 0) __hip_atomic_store(&ctl[NS + lane], consd, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_WORKGROUP);
            idle = 0;
            continue;
        }
        // nothing pending: done when every queue's wave has finished (row
        // -1) and published nothing meanwhile
        bool done = true;
        if (lane < NS)
            done = row == -1 && __hip_atomic_load(&ctl[lane], __ATOMIC_ACQUIRE,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP) == consd;
        if (__ballot(!done) == 0ull) break;
        if (++idle > kIdle) {
            if (lane == 0) atomicOr(err, 16);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

template <int LPR, int J, bool HOPS, int RING, int NS, int FMT, int PK>
__global__ __launch_bounds__((NS + 1) * 64) void dfs_split_kernel(
    int V, int W, const void *__restrict__ rows, const uint32_t *__restrict__ rhi,
    const int32_t *__restrict__ ell_port, const int32_t *__restrict__ src, int nsrc,
    int32_t *__restrict__ out_parent, int32_t *__restrict__ out_port,
    int32_t *__restrict__ out_hops, uint2 *__restrict__ spill_all, int *__restrict__ err,
    int flags, int *__restrict__ wq, int nch, const uint32_t *__restrict__ dict_bp,
    const uint32_t *__restrict__ dict_bt, const int32_t *__restrict__ dict_off, int dict_bpw,
    int dict_NB, int dict_P)
{
    // kRowDict: a stack entry carries its vertex's pattern id (ring .y =
    // pattern | depth << 8), a window's row is u + D[pattern][slot] from LDS
    // and the new children's pattern ids (two dictionary levels, capi.hip
    // upload_dict) are read beside their visited words, so the chain touches
    // no global memory (the torus's window was one dependent
    // L2 row read at the loaded L2 latency)
    constexpr bool DICT = FMT == kRowDict;
    static_assert(!DICT || LPR == 8, "dictionary rows: 8 lanes per row");
    constexpr int R = 64 / LPR;
    constexpr int K = R * J;
    constexpr unsigned kSpin = 1u << 22;
    constexpr bool PACKED = PK != kTreeInt32;
    static_assert(K <= 64, "one stack slot per lane");
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 31) >> 5;
    const int VWp = (VW + 31) & ~31;          // whole 32-word blocks (swizzled)
    constexpr bool WR = split_wide_ring(LPR, HOPS, DICT);
    // entries carry (vertex, y): y = depth, or with dictionary rows the
    // pattern id (| depth << 8 with hop counts: the wide ring)
    constexpr bool YR = WR || DICT;
    using RE = typename std::conditional<DICT && !WR, SplitRingDict, SplitRing<WR>>::type;
    using RT = typename RE::T;
    const int per = VWp + (WR ? 2 : 1) * RING;   // words per search wave: vis | stack ring
    uint2 *qrec = reinterpret_cast<uint2 *>(lds + NS * per);
    uint32_t *qdep = reinterpret_cast<uint32_t *>(qrec + NS * kSplitQ);
    // ctl[k] records published by search wave k, ctl[NS + k] records the
    // writer consumed, ctl[2NS + k] table row of wave k's source (-2 none
    // yet, -1 no more)
    int *ctl = reinterpret_cast<int *>(qdep + (HOPS ? NS * kSplitQ : 0));
    // dictionary: block ids (4 per word), block tuples (8 words each), then
    // D (8 offsets per pattern id)
    uint32_t *lbp = reinterpret_cast<uint32_t *>(ctl) + ((3 * NS + 3) & ~3);
    uint32_t *lbt = lbp + (DICT ? dict_bpw : 0);
    const int32_t *loff = reinterpret_cast<const int32_t *>(lbt + (DICT ? 8 * dict_NB : 0));
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    if (threadIdx.x < 3 * NS) ctl[threadIdx.x] = (int)threadIdx.x >= 2 * NS ? -2 : 0;
    if (DICT) {
        for (int i = threadIdx.x; i < dict_bpw; i += blockDim.x) lbp[i] = dict_bp[i];
        for (int i = threadIdx.x; i < 8 * dict_NB; i += blockDim.x) lbt[i] = dict_bt[i];
        int32_t *lo = reinterpret_cast<int32_t *>(lbt + 8 * dict_NB);
        for (int i = threadIdx.x; i < dict_P * 8; i += blockDim.x) lo[i] = dict_off[i];
    }
    __syncthreads();
    // pattern id of v in [0, V): block id, then the block tuple's byte
    auto blk_of = [&](int v) -> uint32_t { return (lbp[v >> 7] >> (8 * ((v >> 5) & 3))) & 0xFFu; };
    auto pat_in = [&](uint32_t b, int v) -> uint32_t {
        return (lbt[b * 8 + ((v & 31) >> 2)] >> (8 * (v & 3))) & 0xFFu;
    };
    auto pat_of = [&](int v) -> uint32_t { return pat_in(blk_of(v), v); };

    if (w < NS) {
        // ------------------------------------------------------ a search wave
        if (flags & kFlagPrio) __builtin_amdgcn_s_setprio(3);
        const int pos = lane % LPR;
        const int sub = lane / LPR;
        const uint64_t lowmask = (LPR == 64) ? ~0ull : ((1ull << LPR) - 1ull);
        uint32_t *vis = lds + w * per;
        RT *ring = reinterpret_cast<RT *>(vis + VWp);   // (v[, depth])
        uint2 *q = qrec + w * kSplitQ;
        uint32_t *qd = qdep + w * kSplitQ;
        const int slot_id = blockIdx.x * NS + w;
        RT *spill = reinterpret_cast<RT *>(spill_all) + (size_t)slot_id * (size_t)V;
        int pub = 0, cons = 0;
#ifdef SDNR_STAMPS
        unsigned long long z_t0, z_t1, z_a, z_b, z_c, z_rd = 0, z_qw = 0, z_push = 0, z_it = 0,
                                                   z_nl = 0, z_sp = 0, z_rf = 0, z_rfc = 0;
        SDNR_STAMP(z_t0);
#endif
        // source order: blockIdx-strided, or (kFlagCuMap) the CU's own chunk
        const bool cumap = (flags & kFlagCuMap) != 0;
        int chunk = cumap ? split_cu_number(wq, nch, lane, err) : 0;
        auto next_source = [&](int prev) -> int {
            if (!cumap) return prev < 0 ? slot_id : prev + (int)gridDim.x * NS;
            return split_next_source(wq, nch, nsrc, &chunk, lane);
        };
        for (int si = next_source(-1); si < nsrc; si = next_source(si)) {
            const int s = uniform(src[si]);
            int32_t *prow = out_parent + (size_t)si * V;
            int32_t *trow = PACKED ? nullptr : out_port + (size_t)si * V;
            const size_t hb = (size_t)si * V;        // row of the hop table
            if (s < 0 || s >= V) {                 // unknown source: empty row
                for (int v = lane; v < V; v += SDNR_WAVE) {
                    prow[v] = -1;                  // packed: 0xFFFFFFFF
                    if (!PACKED) trow[v] = -1;
                    if (HOPS) put_hop(out_hops, hb + v, -1, flags);
                }
                continue;
            }
            for (int i = lane; i < VWp; i += SDNR_WAVE) vis[i] = 0u;
            if (lane == 0) {                       // the wave's LDS ops stay in order
                vis[vsw(s >> 5)] = 1u << (s & 31);
                prow[s] = PK == kTreePort16 ? (int32_t)((uint32_t)s | 0xFFFF0000u)
                        : PK == kTreeSlot  ? (int32_t)((uint32_t)s | (63u << 26)) : s;
                if (!PACKED) trow[s] = -1;
                if (HOPS) put_hop(out_hops, hb + s, 0, flags);
                ring[0] = RE::put((uint32_t)s, DICT ? pat_of(s) : 0u);
                __hip_atomic_store(&ctl[2 * NS + w], si, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            int lsp = 1, bot = 0, gsp = 0;
            int pubd = pub;                        // records announced to the writer
            for (;;) {
                if (lsp == 0) {
                    if (gsp == 0) break;
                    const int n = gsp < RING / 2 ? gsp : RING / 2;
                    // own spill stores: this wave wrote them through this
                    // CU's L1, so a workgroup-scope acquire (wait for them;
                    // no L1 invalidate) suffices -- the agent-scope one cost
                    // ~9.7 k cycles per refill under the writers' store
                    // traffic (stamps)
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    bot = (bot - n) & (RING - 1);
#ifdef SDNR_STAMPS
                    SDNR_STAMP(z_a);
#endif
                    for (int i = lane; i < n; i += SDNR_WAVE)
                        ring[(bot + i) & (RING - 1)] = spill[gsp - n + i];
                    gsp -= n;
                    lsp = n;
#ifdef SDNR_STAMPS
                    SDNR_STAMP(z_b);
                    z_rf++;
                    z_rfc += z_b - z_a;
#endif
                }
#ifdef SDNR_STAMPS
                SDNR_STAMP(z_a);
                z_it++;
#endif
                const int kk = lsp < K ? lsp : K;
                // every lane reads its slot's stack entry itself (no
                // cross-lane shuffle on the chain); slots past the stack
                // become vertex 0 and are masked below
                // (one slot per lane group: J == 1; with several groups per
                // lane, one read per lane + shuffles moves fewer LDS bytes)
                uint2 ue[J];
                int x[J];
                if (J == 1) {
                    ue[0] = RE::get(ring[(bot + lsp - 1 - sub) & (RING - 1)]);
                    ue[0].x = sub < kk ? ue[0].x : 0u;
                    if (DICT) ue[0].y = sub < kk ? ue[0].y : 0u;
                } else {
                    uint2 me = RE::get(ring[(bot + lsp - 1 - lane) & (RING - 1)]);
                    me.x = lane < kk ? me.x : 0u;
                    if (DICT) me.y = lane < kk ? me.y : 0u;
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                        ue[j].x = (uint32_t)__shfl((int)me.x, j * R + sub);
                        ue[j].y = YR ? (uint32_t)__shfl((int)me.y, j * R + sub) : 0u;
                    }
                }
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    if constexpr (DICT) {
                        const int xj = (int)ue[j].x + loff[(int)(ue[j].y & 0xFFu) * 8 + pos];
                        x[j] = xj < V ? xj : -1;                 // padding: u + kDictPad
                    } else {
                        x[j] = split_row<FMT>(rows, rhi, V, W, (int)ue[j].x, pos);
                    }
                }
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int ok = -(int)(((j * R + sub) < kk) & (pos < W));
                    x[j] = (x[j] & ok) | ~ok;
                }
                uint64_t m[J];
                uint32_t pw[J];                    // DICT: the pattern id of x[j]
#pragma unroll
                for (int j = 0; j < J; ++j) {
                    const int xi = x[j] & 0x7FFFFFFF;
                    const int xs = xi & ((x[j] >> 31) ^ -1);    // padding -> vertex 0
                    const uint32_t wv = vis[vsw(xs >> 5)];
                    // the block id beside the visited word, its tuple byte
                    // right behind (both off the ballot's path: only a push
                    // uses them)
                    if (DICT) pw[j] = pat_in(blk_of(xs), xs);
                    m[j] = __ballot((x[j] >= 0) & (((wv >> (xi & 31)) & 1u) == 0u));
                }
                // announce the previous push's records now: the LDS reads of
                // this batch have already waited for those writes, so the
                // LDS-only release costs no extra round trip
                if (pub != pubd) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    if (lane == 0) __hip_atomic_store(&ctl[w], pub, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    pubd = pub;
                }
                int jstar = J;
#pragma unroll
                for (int j = J - 1; j >= 0; --j)
                    if (m[j] != 0) jstar = j;
#ifdef SDNR_STAMPS
                SDNR_STAMP(z_b);
                z_rd += z_b - z_a;
#endif
                if (jstar == J) {
                    lsp -= kk;
                    continue;
                }
                uint64_t mj = 0;
                int vv = -1;
                uint32_t pv = 0;
                uint2 uj = make_uint2(0u, 0u);
#pragma unroll
                for (int j = 0; j < J; ++j)
                    if (j == jstar) {
                        mj = m[j];
                        vv = x[j];
                        if (DICT) pv = pw[j];
                        uj = ue[j];
                    }
                const int sstar = (__ffsll((unsigned long long)mj) - 1) / LPR;
                const int istar = jstar * R + sstar;
                const uint64_t mm = mj & (lowmask << (sstar * LPR));
                const int eu = read_lane((int)uj.x, sstar * LPR);
                const uint32_t ey = YR ? (uint32_t)read_lane((int)uj.y, sstar * LPR) : 0u;
                const uint32_t ed = DICT ? ey >> 8 : ey;   // the popped entry's depth
                lsp -= istar + 1;
                const int cnt = __popcll(mm);
                // room in the record queue (the writer publishes its progress)
                if (pub + cnt - cons > kSplitQ) {
                    if (pub != pubd) {             // the writer must see what is queued
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                        if (lane == 0) __hip_atomic_store(&ctl[w], pub, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                        pubd = pub;
                    }
                    for (unsigned spin = 0; pub + cnt - cons > kSplitQ; ++spin) {
                        cons = __hip_atomic_load(&ctl[NS + w], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (pub + cnt - cons <= kSplitQ) break;
                        if (spin > kSpin) {
                            if (lane == 0) atomicOr(err, 4);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
#ifdef SDNR_STAMPS
                SDNR_STAMP(z_c);
                z_qw += z_c - z_b;
                z_nl++;
                if (lsp + cnt > RING) z_sp++;
#endif
                if (lsp + cnt > RING) {            // spill the oldest half
                    for (int i = lane; i < RING / 2; i += SDNR_WAVE)
                        spill[gsp + i] = ring[(bot + i) & (RING - 1)];
                    gsp += RING / 2;
                    bot = (bot + RING / 2) & (RING - 1);
                    lsp -= RING / 2;
                }
                if ((mm >> lane) & 1ull) {
                    const int rank = lanes_below(mm);
                    atomicOr(&vis[vsw(vv >> 5)], 1u << (vv & 31));
                    q[(pub + rank) & (kSplitQ - 1)] =
                        make_uint2((uint32_t)vv | ((uint32_t)pos << 26), (uint32_t)eu);
                    if (HOPS) qd[(pub + rank) & (kSplitQ - 1)] = ed + 1u;
                    ring[(bot + lsp + rank) & (RING - 1)] =
                        RE::put((uint32_t)vv, DICT ? pv | ((ed + 1u) << 8) : ed + 1u);
                }
                lsp += cnt;
                pub += cnt;
#ifdef SDNR_STAMPS
                SDNR_STAMP(z_a);
                z_push += z_a - z_c;
#endif
            }
            if (pub != pubd) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_store(&ctl[w], pub, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            // this source's records drained before its row changes, then the
            // entries of unreached vertices
            for (unsigned spin = 0; cons != pub; ++spin) {
                cons = __hip_atomic_load(&ctl[NS + w], __ATOMIC_ACQUIRE,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                if (cons == pub) break;
                if (spin > kSpin) {
                    if (lane == 0) atomicOr(err, 8);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            for (int v = lane; v < V; v += SDNR_WAVE) {
                if (((vis[vsw(v >> 5)] >> (v & 31)) & 1u) == 0u) {
                    prow[v] = -1;
                    if (!PACKED) trow[v] = -1;
                    if (HOPS) put_hop(out_hops, hb + v, -1, flags);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) __hip_atomic_store(&ctl[2 * NS + w], -1, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef SDNR_STAMPS
        SDNR_STAMP(z_t1);
        if (lane == 0) {
            atomicAdd(&g_stamp[0], z_t1 - z_t0);   // search wave lifetime
            atomicAdd(&g_stamp[1], z_rd);          // stack + row + visited per iteration
            atomicAdd(&g_stamp[2], z_it);          // iterations
            atomicAdd(&g_stamp[3], z_nl);          // non-leaf pops
            atomicAdd(&g_stamp[4], z_qw);          // queue-room waits
            atomicAdd(&g_stamp[5], z_push);        // push (+ spill)
            atomicAdd(&g_stamp[6], z_sp);          // spills
            atomicAdd(&g_stamp[7], z_rf);          // refills
            atomicAdd(&g_stamp[8], z_rfc);         // refill cycles
        }
#endif
    } else {
        split_writer<NS, HOPS, PK>(V, W, ell_port, qrec, qdep, ctl, lane, out_parent, out_port,
                                   out_hops, err, flags);
    }
}

// ---------------------------------------------------------------------------
// Asynchronous counted pops (the k=48 headline kernel).
//
// Same counts as dfs_count_kernel, one observation further: a count may be
// STALE HIGH without breaking exactness.  If the skip stops at an entry whose
// count still includes a neighbour visited a moment ago, the row check finds
// no fresh child and the entry is popped as the leaf pop it is.  A count is
// never low (a decrement is published only after its mark).  So the
// decrements need not finish before the next pop: wave 0 runs the search
// chain alone -- skip, row, visited gather, push -- with no barrier, and
// publishes each push's children into an LDS ring; waves 1..NW-1 drain the
// ring (child j belongs to worker 1 + j % (NW-1)), load the children's
// in-rows and ds_sub the counts.  Hand-off inside the workgroup: ring writes,
// release fence, relaxed store of the published count; workers acquire-load
// it.  Back-pressure keeps the ring from overrunning the slowest worker.
// Every spin is bounded; the bound only trips on a bug, and then sets the
// error word instead of hanging the GPU.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int swz(int x) { return lds_swz(x); }   // common.h

// PAIR: how a worker loads the pre-swizzled in-rows -- 0: one u16 row (64
// lanes) per child; 1: rows of <= 32 entries repeated in lanes 32..63, one
// load for two children; 2: the 64-entry rows read as 32 u32 words, lanes
// 0..31 child 2g and 32..63 child 2g + 1, two ds_sub per lane -- half the
// load instructions and half the returned dwords of PAIR 0 (the CU's
// vector-memory data return is 71 % busy at the k=48 headline's load)
// SPEC: the speculative stack pop (kFlagSpecPop) compiled in.  A separate
// instantiation, not only a runtime flag: its code in the hot loop costs the
// low-load (<= 2 sources per CU) kernel ~8 us at k=48 even when the flag is
// off (144 sources 44.3 vs 52.0 us, same box, gpurun_out/r5_abr4), while at
// the headline's load the pop itself gains
template <int NW, bool HOPS, bool PACKED, bool C16, int PAIR, bool SPEC = false>
__global__ __launch_bounds__(NW * 64, C16 ? 7 : 1) void dfs_async_kernel(
    int V, const uint16_t *__restrict__ adj, const uint16_t *__restrict__ radj,
    const uint32_t *__restrict__ deg, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ port, int W, const int32_t *__restrict__ ell_port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops, int *__restrict__ err,
    int flags)
{
    static_assert(NW >= 2, "wave 0 searches, the others decrement");
    constexpr int U = 4;                         // init / flush vertices per thread per step
    constexpr int S = NW - 1;                    // workers
    constexpr int RING = 512;                    // children in flight (u16)
#ifndef SDNR_ASYNC_G
#define SDNR_ASYNC_G 8
#endif
// table flush: vertices per thread per pass (one pass for k=48's 2,880
// switches at 8 waves: 1 / 144 sources 45.4 / 47.1 -> 43.7 / 45.1 us; 12
// gained 1 % more there but cost the dragonfly's compact kernel registers:
// 2,064 sources 169 -> 217 us; profiles/r06_flush_ab)
#ifndef SDNR_ASYNC_FLUSH_U
#define SDNR_ASYNC_FLUSH_U 6
#endif
#ifndef SDNR_ASYNC_G_DW
#define SDNR_ASYNC_G_DW 16
#endif
#ifndef SDNR_ASYNC_G_P1
#define SDNR_ASYNC_G_P1 8
#endif
#ifndef SDNR_ASYNC_G_U16
#define SDNR_ASYNC_G_U16 48
#endif
    // children per worker step: 16 (8 above 4 waves), and 16 with the
    // dword-paired rows of the 5-worker regime (8 loads): k=48 144 sources
    // 54.9 -> 48.8 us, one source 53.3 -> 47.2 us (fresher counts)
    // Round 5: 32 with the plain u16 in-rows at <= 4 waves (the k=48
    // headline; library A/B, one box, gpurun_out/r5_abg3: 1,152 sources
    // 82.5 / 80.6 / 79.4 / 78.8 / 85.1 us at 16 / 24 / 32 / 48 / 64, 576
    // sources 67.4 -> 64.9 at 32), while the dragonfly's paired rows want
    // narrower steps: 8 (2,064 sources 178.9 / 171.8 / 168.5 us at 16 / 12 /
    // 8, 214.1 at 32; gpurun_out/r5_abg5).  48 for the plain rows after a
    // second A/B on the final library (profiles/r05_async_g48_ab.log): 1,152
    // sources 79.5 -> 78.2 us, every smaller share within 0.3 us
    constexpr int G = NW <= 4 ? (PAIR == 0 ? SDNR_ASYNC_G_U16 : SDNR_ASYNC_G)
                              : (PAIR == 2 ? SDNR_ASYNC_G_DW : (PAIR == 1 ? SDNR_ASYNC_G_P1 : 8));
    constexpr unsigned kSpin = 1u << 22;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int VW = (V + 1 + 31) >> 5;
    const int VWp = (VW + 3) & ~3;
    // C16 (compact): u16 counts in pairs, u16 parents + u8 slots -- 2,064
    // dragonfly sources fit 9 per CU (all resident) instead of 6
    // count words, swizzled within 32-word groups, then 64 dummy words (the
    // pre-swizzled in-rows' padding targets, one per lane), whole 256-blocks
    const int CWp = ((((C16 ? (V + 2) >> 1 : V + 1) + 31) & ~31) + 64 + 255) & ~255;
    const int SWp = (((V + 1) >> 1) + 3) & ~3;
    const int PW = (V + 255) & ~255;                         // parent entries
    const int PWp = C16 ? PW / 2 + PW / 4 : PW;
    uint32_t *vis = lds;
    uint32_t *cnt = vis + VWp;                   // cnt[swz(v)] (C16: swz(v >> 1), halves)
    uint16_t *stk = reinterpret_cast<uint16_t *>(cnt + CWp);
    uint32_t *ps = cnt + CWp + SWp;              // ps[swz(v)] = parent | slot << 16
    uint16_t *ps16 = reinterpret_cast<uint16_t *>(ps);        // C16: ps16[swz(v)] = parent
    uint8_t *sl8 = reinterpret_cast<uint8_t *>(ps16 + PW);    //      sl8[swz(v)] = slot
    uint16_t *dep = reinterpret_cast<uint16_t *>(ps + PWp);   // dep[v]
    auto cnt_of = [&](int v) -> uint32_t {
        if constexpr (C16) {
            const uint32_t x = __hip_atomic_load(&cnt[swz(v >> 1)], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            return (x >> ((v & 1) << 4)) & 0xFFFFu;
        } else {
            return __hip_atomic_load(&cnt[swz(v)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    };
    uint16_t *ring = reinterpret_cast<uint16_t *>(ps + PWp + (HOPS ? ((V + 1) >> 1) : 0));
    int *ctl = reinterpret_cast<int *>(ring + RING);   // [0] published [1] done [2+k] consumed
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
#ifdef SDNR_STAMPS
    unsigned long long kstart;
    SDNR_STAMP(kstart);
#endif

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = PACKED ? nullptr : out_port + (size_t)si * V;
        const size_t hb = (size_t)si * V;        // row of the hop table
        if (s < 0 || s >= V) {
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                prow[v] = -1;                    // packed: 0xFFFFFFFF
                if (!PACKED) trow[v] = -1;
                if (HOPS) put_hop(out_hops, hb + v, -1, flags);
            }
            continue;
        }
#ifdef SDNR_STAMPS
        unsigned long long ph0, ph1, ph2, ph3;
        SDNR_STAMP(ph0);
#endif
        for (int i = threadIdx.x; i < VW; i += blockDim.x) vis[i] = 0u;
        // counts start at the out-degrees: U independent loads per thread in
        // flight before the LDS stores
        if constexpr (C16) {                     // deg is padded to an even length
            const int nw = (V + 2) >> 1;
            for (int i0 = threadIdx.x; i0 < nw; i0 += U * blockDim.x) {
                uint2 dg[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int i = i0 + k * (int)blockDim.x;
                    dg[k] = reinterpret_cast<const uint2 *>(deg)[i < nw ? i : 0];
                }
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int i = i0 + k * (int)blockDim.x;
                    if (i < nw) cnt[swz(i)] = dg[k].x | (dg[k].y << 16);
                }
            }
        } else {
            for (int i0 = threadIdx.x; i0 <= V; i0 += U * blockDim.x) {
                uint32_t dg[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int i = i0 + k * (int)blockDim.x;
                    dg[k] = deg[i <= V ? i : V];
                }
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int i = i0 + k * (int)blockDim.x;
                    if (i <= V) cnt[swz(i)] = dg[k];
                }
            }
        }
        if (threadIdx.x < 2 + S) ctl[threadIdx.x] = 0;
        __syncthreads();
#ifdef SDNR_STAMPS
        SDNR_STAMP(ph1);
#endif

        if (w == 0) {
            // ------------------------------------------------ the search
            if (flags & kFlagPrio) __builtin_amdgcn_s_setprio(3);
            if (lane == 0) {
                vis[s >> 5] |= 1u << (s & 31);
                vis[V >> 5] |= 1u << (V & 31);
                if (C16) ps16[swz(s)] = (uint16_t)s;
                else ps[swz(s)] = (uint32_t)s;
                if (HOPS) dep[s] = 0;
                stk[0] = (uint16_t)s;
                ring[0] = (uint16_t)s;           // s's in-neighbours lose one
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            int pub = 1, pubd = 1, sp = 1, lo = 0;       // published / announced
            constexpr int NPF = 1;        // rows of the NPF largest children in flight
            // the prefetched rows stay u16 across the loop back-edge: an int
            // copy there needs the load's data (s_waitcnt vmcnt(0) at the end
            // of every push), a u16 one is widened where the row is used
            int pu[NPF];
            uint16_t xp[NPF];
#pragma unroll
            for (int k = 0; k < NPF; ++k) {
                pu[k] = -1;
                xp[k] = (uint16_t)V;
            }
#ifdef SDNR_STAMPS
            unsigned long long st_t0, st_t1, st_row = 0, st_cand = 0, st_false = 0, st_bp = 0,
                                               st_miss = 0, st_skip = 0, st_tc = 0, st_skipc = 0,
                                               st_pushc = 0;
            SDNR_STAMP(st_t0);
            st_tc = st_t0;
#endif
            // one candidate: its row, fresh children, push; returns the
            // next candidate when it is one of the new children (the
            // common case: a tight inner loop), else -1 (pop from the stack)
            auto explore = [&](const int u) -> int {
#ifdef SDNR_STAMPS
                unsigned long long ta, tb;
                SDNR_STAMP(ta);
                st_skipc += ta - st_tc;
                {
                    bool hit = false;
#pragma unroll
                    for (int k = 0; k < NPF; ++k) hit |= u == pu[k];
                    if (!hit) st_miss++;
                }
#endif
                int x = -1;
#pragma unroll
                for (int k = 0; k < NPF; ++k)
                    if (x < 0 && u == pu[k]) x = (int)xp[k];
                if (x < 0) x = (int)adj[(size_t)u * 64 + lane];
                const uint32_t wv = vis[x >> 5];
                // the row's counts ride along with its visited words (one
                // wait for both; read in every lane: x <= V is always a count
                // word); a count read earlier is at most staler, i.e. high,
                // which the row check absorbs -- so a plain load will do (as
                // an atomic load it waited for this wave's earlier LDS writes)
                uint32_t cc;
                if constexpr (C16)
                    cc = (cnt[swz(x >> 1)] >> ((x & 1) << 4)) & 0xFFFFu;
                else
                    cc = cnt[swz(x)];
                const bool fresh = ((wv >> (x & 31)) & 1u) == 0u;
                const uint64_t mm = __ballot(fresh);
                // balloted here, ahead of the leaf-pop exit, so the count
                // read stays beside the visited read (used after the exit, the
                // compiler sank it there: a second round trip)
                const uint64_t ccm = __ballot(cc != 0u);
#ifdef SDNR_STAMPS
                SDNR_STAMP(tb);
                st_row += tb - ta;
                st_cand++;
                if (mm == 0) st_false++;
#endif
#ifdef SDNR_STAMPS
                if (mm == 0) st_tc = tb;
#endif
                if (mm == 0) return -1;          // stale count: a leaf pop after all
                const int c = __popcll(mm);
                const int rank = lanes_below(mm);
                // the next candidate is known here, the counts having come
                // with the visited words: the highest fresh child with a count
                // (the children above it are leaves -- counts are never low --
                // and are popped).  Its row is the one prefetched, and its
                // stack position is a scalar popcount: one ballot -> readlane
                // chain per candidate instead of two
                const uint64_t mc = ccm & mm;
                int nu = -1, below = 0;
                if (mc) {
                    const int hl = highest_lane(mc);
                    nu = read_lane(x, hl);
                    below = __popcll(mm & ((1ull << hl) - 1ull));   // fresh children under it
                    pu[0] = nu;
                    xp[0] = adj[(size_t)nu * 64 + lane];
                } else if (SPEC && (flags & kFlagSpecPop) && sp > 0) {
                    // every fresh child is a leaf (its count is 0 and counts
                    // never rise), so none stays on the stack and the next
                    // candidate is the first entry with a count from the top
                    // of the stack as it is NOW: the push below writes only
                    // above sp and changes no count.  Its window, counts and
                    // row are read here, so the row load runs beside the
                    // push (a count read early is at most staler -- high --
                    // which the row check absorbs).  A window without a
                    // candidate is skipped as the outer loop would.
                    const int kk = sp < 64 ? sp : 64;
                    const int at = sp - 1 - lane;
                    int e2 = stk[at < 0 ? 0 : at];
                    e2 = lane < kk ? e2 : V;
                    uint32_t c2;
                    if constexpr (C16)
                        c2 = (cnt[swz(e2 >> 1)] >> ((e2 & 1) << 4)) & 0xFFFFu;
                    else
                        c2 = cnt[swz(e2)];
                    const uint64_t m2 = __ballot(c2 != 0u);
                    if (m2) {
                        const int f2 = __ffsll((unsigned long long)m2) - 1;
                        nu = read_lane(e2, f2);
                        sp -= f2 + 1;
                        pu[0] = nu;
                        xp[0] = adj[(size_t)nu * 64 + lane];
                    } else {
                        sp -= kk;
                        pu[0] = -1;
                    }
                } else {
                    pu[0] = -1;                  // the next candidate comes off the stack
                }
                int du = 0;
                if (HOPS) du = uniform((int)dep[u]);
                // back-pressure: ring slots below every worker's progress are
                // free; the bound only needs refreshing when it would block
                for (unsigned spin = 0; pub + c - lo > RING; ++spin) {
                    lo = 0x7FFFFFFF;
#pragma unroll
                    for (int q = 0; q < S; ++q)
                        lo = min(lo, __hip_atomic_load(&ctl[2 + q], __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP));
                    lo = uniform(lo);            // scalar: the bound test stays off the VALU
                    if (pub + c - lo <= RING) break;
                    if (spin > kSpin) {
                        if (lane == 0) atomicOr(err, 1);
                        break;
                    }
#ifdef SDNR_STAMPS
                    st_bp++;
#endif
                    __builtin_amdgcn_s_sleep(1);
                }
                if (fresh) {
                    atomicOr(&vis[x >> 5], 1u << (x & 31));
                    if (C16) {
                        ps16[swz(x)] = (uint16_t)u;
                        sl8[swz(x)] = (uint8_t)lane;
                    } else {
                        ps[swz(x)] = (uint32_t)u | ((uint32_t)lane << 16);
                    }
                    if (HOPS) dep[x] = (uint16_t)(du + 1);
                    stk[sp + rank] = (uint16_t)x;
                    ring[(pub + rank) & (RING - 1)] = (uint16_t)x;
                }
                pub += c;
                // announce the children without waiting for the writes: one
                // wave's LDS ops execute in issue order, so a worker that
                // reads the new count reads the ring after its entries were
                // written; the empty asm keeps the compiler from moving the
                // store above them
                __asm__ volatile("" ::: "memory");
                if (lane == 0) __hip_atomic_store(&ctl[0], pub, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
                pubd = pub;
                sp += below;
#ifdef SDNR_STAMPS
                SDNR_STAMP(st_tc);
                st_pushc += st_tc - tb;
#endif
                return nu;
            };
            for (;;) {
                uint64_t m = 0;
                int e = V;
                while (sp > 0) {
#ifdef SDNR_STAMPS
                    st_skip++;
#endif
                    const int kk = sp < 64 ? sp : 64;
                    const int at = sp - 1 - lane;
                    e = stk[at < 0 ? 0 : at];
                    e = lane < kk ? e : V;
                    const uint32_t c = cnt_of(e);
                    m = __ballot(c != 0u);
                    if (m) break;
                    sp -= kk;
                }
                // children of the last push not yet announced (the push
                // block announces its own; kept for the first pops)
                if (pub != pubd) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    if (lane == 0) __hip_atomic_store(&ctl[0], pub, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    pubd = pub;
                }
                if (!m) break;
                const int first = __ffsll((unsigned long long)m) - 1;
                sp -= first + 1;
                for (int u = read_lane(e, first); u >= 0;) u = explore(u);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (flags & kFlagPrio) __builtin_amdgcn_s_setprio(0);
#ifdef SDNR_STAMPS
            SDNR_STAMP(st_t1);
            if (lane == 0) {
                atomicAdd(&g_stamp[0], st_t1 - st_t0);   // search wave lifetime
                atomicAdd(&g_stamp[1], st_row);          // row + gather cycles
                atomicAdd(&g_stamp[2], st_cand);         // candidates popped
                atomicAdd(&g_stamp[3], st_false);        // ... with no fresh child
                atomicAdd(&g_stamp[4], st_bp);           // back-pressure sleeps
                atomicAdd(&g_stamp[5], st_skip * 1000000ull + st_miss);   // skips, prefetch misses
                atomicAdd(&g_stamp[6], st_skipc);        // skip cycles
                atomicAdd(&g_stamp[7], st_pushc);        // push+publish cycles
            }
#endif
        } else {
            // ------------------------------------------------ the decrements
            int j = w - 1;                       // next child index of this worker
            for (unsigned spin = 0;;) {
                const int P = __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (j >= P) {
                    if (__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                        j >= __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
                        break;
                    if (++spin > kSpin) {
                        if (lane == 0) atomicOr(err, 2);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                spin = 0;
                const int n = (P - j + S - 1) / S < G ? (P - j + S - 1) / S : G;
                const int mine = lane < n ? (int)ring[(j + lane * S) & (RING - 1)] : V;
                if constexpr (PAIR == 2) {
                    constexpr int G2 = G / 2;
                    const int hiw = lane >> 5;
                    const uint32_t *rw32 = reinterpret_cast<const uint32_t *>(radj);
                    uint32_t r[G2];
#pragma unroll
                    for (int g = 0; g < G2; ++g) {
                        const int ca = read_lane(mine, 2 * g), cb = read_lane(mine, 2 * g + 1);
                        r[g] = rw32[(size_t)(hiw ? cb : ca) * 32 + (lane & 31)];
                    }
#pragma unroll
                    for (int g = 0; g < G2; ++g)
                        if (2 * g + hiw < n) {
                            atomicSub(&cnt[r[g] & 0xFFFFu], 1u);
                            atomicSub(&cnt[r[g] >> 16], 1u);
                        }
                    j += n * S;
                    if (lane == 0) __hip_atomic_store(&ctl[2 + w - 1], j, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    continue;
                }
                if constexpr (PAIR == 1) {
                    // rows repeat in lanes 32..63: load g serves child 2g in
                    // lanes 0..31 and child 2g + 1 in lanes 32..63 (a template
                    // case: a runtime branch here cost the unpaired k=48
                    // kernel 3 %)
                    constexpr int G2 = G / 2;
                    const int hiw = lane >> 5;
                    int r[G2];
#pragma unroll
                    for (int g = 0; g < G2; ++g) {
                        const int ca = read_lane(mine, 2 * g), cb = read_lane(mine, 2 * g + 1);
                        r[g] = radj[(size_t)(hiw ? cb : ca) * 64 + lane];
                    }
#pragma unroll
                    for (int g = 0; g < G2; ++g)
                        if (2 * g + hiw < n) {
                            if (C16) atomicSub(&cnt[r[g] >> 1], 1u << ((r[g] & 1) << 4));
                            else atomicSub(&cnt[r[g]], 1u);
                        }
                    j += n * S;
                    if (lane == 0) __hip_atomic_store(&ctl[2 + w - 1], j, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    continue;
                }
                int r[G];
                // unconditional: a slot past n loads the sentinel row V (L2
                // resident); guarding each load measured 20 % slower
#pragma unroll
                for (int g = 0; g < G; ++g) r[g] = radj[(size_t)read_lane(mine, g) * 64 + lane];
                if (flags & kFlagPreSwz) {
                    // pre-swizzled in-rows: entries are count-word indices
                    // (C16: word << 1 | half), padding points at a dummy
                    // word of its lane past the counts -- no compare, mask
                    // or swizzle arithmetic per child
#pragma unroll
                    for (int g = 0; g < G; ++g)
                        if (g < n) {
                            if (C16) atomicSub(&cnt[r[g] >> 1], 1u << ((r[g] & 1) << 4));
                            else atomicSub(&cnt[r[g]], 1u);
                        }
                } else {
#pragma unroll
                    for (int g = 0; g < G; ++g)
                        if (g < n && r[g] != V) {
                            if (C16) atomicSub(&cnt[swz(r[g] >> 1)], 1u << ((r[g] & 1) << 4));
                            else atomicSub(&cnt[swz(r[g])], 1u);
                        }
                }
                j += n * S;
                if (lane == 0) __hip_atomic_store(&ctl[2 + w - 1], j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
#ifdef SDNR_STAMPS
        SDNR_STAMP(ph2);
#endif

        // tables: UF vertices per thread, their port loads (one ELL load, or
        // row_ptr + port) all in flight before the stores.  A wave's
        // vector-memory counter retires loads and stores in issue order, so
        // a port gather issued after the previous pass's table stores waits
        // for their acknowledgement: fewer, wider passes (k=48 at 8 waves:
        // one pass)
        constexpr int UF = SDNR_ASYNC_FLUSH_U;
        for (int v0 = threadIdx.x; v0 < V; v0 += UF * blockDim.x) {
            int p[UF], sl[UF], pt[UF];
#pragma unroll
            for (int k = 0; k < UF; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                p[k] = -1;
                sl[k] = -1;
                if (v < V && ((vis[v >> 5] >> (v & 31)) & 1u)) {
                    if (C16) {
                        p[k] = (int)ps16[swz(v)];
                        if (v != s) sl[k] = (int)sl8[swz(v)];
                    } else {
                        const uint32_t xx = ps[swz(v)];
                        p[k] = (int)(xx & 0xFFFFu);
                        if (v != s) sl[k] = (int)(xx >> 16);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < UF; ++k) {
                pt[k] = -1;
                if (sl[k] >= 0)
                    pt[k] = W > 0 ? ell_port[(size_t)p[k] * W + sl[k]] : port[row_ptr[p[k]] + sl[k]];
            }
#pragma unroll
            for (int k = 0; k < UF; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                if (v < V) {
                    if (PACKED) {                // parent | port << 16, -1 -> 0xFFFF
                        prow[v] = (int32_t)(((uint32_t)p[k] & 0xFFFFu) |
                                            ((uint32_t)pt[k] << 16));
                    } else {
                        prow[v] = p[k];
                        trow[v] = pt[k];
                    }
                    if (HOPS) put_hop(out_hops, hb + v, p[k] < 0 ? -1 : (v == s ? 0 : (int)dep[v]),
                                      flags);
                }
            }
        }
        // the next source's init reuses the LDS state; a workgroup on its
        // last source (the headline: one source per workgroup) skips the
        // barrier, whose release fence waited for every table store of the
        // wave to be acknowledged (the flush measured 57.5 k of a 291 k-cycle
        // source life at 1,152 sources, 4.2 k at one: stamps)
        if (si + (int)gridDim.x < nsrc) __syncthreads();
#ifdef SDNR_STAMPS
        SDNR_STAMP(ph3);
        if (threadIdx.x == 0) {
            atomicAdd(&g_stamp[8], ph1 - ph0);       // init
            atomicAdd(&g_stamp[9], ph2 - ph1);       // search + worker tail
            atomicAdd(&g_stamp[10], ph3 - ph2);      // flush
        }
#endif
    }
#ifdef SDNR_STAMPS
    if (threadIdx.x == 0) {                      // span of the launch: last end, first start
        unsigned long long t;
        SDNR_STAMP(t);
        atomicMax(&g_stamp[11], t);
        atomicMax(&g_stamp[12], ~kstart);
    }
#endif
}

// slot trees from int32 ones: slot = position of v in parent's ascending CSR
// row (binary search); the root (parent == v) gets slot 63
__global__ __launch_bounds__(256) void dfs_slot_pack_kernel(size_t n, int V,
                                                            const int32_t *__restrict__ parent,
                                                            const int32_t *__restrict__ row_ptr,
                                                            const int32_t *__restrict__ col,
                                                            uint32_t *__restrict__ tree)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int v = (int)(i % (size_t)V), p = parent[i];
        uint32_t t = 0xFFFFFFFFu;
        if (p == v) {
            t = (uint32_t)p | (63u << 26);
        } else if (p >= 0) {
            int lo = row_ptr[p], hi = row_ptr[p + 1];
            const int base = lo;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (col[mid] < v) lo = mid + 1; else hi = mid;
            }
            t = (uint32_t)p | ((uint32_t)(lo - base) << 26);
        }
        tree[i] = t;
    }
}

// packed tables from int32 ones (strategies without a packed epilogue)
__global__ __launch_bounds__(256) void dfs_pack_kernel(size_t n, const int32_t *__restrict__ parent,
                                                       const int32_t *__restrict__ port,
                                                       uint32_t *__restrict__ tree)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        tree[i] = ((uint32_t)parent[i] & 0xFFFFu) | ((uint32_t)port[i] << 16);
}

template <typename Kern>
void allow_full_lds(Kern kernel)
{
    sdnr_allow_lds(reinterpret_cast<const void *>(kernel), SDNR_MAX_LDS_PER_BLOCK);
}

size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

}  // namespace

// LDS bytes per source of the two strategies
static size_t dfs_lds_bytes_small(int V)
{
    const size_t VWp = (size_t)((((V + 31) >> 5) + 3) & ~3);
    return align16(4 * VWp + 8 * (size_t)V + 2 * (size_t)V);
}

static size_t dfs_lds_bytes_global(int V, int ring = kRing)
{
    const size_t VWp = (size_t)((((V + 31) >> 5) + 3) & ~3);
    return align16(4 * VWp + 8 * (size_t)ring);
}

// stack-ring entries of the lane-packed kernel: small rings leave room for
// more resident sources on large graphs (the torus search is a chain of
// ~14k non-leaf pops per source: throughput comes from sources in flight);
// SDNROUTE_DFS_RING=128|1024 overrides
static int packed_ring(int V, int W)
{
    if (const char *f = getenv("SDNROUTE_DFS_RING")) {
        const int r = atoi(f);
        if (r == 128 || r == 1024) return r;
    }
    return V > 16384 && W <= 8 ? 128 : 1024;
}

// stack entries checked per batch by the lane-packed kernel with 8 lanes per
// row: J = 1 (8 entries) or 2 (16).  On the torus 13.6k of 32.8k pops push
// children, so a batch rarely retires more than two entries: the narrower
// batch halves the row traffic per step (torus 32^3: 108 -> 99 ms).
// SDNROUTE_DFS_PACKED_J overrides
static int packed_j8(int V)
{
    if (const char *f = sdnr_tune_env("SDNROUTE_DFS_PACKED_J")) {
        const int j = atoi(f);
        if (j == 1 || j == 2) return j;
    }
    return V > 16384 ? 1 : 2;
}

namespace {

struct DfsArgs {
    int V, W;
    const int32_t *row_ptr, *col, *port, *src;
    int nsrc;
    int32_t *parent, *port_out, *hops;
    uint2 *spill;
    const int32_t *port_csr;
};

template <bool ELL, bool HOPS, int K>
void launch_batch(bool small, int grid, size_t lds, hipStream_t st, const DfsArgs &a)
{
    if (small) {
        auto k = dfs_lds_batch_kernel<ELL, HOPS, K>;
        allow_full_lds(k);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, st, a.V, a.W, a.row_ptr, a.col, a.port,
                           a.src, a.nsrc, a.parent, a.port_out, a.hops);
    } else {
        auto k = dfs_global_batch_kernel<ELL, HOPS, K>;
        allow_full_lds(k);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, st, a.V, a.W, a.row_ptr, a.col, a.port,
                           a.src, a.nsrc, a.parent, a.port_out, a.hops, a.spill);
    }
}

template <bool ELL, bool HOPS>
void launch_batch_k(int K, bool small, int grid, size_t lds, hipStream_t st, const DfsArgs &a)
{
    if (K >= 16) launch_batch<ELL, HOPS, 16>(small, grid, lds, st, a);
    else if (K >= 8) launch_batch<ELL, HOPS, 8>(small, grid, lds, st, a);
    else if (K >= 4) launch_batch<ELL, HOPS, 4>(small, grid, lds, st, a);
    else launch_batch<ELL, HOPS, 1>(small, grid, lds, st, a);
}

template <bool HOPS>
void launch_wide(bool small, int grid, size_t lds, hipStream_t st, const DfsArgs &a)
{
    if (small) {
        auto k = dfs_lds_wide_kernel<false, HOPS>;
        allow_full_lds(k);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, st, a.V, a.W, a.row_ptr, a.col, a.port,
                           a.src, a.nsrc, a.parent, a.port_out, a.hops);
    } else {
        auto k = dfs_global_wide_kernel<false, HOPS>;
        allow_full_lds(k);
        hipLaunchKernelGGL(k, dim3(grid), dim3(64), lds, st, a.V, a.W, a.row_ptr, a.col, a.port,
                           a.src, a.nsrc, a.parent, a.port_out, a.hops, a.spill);
    }
}

}  // namespace

static size_t dfs_lds_bytes_count(int V, bool hops)
{
    const size_t VWp = (size_t)((((V + 1 + 31) >> 5) + 3) & ~3);
    const size_t CWp = (size_t)((V + 1 + 3) & ~3);
    const size_t SWp = (size_t)((((V + 1) >> 1) + 3) & ~3);
    return align16(4 * (VWp + CWp + SWp) + 4 * (size_t)V + (hops ? 2 * (size_t)V : 0));
}

static size_t dfs_lds_bytes_async(int V, bool hops, bool c16 = false)
{
    const size_t VWp = (size_t)((((V + 1 + 31) >> 5) + 3) & ~3);
    const size_t CWp = (size_t)(((((c16 ? (V + 2) >> 1 : V + 1) + 31) & ~31) + 64 + 255) & ~255);
    const size_t SWp = (size_t)((((V + 1) >> 1) + 3) & ~3);
    const size_t PW = (size_t)((V + 255) & ~255);
    const size_t PWp = c16 ? PW / 2 + PW / 4 : PW;
    return align16(4 * (VWp + CWp + SWp) + 4 * PWp +
                   (hops ? 4 * (size_t)((V + 1) >> 1) : 0) + 2 * 512 + 4 * 16);
}

static size_t dfs_lds_bytes_coop(int V)
{
    const size_t VWp = (size_t)((((V + 1 + 31) >> 5) + 3) & ~3);
    return align16(4 * VWp + 8 * (size_t)V + 4 * (size_t)((V + 1) >> 1) + 4 * 32);
}

namespace {

template <bool HOPS, int KW>
void launch_coop_kw(int grid, size_t lds, hipStream_t st, int V, const uint16_t *adj,
                    const DfsArgs &a)
{
    auto k = dfs_coop_kernel<4, KW, HOPS>;
    allow_full_lds(k);
    hipLaunchKernelGGL(k, dim3(grid), dim3(4 * 64), lds, st, V, adj, a.row_ptr,
                       a.port_csr, a.src, a.nsrc, a.parent, a.port_out,
                       a.hops);
}

template <bool HOPS>
void launch_coop(int kw, int grid, size_t lds, hipStream_t st, int V, const uint16_t *adj,
                 const DfsArgs &a)
{
    if (kw >= 8) launch_coop_kw<HOPS, 8>(grid, lds, st, V, adj, a);
    else if (kw >= 4) launch_coop_kw<HOPS, 4>(grid, lds, st, V, adj, a);
    else launch_coop_kw<HOPS, 2>(grid, lds, st, V, adj, a);
}

}  // namespace

// slots per wave of the cooperative kernel (4 waves): SDNROUTE_DFS_COOP_KW
static int dfs_coop_kw()
{
    if (const char *f = sdnr_tune_env("SDNROUTE_DFS_COOP_KW")) {
        const int k = atoi(f);
        if (k == 2 || k == 4 || k == 8) return k;
    }
    return 4;
}

#ifdef SDNR_STAMPS
extern "C" int sdnr_debug_stamps(unsigned long long *out16)
{
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_stamp), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -5;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), z, sizeof z) == hipSuccess ? 0 : -5;
}
#endif

// waves per source of the asynchronous kernel: SDNROUTE_DFS_ASYNC_WAVES=2|3|4
// waves per source of the async kernel: 1 search + decrement workers, whose
// work per child is its in-degree -- 3 workers for rows of 33-64 neighbours
// (k=48: 0.116 ms vs 0.138 with 2), 2 for rows of <= 32 (dragonfly, 23
// neighbours: 0.289 vs 0.300 ms with 3); SDNROUTE_DFS_ASYNC_WAVES=2..6
static int dfs_async_waves(const sdnr_ctx *ctx, int nsrc)
{
    if (const char *f = getenv("SDNROUTE_DFS_ASYNC_WAVES")) {
        const int k = atoi(f);
        if ((k >= 2 && k <= 6) || k == 8) return k;
    }
    // at most ~2 sources per CU (one GPU's share of a multi-GPU step, single
    // sources): 5 decrement workers keep the counts fresher and the search
    // wave still has its SIMD mostly to itself -- k=48 1 / 144 / 256 / 288
    // sources 63.4 / 64.3 / 65.1 / 69.1 -> 56.8 / 58.4 / 59.4 / 64.2 us,
    // dragonfly 258 sources 127.7 -> 120.8 us; equal at 576 sources, and
    // slower once every CU holds several sources (k=48 1,152: 91.6 -> 137 us
    // with 4 workers), where the workers compete with the search waves.
    // Round 4: with the dword-paired rows (in-degree > 32) 7 workers -- k=48
    // 144 / 1 sources 48.8 / 47.1 -> 46.9 / 45.1 us
    if (nsrc <= 2 * ctx->num_cus) return ctx->radj_pair ? 6 : 8;
    return ctx->max_deg <= 32 ? 3 : 4;
}

// waves per source of the counted-pop kernel: SDNROUTE_DFS_COUNT_WAVES=2|4|6
static int dfs_count_waves()
{
    if (const char *f = sdnr_tune_env("SDNROUTE_DFS_COUNT_WAVES")) {
        const int k = atoi(f);
        if (k == 2 || k == 4 || k == 6) return k;
    }
    return 4;
}

// SDNROUTE_DFS_PACKED=0 disables the lane-packed large-graph kernel
static bool packed_ok()
{
    const char *f = getenv("SDNROUTE_DFS_PACKED");
    return !(f && !strcmp(f, "0"));
}

// pops checked per batch: wide rows make each leaf pop expensive, so batch
// deeper; SDNROUTE_DFS_BATCH=1|4|8|16 overrides (tuning / tests)
static int dfs_batch_depth(const sdnr_ctx *ctx)
{
    if (const char *f = sdnr_tune_env("SDNROUTE_DFS_BATCH")) {
        const int k = atoi(f);
        if (k == 1 || k == 4 || k == 8 || k == 16) return k;
    }
    return ctx->max_deg >= 12 ? 16 : 8;
}

static int dfs_flags(int dflt = 0)
{
    const char *f = sdnr_tune_env("SDNROUTE_DFS_FLAGS");
    const int v = f ? atoi(f) : dflt;
#ifdef SDNR_DIAG_VARIANTS
    return v;
#else
    // the timing diagnostics that leave the tables wrong (no stores, no port
    // lookups) exist only in the diagnostic build
    return v & ~(kFlagNoStore | kFlagNoPort);
#endif
}

// SDNROUTE_DFS_SPLIT=0 keeps the single-wave lane-packed kernel (A/B, tests)
static bool split_ok()
{
    const char *f = getenv("SDNROUTE_DFS_SPLIT");
    return !(f && !strcmp(f, "0"));
}

// search / writer split kernel (large graphs, rows of <= 32 slots); records
// the end event itself
template <int NS>
static int launch_split_ns(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                           int32_t *d_port, int32_t *d_hops, uint32_t *d_tree, int tree,
                           int hflags);

// search waves per workgroup: 7 on sparse tori (4 workgroups of 8 waves fill
// a CU's 32 wave slots with 28 sources), else 3 (LDS-bound: Jellyfish fits 3
// workgroups of 3 sources); SDNROUTE_DFS_SPLIT_NS=3|7 overrides
static int launch_split(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                        int32_t *d_port, int32_t *d_hops, uint32_t *d_tree, int tree, int hflags)
{
    int ns = ctx->W <= 8 && packed_j8(ctx->V) == 1 ? 7 : 3;
    if (ctx->W > 8 && ctx->W <= 16) {
        // rows of 9-16 slots (Jellyfish): 3 or 5 sources per workgroup,
        // whichever keeps more sources resident per CU (100k Jellyfish
        // without hop counts: 2 x 5 = 10 vs 3 x 3 = 9, measured 5 % faster)
        const bool hops = d_hops != nullptr;
        auto per_cu = [&](int k) {
            const size_t l = split_lds_words(ctx->V, 512, k, hops, 16) * 4;
            size_t b = SDNR_LDS_PER_CU / l;
            if (b > (size_t)(32 / (k + 1))) b = 32 / (k + 1);
            return (size_t)k * b;
        };
        if (per_cu(5) > per_cu(3)) ns = 5;
    }
    if (const char *f = getenv("SDNROUTE_DFS_SPLIT_NS")) {
        const int k = atoi(f);
        if (k == 3 || k == 7) ns = k;
        if ((k == 5 || k == 11) && ctx->W > 8 && ctx->W <= 16) ns = k;   // rows of 9-16 slots
    }
    switch (ns) {
    case 7: return launch_split_ns<7>(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree, tree,
                                     hflags);
    case 5: return launch_split_ns<5>(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree, tree,
                                     hflags);
    case 11: return launch_split_ns<11>(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree, tree,
                                      hflags);
    default: return launch_split_ns<3>(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree, tree,
                                     hflags);
    }
}

template <int NS>
static int launch_split_ns(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                           int32_t *d_port, int32_t *d_hops, uint32_t *d_tree, int tree,
                           int hflags)
{
    const int V = ctx->V, W = ctx->W;
    const bool packed = d_tree != nullptr, hops = d_hops != nullptr;
    const int lpr = W <= 8 ? 8 : (W <= 16 ? 16 : 32);
    const int j8 = packed_j8(V);
    // stack ring: 128 entries on sparse tori (more sources per CU), 512 for
    // rows of 9-32 slots (Jellyfish: 3 workgroups of 3 sources per CU)
    int ring = lpr == 8 ? (j8 == 1 ? 128 : 1024) : 512;
    if (const char *f = getenv("SDNROUTE_DFS_SPLIT_RING"))   // rows of 9-16 slots
        if (lpr == 16 && !strcmp(f, "256")) ring = 256;
    constexpr bool kWide = NS == 5 || NS == 11;   // only for rows of 9-16 slots
    if (kWide && lpr != 16) return sdnr_fail(SDNR_ERR_INVAL, "dfs split: NS=%d needs rows of 9-16 slots", NS);
    const int fmt = ctx->ell16 && V <= 65535 ? kRow16 : (ctx->ell16 && ctx->ell_hi ? kRow17 : kRow32);
    if (tree == kTreePort16 && fmt != kRow16)
        return sdnr_fail(SDNR_ERR_INVAL, "dfs split: packed tables need V <= 65535");
    if (tree == kTreeSlot && hops && fmt == kRow32)
        return sdnr_fail(SDNR_ERR_INVAL, "dfs split: slot trees with hop counts need V < 131071");
    // dictionary rows where the upload built them (rows of <= 8 slots)
    const bool dict = ctx->dict_bp && lpr == 8 && !kWide;
    const size_t dict_words =
        dict ? (size_t)ctx->dict_bpw + 8 * (size_t)ctx->dict_NB + 8 * (size_t)ctx->dict_P : 0;
    const size_t lds = (split_lds_words(V, ring, NS, hops, lpr, dict) + dict_words) * 4;
    if (lds > SDNR_MAX_LDS_PER_BLOCK)
        return sdnr_fail(SDNR_ERR_INVAL, "graph too large for the LDS visited sets (V=%d)", V);
    size_t bpc = SDNR_LDS_PER_CU / lds;
    if (bpc > (size_t)(32 / (NS + 1))) bpc = 32 / (NS + 1);    // 32 wave slots per CU
    if (bpc < 1) bpc = 1;
    int grid = (int)((size_t)ctx->num_cus * bpc);
    const int need = (nsrc + NS - 1) / NS;
    if (grid > need) grid = need;
    int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes,
                          (size_t)grid * NS * (size_t)V * sizeof(uint2));
    if (rc) return rc;
    uint2 *spill = static_cast<uint2 *>(ctx->scratch);
    const void *rows = fmt == kRow32 ? static_cast<const void *>(ctx->ell_col)
                                     : static_cast<const void *>(ctx->ell16);
    int32_t *par = packed ? reinterpret_cast<int32_t *>(d_tree) : d_parent;
    static const char *names[4][3] = {
        {"dfs_split_kernel<row32>", "dfs_split_kernel<row32>", "dfs_split_kernel<row32,slots>"},
        {"dfs_split_kernel<row16>", "dfs_split_kernel<row16,packed>", "dfs_split_kernel<row16,slots>"},
        {"dfs_split_kernel<row17>", "dfs_split_kernel<row17>", "dfs_split_kernel<row17,slots>"},
        {"dfs_split_kernel<dict>", "dfs_split_kernel<dict,packed>", "dfs_split_kernel<dict,slots>"}};
    ctx->last_kernel = names[dict ? kRowDict : fmt][tree];
    // rows of 9-16 slots (Jellyfish): search waves issue at raised priority
    // over their writer (measured 1.027 -> 0.973 s on the 100k Jellyfish; the
    // torus rows of 6 slots measured 3 % slower with it, so not there)
    int flags = dfs_flags(lpr == 16 ? kFlagPrio : 0) | hflags;
    // sources by CU chunk (kFlagCuMap; SDNROUTE_DFS_CUMAP=0|1 overrides):
    // same box A/B, torus 32^3 99.6 -> 86.4 ms, Jellyfish 100k 976 -> 883 ms
    bool cumap = true;
    if (const char *f = getenv("SDNROUTE_DFS_CUMAP")) cumap = !strcmp(f, "1");
    const int nch = ctx->num_cus;
    int *wq = nullptr;
    if (cumap) {
        flags |= kFlagCuMap;
        rc = sdnr_reserve(&ctx->wq, &ctx->wq_bytes, (size_t)(nch + 1 + 1024) * sizeof(int));
        if (rc) return rc;
        wq = static_cast<int *>(ctx->wq);
        SDNR_HIP(hipMemsetAsync(wq, 0, (size_t)(nch + 1) * sizeof(int), ctx->stream));
        SDNR_HIP(hipMemsetAsync(wq + nch + 1, 0xFF, 1024 * sizeof(int), ctx->stream));
    }
#define SDNR_SPLIT(L_, J_, R_, H_, F_, P_)                                                    \
    do {                                                                                     \
        auto k = dfs_split_kernel<L_, J_, H_, R_, NS, F_, P_>;                               \
        sdnr_allow_lds(reinterpret_cast<const void *>(k), lds);                              \
        hipLaunchKernelGGL(k, dim3(grid), dim3((NS + 1) * 64), lds, ctx->stream, V, W, rows,     \
                           ctx->ell_hi, ctx->ell_port, d_src, nsrc, par, d_port, d_hops,     \
                           spill, ctx->d_err, flags, wq, nch, ctx->dict_bp, ctx->dict_bt,    \
                           ctx->dict_off, ctx->dict_bpw, ctx->dict_NB, ctx->dict_P);         \
    } while (0)
#define SDNR_SPLIT_F(L_, J_, R_, H_)                                                          \
    do {                                                                                     \
        if constexpr (L_ == 8 && !kWide) {                                                   \
            if (dict) {                                                                      \
                if (tree == kTreeSlot) SDNR_SPLIT(L_, J_, R_, H_, kRowDict, kTreeSlot);      \
                else if (packed) SDNR_SPLIT(L_, J_, R_, H_, kRowDict, kTreePort16);          \
                else SDNR_SPLIT(L_, J_, R_, H_, kRowDict, kTreeInt32);                       \
                break;                                                                       \
            }                                                                                \
        }                                                                                    \
        if (tree == kTreeSlot) {                                                             \
            if (fmt == kRow16) SDNR_SPLIT(L_, J_, R_, H_, kRow16, kTreeSlot);                \
            else if (fmt == kRow17) SDNR_SPLIT(L_, J_, R_, H_, kRow17, kTreeSlot);           \
            else if constexpr (!H_) SDNR_SPLIT(L_, J_, R_, H_, kRow32, kTreeSlot);           \
            break;                                                                           \
        }                                                                                    \
        if (fmt == kRow16 && packed) SDNR_SPLIT(L_, J_, R_, H_, kRow16, kTreePort16);        \
        else if (fmt == kRow16) SDNR_SPLIT(L_, J_, R_, H_, kRow16, kTreeInt32);              \
        else if (fmt == kRow17) SDNR_SPLIT(L_, J_, R_, H_, kRow17, kTreeInt32);              \
        else SDNR_SPLIT(L_, J_, R_, H_, kRow32, kTreeInt32);                                 \
    } while (0)
#define SDNR_SPLIT_H(L_, J_, R_)                                                              \
    do {                                                                                     \
        if (hops) SDNR_SPLIT_F(L_, J_, R_, true); else SDNR_SPLIT_F(L_, J_, R_, false);      \
    } while (0)
    if constexpr (kWide) {
        // stack entries per window: 8 (J = 2; SDNROUTE_DFS_SPLIT_J=4|1 for 16 |
        // 4).  Same box, 100k Jellyfish, all sources (gpurun_out/r5_jfj2): 16
        // entries 880 ms, 8 entries 833 ms, 4 entries 875 ms -- the window's
        // row loads (the CU's data return is ~90 % busy) against the leaf
        // skips a narrower window takes more iterations for
        const char *jf = getenv("SDNROUTE_DFS_SPLIT_J");
        const int jw = jf && (atoi(jf) == 4 || atoi(jf) == 1) ? atoi(jf) : 2;
        if (ring == 256) SDNR_SPLIT_H(16, 4, 256);
        else if (jw == 2) SDNR_SPLIT_H(16, 2, 512);
        else if (jw == 1) SDNR_SPLIT_H(16, 1, 512);
        else SDNR_SPLIT_H(16, 4, 512);
    } else {
        if (lpr == 8 && ring == 128) SDNR_SPLIT_H(8, 1, 128);
        else if (lpr == 8) SDNR_SPLIT_H(8, 2, 1024);
        else if (lpr == 16 && ring == 256) SDNR_SPLIT_H(16, 4, 256);
        else if (lpr == 16) SDNR_SPLIT_H(16, 4, 512);
        else SDNR_SPLIT_H(32, 8, 512);
    }
#undef SDNR_SPLIT_H
#undef SDNR_SPLIT_F
#undef SDNR_SPLIT
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}

int sdnr_launch_tree_pack(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port, size_t n,
                          uint32_t *tree, bool slots)
{
    const int V = ctx->V;
    if (slots)
        hipLaunchKernelGGL(dfs_slot_pack_kernel, dim3(ctx->num_cus * 8), dim3(256), 0,
                           ctx->stream, n, V, parent, ctx->row_ptr, ctx->col, tree);
    else
        hipLaunchKernelGGL(dfs_pack_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                           n, parent, port, tree);
    SDNR_HIP(hipGetLastError());
    return SDNR_OK;
}

#ifdef SDNR_DIAG_VARIANTS
// the register-visited kernel (dfs_bits.hip) where it applies: forced with
// SDNROUTE_DFS_STRATEGY=bits (A/B; not yet the default)
static bool dfs_bits_default(const char *force)
{
    return force && !strcmp(force, "bits");
}

#endif

// the async kernel for a row form: compact LDS (C16), paired in-rows,
// dword-paired in-rows, or plain u16 in-rows
template <int N_, bool H_, bool P_, bool SPEC>
static auto async_pick(bool c16, bool pair, bool dw)
{
    // (SPEC: the plain-row kernel only -- the compact / paired forms, the
    // dragonfly's, measured slower with the speculative pop compiled in:
    // 2,064 sources 177.3 -> 180.4 us, gpurun_out/r5_abspec)
    return c16 ? (pair ? dfs_async_kernel<N_, H_, P_, true, 1>
                       : dfs_async_kernel<N_, H_, P_, true, 0>)
               : (pair ? dfs_async_kernel<N_, H_, P_, false, 1>
                       : (dw ? dfs_async_kernel<N_, H_, P_, false, 2>
                             : dfs_async_kernel<N_, H_, P_, false, 0, SPEC>));
}

// hop counts as u16 (0xFFFF unreached) into d_hops
__global__ __launch_bounds__(256) void dfs_hops16_kernel(size_t n, const int32_t *__restrict__ h,
                                                         uint16_t *__restrict__ out)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        out[i] = (uint16_t)h[i];
}

int sdnr_launch_dfs(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc,
                    int32_t *d_parent, int32_t *d_port, int32_t *d_hops, uint32_t *d_tree,
                    bool slots, bool hops16)
{
    const int V = ctx->V;
    if (nsrc == 0 || V == 0) return SDNR_OK;
    const bool packed = d_tree != nullptr;
    const bool ell = ctx->W > 0;
    const bool hops = d_hops != nullptr;
    const bool narrow = ctx->max_deg <= SDNR_WAVE;     // one row = one wavefront
    const size_t small_b = dfs_lds_bytes_small(V);
    const size_t cu_blocks_small = SDNR_LDS_PER_CU / small_b;
    bool small = V < 65536 && small_b <= 64 * 1024 &&
                 (small_b <= 40 * 1024 ||
                  (size_t)nsrc <= (size_t)ctx->num_cus * cu_blocks_small);
    // debug/test knob: SDNROUTE_DFS_STRATEGY=lds|global forces a strategy
    if (const char *f = getenv("SDNROUTE_DFS_STRATEGY")) {
        if (!strcmp(f, "global")) small = false;
        else if ((!strcmp(f, "lds") || !strcmp(f, "coop") || !strcmp(f, "count") ||
                  !strcmp(f, "async")) && V < 65536 &&
                 small_b <= SDNR_MAX_LDS_PER_BLOCK)
            small = true;
    }
    size_t lds = small ? small_b : dfs_lds_bytes_global(V);
    if (lds > SDNR_MAX_LDS_PER_BLOCK)
        return sdnr_fail(SDNR_ERR_INVAL, "graph too large for the LDS visited set (V=%d)", V);
    size_t bpc = SDNR_LDS_PER_CU / lds;
    if (bpc > 16) bpc = 16;
    if (bpc < 1) bpc = 1;
    int grid = (int)((size_t)ctx->num_cus * bpc);
    if (grid > nsrc) grid = nsrc;
    uint2 *spill = nullptr;
    if (!small) {
        const size_t need = (size_t)grid * (size_t)V * sizeof(uint2);
        int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes, need);
        if (rc) return rc;
        spill = static_cast<uint2 *>(ctx->scratch);
    }
    DfsArgs a{V, ctx->W, ctx->row_ptr, ell ? ctx->ell_col : ctx->col,
              ell ? ctx->ell_port : ctx->port, d_src, nsrc, d_parent, d_port, d_hops, spill,
              ctx->port};
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    const char *force = getenv("SDNROUTE_DFS_STRATEGY");
#ifdef SDNR_DIAG_VARIANTS
    // diagnostic build only (tools/diag/build_diag.sh): the two losing
    // variants of DESIGN.md 4.1a / 4.1b, forced by SDNROUTE_DFS_STRATEGY
    // rows in LDS as arithmetic runs (dfs_runs.hip), SDNROUTE_DFS_STRATEGY=
    // runs: measured no faster than dfs_async_kernel, so
    // opt-in
    if (!(slots && packed) && sdnr_dfs_runs_ok(ctx, hops) && force && !strcmp(force, "runs")) {
        int rc = sdnr_launch_dfs_runs(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree);
        if (rc) return rc;
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    // bitmap rows, visited set in registers (dfs_bits.hip): V <= 4096;
    // SDNROUTE_DFS_STRATEGY=bits forces it (A/B), =async the round-3 kernel
    if (!slots && sdnr_dfs_bits_ok(ctx) && dfs_bits_default(force)) {
        int rc = sdnr_launch_dfs_bits(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree, hops16);
        if (rc) return rc;
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
#endif
    const bool count_ok = ctx->adj16 != nullptr && ctx->radj16 != nullptr && V < 65535 &&
                          dfs_lds_bytes_count(V, hops) <= SDNR_MAX_LDS_PER_BLOCK;
    const bool async_ok = count_ok && dfs_lds_bytes_async(V, hops) <= SDNR_MAX_LDS_PER_BLOCK;
    const bool async = async_ok && (force ? !strcmp(force, "async") : small);
    slots = slots && packed;
    const int hflags = hops && hops16 ? kFlagHops16 : 0;
    if (!async && !small && ell && ctx->W <= 32 && packed_ok() && split_ok() &&
        (!packed || slots || (ctx->ell16 && V <= 65535)) &&
        !(slots && hops && !(ctx->ell16 && (V <= 65535 || ctx->ell_hi))))
        return launch_split(ctx, d_src, nsrc, d_parent, d_port, d_hops, d_tree,
                            slots ? kTreeSlot : (packed ? kTreePort16 : kTreeInt32), hflags);
    if ((packed && (!async || slots)) || (hops && hops16 && !async)) {
        // no such epilogue in this strategy: int32 tables into scratch, then
        // pack (and narrow the hop counts)
        const size_t n = (size_t)nsrc * (size_t)V;
        const bool h16 = hops && hops16;
        int rc = sdnr_reserve(&ctx->scratch2, &ctx->scratch2_bytes,
                              (h16 ? 3 : 2) * n * sizeof(int32_t));
        if (rc) return rc;
        int32_t *tp = static_cast<int32_t *>(ctx->scratch2);
        int32_t *th = h16 ? tp + 2 * n : d_hops;
        if (!packed) {                           // int32 tables, u16 hop counts
            if ((rc = sdnr_launch_dfs(ctx, d_src, nsrc, d_parent, d_port, tp, nullptr))) return rc;
            hipLaunchKernelGGL(dfs_hops16_kernel, dim3(ctx->num_cus * 8), dim3(256), 0,
                               ctx->stream, n, tp, reinterpret_cast<uint16_t *>(d_hops));
            SDNR_HIP(hipGetLastError());
            if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
            return SDNR_OK;
        }
        if ((rc = sdnr_launch_dfs(ctx, d_src, nsrc, tp, tp + n, th, nullptr))) return rc;
        if (h16)
            hipLaunchKernelGGL(dfs_hops16_kernel, dim3(ctx->num_cus * 8), dim3(256), 0,
                               ctx->stream, n, th, reinterpret_cast<uint16_t *>(d_hops));
        if (slots)
            hipLaunchKernelGGL(dfs_slot_pack_kernel, dim3(ctx->num_cus * 8), dim3(256), 0,
                               ctx->stream, n, V, tp, ctx->row_ptr, ctx->col, d_tree);
        else
            hipLaunchKernelGGL(dfs_pack_kernel, dim3(ctx->num_cus * 8), dim3(256), 0, ctx->stream,
                               n, tp, tp + n, d_tree);
        SDNR_HIP(hipGetLastError());
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    const bool count = !async && count_ok && (force ? !strcmp(force, "count") : small);
    const bool coop_ok = ctx->adj16 != nullptr && V < 65535 &&
                         dfs_lds_bytes_coop(V) <= SDNR_MAX_LDS_PER_BLOCK;
    const bool coop = !count && coop_ok && (force ? !strcmp(force, "coop") : small);
    if (async) {
        int *err = ctx->d_err;
        const int nw = dfs_async_waves(ctx, nsrc);
        // workgroups per CU: LDS, and the 32 wave slots; the compact layout
        // (u16 counts, u16 parents + u8 slots) where it holds more sources
        // at once and the full layout cannot hold them all (dragonfly 2,064
        // sources: 9 x 3 waves per CU vs 6); SDNROUTE_DFS_C16=0|1 forces it
        auto per_cu = [&](bool c) {
            size_t b = SDNR_LDS_PER_CU / dfs_lds_bytes_async(V, hops, c);
            if (b > (size_t)(32 / nw)) b = 32 / nw;
            return b < 1 ? (size_t)1 : b;
        };
        bool c16 = per_cu(true) > per_cu(false) &&
                   (size_t)ctx->num_cus * per_cu(false) < (size_t)nsrc;
        if (const char *f = getenv("SDNROUTE_DFS_C16")) c16 = !strcmp(f, "1");
        const size_t cl = dfs_lds_bytes_async(V, hops, c16);
        const size_t cpc = per_cu(c16);
        // pre-swizzled worker rows (SDNROUTE_DFS_PRESWZ=0 keeps the plain ones)
        const char *pz = getenv("SDNROUTE_DFS_PRESWZ");
        const uint16_t *rw = c16 ? ctx->radjc : ctx->radjw;
        const bool preswz = rw && !(pz && !strcmp(pz, "0"));
        // speculative stack pops (SDNROUTE_DFS_SPECPOP=0|1).
        // Compiled into the 4-wave plain-row kernel only (the k=48
        // headline's regime: 1,152 sources 83.0 -> 82.3 us, same ISA with
        // the pop off / on): its code cost the 8-wave low-load kernel ~8 us
        // even switched off, and the dragonfly's 3-wave compact kernel 1-2 %
        // (see dfs_async_kernel's SPEC; gpurun_out/r5_abr4, r5_abspec)
        bool specpop = true;
        if (const char *f = getenv("SDNROUTE_DFS_SPECPOP")) specpop = !strcmp(f, "1");
        const bool spec = specpop;
        const int aflags = dfs_flags(kFlagPrio) | (preswz ? kFlagPreSwz : 0) | hflags |
                           (specpop ? kFlagSpecPop : 0);
        // paired worker rows (in-degree <= 32, pre-swizzled rows only);
        // else, at <= 2 sources per CU (the 5-worker regime), dword-paired
        // rows: k=48 1 / 144 sources 56.3 / 57.8 -> 54.7 / 56.4 us; at the
        // 1,152-source headline they measured 0.0895 -> 0.1010 ms, so the
        // u16 rows stay there (SDNROUTE_DFS_DW=0|1 forces either)
        const bool pair = preswz && ctx->radj_pair;
        const char *dq = sdnr_tune_env("SDNROUTE_DFS_DW");
        bool dw = preswz && !pair && !c16 && nw >= 6;
        if (dq) dw = preswz && !pair && !c16 && !strcmp(dq, "1");
        int cgrid = (int)((size_t)ctx->num_cus * cpc);
        if (cgrid > nsrc) cgrid = nsrc;
        // the search wave issues at raised priority over the decrement
        // workers (dragonfly 0.316 -> 0.300 ms, k=48 unchanged)
        static const char *names[] = {"", "", "dfs_async_kernel<2>", "dfs_async_kernel<3>",
                                      "dfs_async_kernel<4>", "dfs_async_kernel<5>",
                                      "dfs_async_kernel<6>", "", "dfs_async_kernel<8>"};
        ctx->last_kernel = names[nw];
#define SDNR_ASYNC_P(N_, H_, P_)                                                             \
    do {                                                                                     \
        constexpr bool kSpecOk = N_ == 4;              /* the k=48 headline's regime */      \
        auto k = spec && kSpecOk ? async_pick<N_, H_, P_, kSpecOk>(c16, pair, dw)            \
                                 : async_pick<N_, H_, P_, false>(c16, pair, dw);             \
        allow_full_lds(k);                                                                   \
        hipLaunchKernelGGL(k, dim3(cgrid), dim3(N_ * 64), cl, ctx->stream, V, ctx->adj16,    \
                           preswz ? rw : ctx->radj16, ctx->deg32, ctx->row_ptr,              \
                           ctx->port, ctx->W, ctx->ell_port, d_src, nsrc,                    \
                           P_ ? reinterpret_cast<int32_t *>(d_tree) : d_parent, d_port,      \
                           d_hops, err, aflags);                                             \
    } while (0)
#define SDNR_ASYNC(N_, H_) SDNR_ASYNC_P(N_, H_, false)
        if (packed) {
            static const char *pnames[] = {"", "", "dfs_async_kernel<2,packed>",
                                           "dfs_async_kernel<3,packed>",
                                           "dfs_async_kernel<4,packed>",
                                           "dfs_async_kernel<5,packed>",
                                           "dfs_async_kernel<6,packed>", "",
                                           "dfs_async_kernel<8,packed>"};
            ctx->last_kernel = pnames[nw];
            if (hops) {                          // the drop-in's pool: tree words + depth
                static const char *hnames[] = {"", "", "", "dfs_async_kernel<3,packed,hops>",
                                               "dfs_async_kernel<4,packed,hops>", "",
                                               "dfs_async_kernel<6,packed,hops>"};
                const int hw = nw <= 3 ? 3 : (nw >= 6 ? 6 : 4);
                ctx->last_kernel = hnames[hw];
                if (hw == 3) SDNR_ASYNC_P(3, true, true);
                else if (hw == 6) SDNR_ASYNC_P(6, true, true);
                else SDNR_ASYNC_P(4, true, true);
            } else if (nw == 2) SDNR_ASYNC_P(2, false, true);
            else if (nw == 3) SDNR_ASYNC_P(3, false, true);
            else if (nw == 5) SDNR_ASYNC_P(5, false, true);
            else if (nw == 6) SDNR_ASYNC_P(6, false, true);
            else if (nw == 8) SDNR_ASYNC_P(8, false, true);
            else SDNR_ASYNC_P(4, false, true);
        } else if (nw == 2) {
            if (hops) SDNR_ASYNC(2, true); else SDNR_ASYNC(2, false);
        } else if (nw == 3) {
            if (hops) SDNR_ASYNC(3, true); else SDNR_ASYNC(3, false);
        } else if (nw == 5) {
            if (hops) SDNR_ASYNC(5, true); else SDNR_ASYNC(5, false);
        } else if (nw == 6) {
            if (hops) SDNR_ASYNC(6, true); else SDNR_ASYNC(6, false);
        } else if (nw == 8) {
            if (hops) SDNR_ASYNC(8, true); else SDNR_ASYNC(8, false);
        } else {
            if (hops) SDNR_ASYNC(4, true); else SDNR_ASYNC(4, false);
        }
#undef SDNR_ASYNC
#undef SDNR_ASYNC_P
    } else if (count) {
        const size_t cl = dfs_lds_bytes_count(V, hops);
        size_t cpc = SDNR_LDS_PER_CU / cl;
        if (cpc > 8) cpc = 8;
        if (cpc < 1) cpc = 1;
        int cgrid = (int)((size_t)ctx->num_cus * cpc);
        if (cgrid > nsrc) cgrid = nsrc;
        const int nw = dfs_count_waves();
        ctx->last_kernel = nw == 2 ? "dfs_count_kernel<2>" : nw == 6 ? "dfs_count_kernel<6>"
                                                                    : "dfs_count_kernel<4>";
#define SDNR_COUNT(N_, H_)                                                                   \
    do {                                                                                     \
        auto k = dfs_count_kernel<N_, H_>;                                                   \
        allow_full_lds(k);                                                                   \
        hipLaunchKernelGGL(k, dim3(cgrid), dim3(N_ * 64), cl, ctx->stream, V, ctx->adj16,    \
                           ctx->radj16, ctx->deg32, ctx->row_ptr, ctx->port, d_src, nsrc,     \
                           d_parent, d_port, d_hops);                                        \
    } while (0)
        if (nw == 2) {
            if (hops) SDNR_COUNT(2, true); else SDNR_COUNT(2, false);
        } else if (nw == 6) {
            if (hops) SDNR_COUNT(6, true); else SDNR_COUNT(6, false);
        } else {
            if (hops) SDNR_COUNT(4, true); else SDNR_COUNT(4, false);
        }
#undef SDNR_COUNT
    } else if (coop) {
        const size_t cl = dfs_lds_bytes_coop(V);
        size_t cpc = SDNR_LDS_PER_CU / cl;
        if (cpc > 8) cpc = 8;
        if (cpc < 1) cpc = 1;
        int cgrid = (int)((size_t)ctx->num_cus * cpc);
        if (cgrid > nsrc) cgrid = nsrc;
        const int kw = dfs_coop_kw();
        ctx->last_kernel = "dfs_coop_kernel";
        if (hops) launch_coop<true>(kw, cgrid, cl, ctx->stream, V, ctx->adj16, a);
        else launch_coop<false>(kw, cgrid, cl, ctx->stream, V, ctx->adj16, a);
    } else if (!small && ell && ctx->W <= 32 && packed_ok()) {
        // lanes per row = next power of two >= W
        const int lpr = ctx->W <= 8 ? 8 : (ctx->W <= 16 ? 16 : 32);
        const int ring = packed_ring(V, ctx->W);
        const size_t plds = dfs_lds_bytes_global(V, ring);
        size_t pbpc = SDNR_LDS_PER_CU / plds;
        if (pbpc > 32) pbpc = 32;                // 32 one-wave blocks fill a CU
        if (pbpc < 1) pbpc = 1;
        int pgrid = (int)((size_t)ctx->num_cus * pbpc);
        if (pgrid > nsrc) pgrid = nsrc;
        if (pgrid > grid) {                      // spill area: V entries per block
            int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes,
                                  (size_t)pgrid * (size_t)V * sizeof(uint2));
            if (rc) return rc;
            spill = static_cast<uint2 *>(ctx->scratch);
        }
        ctx->last_kernel = ring == 128 ? "dfs_global_packed_kernel<ring128>"
                                       : "dfs_global_packed_kernel";
#define SDNR_PACKED(L_, J_, H_, R_)                                                          \
    do {                                                                                     \
        auto k = dfs_global_packed_kernel<L_, J_, H_, R_>;                                   \
        allow_full_lds(k);                                                                   \
        hipLaunchKernelGGL(k, dim3(pgrid), dim3(64), plds, ctx->stream, V, ctx->W,           \
                           ctx->ell_col, ctx->ell_port, d_src, nsrc, d_parent, d_port,       \
                           d_hops, spill);                                                   \
    } while (0)
#define SDNR_PACKED_R(L_, J_, H_)                                                            \
    do {                                                                                     \
        if (ring == 128) SDNR_PACKED(L_, J_, H_, 128); else SDNR_PACKED(L_, J_, H_, 1024);   \
    } while (0)
        if (lpr == 8 && packed_j8(V) == 1) {
            if (hops) SDNR_PACKED_R(8, 1, true); else SDNR_PACKED_R(8, 1, false);
        } else if (lpr == 8) {
            if (hops) SDNR_PACKED_R(8, 2, true); else SDNR_PACKED_R(8, 2, false);
        } else if (lpr == 16) {
            if (hops) SDNR_PACKED_R(16, 4, true); else SDNR_PACKED_R(16, 4, false);
        } else {
            if (hops) SDNR_PACKED_R(32, 8, true); else SDNR_PACKED_R(32, 8, false);
        }
#undef SDNR_PACKED_R
#undef SDNR_PACKED
    } else if (narrow) {
        const int K = dfs_batch_depth(ctx);
        ctx->last_kernel = small ? "dfs_lds_batch_kernel" : "dfs_global_batch_kernel";
        if (ell && hops) launch_batch_k<true, true>(K, small, grid, lds, ctx->stream, a);
        else if (ell) launch_batch_k<true, false>(K, small, grid, lds, ctx->stream, a);
        else if (hops) launch_batch_k<false, true>(K, small, grid, lds, ctx->stream, a);
        else launch_batch_k<false, false>(K, small, grid, lds, ctx->stream, a);
    } else {
        ctx->last_kernel = small ? "dfs_lds_wide_kernel" : "dfs_global_wide_kernel";
        if (hops) launch_wide<true>(small, grid, lds, ctx->stream, a);
        else launch_wide<false>(small, grid, lds, ctx->stream, a);
    }
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
