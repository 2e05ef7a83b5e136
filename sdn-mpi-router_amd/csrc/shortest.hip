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
#include <stdlib.h>
#include <string.h>

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

// one BFS level for every batch; masks [nbatch][V] in global memory.  A
// vertex every destination of its batch has already reached is skipped (no
// neighbour gather); ELL rows (W > 0) are read with W independent loads.
__global__ __launch_bounds__(256) void msbfs_level_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ ell_col, int ndst, int lvl, const uint64_t *__restrict__ front,
    uint64_t *__restrict__ next, uint64_t *__restrict__ vis, uint16_t *__restrict__ dist,
    int *__restrict__ changed)
{
    const int x0 = blockIdx.x * blockDim.x + threadIdx.x;
    const int batch = blockIdx.y;
    // every lane stays to the end (the distance stores below are a wave-wide
    // loop); lanes past V work on vertex V-1 and store nothing
    const bool live = x0 < V;
    const int x = live ? x0 : V - 1;
    const size_t off = (size_t)batch * V;
    const int nb = min(64, ndst - batch * 64);
    const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    const uint64_t vx = vis[off + x];
    uint64_t acc = 0;
    if (!live || (vx & all) == all) {         // nothing left to reach at x
        acc = 0;
    } else if (W > 0) {
        const int32_t *r = ell_col + (size_t)x * W;
        for (int j = 0; j < W; ++j) {
            const int n = r[j];
            if (n >= 0) acc |= front[off + n];
        }
    } else {
        const int re = row_ptr[x + 1];
        for (int e = row_ptr[x]; e < re; ++e) acc |= front[off + col[e]];
    }
    const uint64_t nw = live ? acc & ~vx : 0ull;
    if (live) next[off + x] = nw;
    if (nw) {
        vis[off + x] = vx | nw;
        *changed = 1;
    }
    // distances: iterate the destinations any lane of the wave reached, so
    // each store instruction writes one destination row at consecutive x
    // (coalesced) instead of every lane walking its own bits
    uint32_t lo = (uint32_t)nw, hi = (uint32_t)(nw >> 32);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o);
        hi |= (uint32_t)__shfl_xor((int)hi, o);
    }
    uint64_t any = ((uint64_t)hi << 32) | lo;
    const int b0 = batch * 64;
    while (any) {
        const int b = __ffsll((unsigned long long)any) - 1;
        any &= any - 1;
        if (((nw >> b) & 1ull) && b0 + b < ndst) dist[(size_t)(b0 + b) * V + x] = (uint16_t)lvl;
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

// nh/nh_port of whole destination rows, one 1024-thread workgroup per row:
// the row's distances are staged in LDS once (V <= 32768) and every vertex
// tests its W ELL neighbours with independent loads, keeping the first (=
// smallest dpid) one hop closer.
__global__ __launch_bounds__(1024) void nexthop_kernel(
    int V, int W, int ndst, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ col, const int32_t *__restrict__ port,
    const int32_t *__restrict__ ell_col, const int32_t *__restrict__ ell_port,
    const uint16_t *__restrict__ dist, int32_t *__restrict__ nh,
    int32_t *__restrict__ nh_port, int stage)
{
    extern __shared__ __attribute__((aligned(16))) uint16_t ldist[];
    for (int rowi = blockIdx.x; rowi < ndst; rowi += gridDim.x) {
        const size_t row = (size_t)rowi * V;
        const uint16_t *drow = dist + row;
        if (stage) {
            __syncthreads();                     // previous row's readers are done
            for (int x = threadIdx.x; x < V; x += blockDim.x) ldist[x] = drow[x];
            __syncthreads();
            drow = ldist;
        }
        for (int x = threadIdx.x; x < V; x += blockDim.x) {
            const uint32_t dx = drow[x];
            int best = -1, bport = -1;
            if (dx != 0xFFFFu && dx != 0u) {
                if (W > 0) {
                    const int32_t *r = ell_col + (size_t)x * W;
                    int bj = -1;
                    for (int j = W - 1; j >= 0; --j) {   // no early exit: loads overlap
                        const int n = r[j];
                        if (n >= 0 && (uint32_t)drow[n] + 1u == dx) {
                            best = n;
                            bj = j;
                        }
                    }
                    if (bj >= 0) bport = ell_port[(size_t)x * W + bj];
                } else {
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
            }
            nh[row + x] = best;
            nh_port[row + x] = bport;
        }
    }
}

// ---------------------------------------------------------------------------
// Per-destination BFS with fused next-hop extraction (V < 65534, in- and
// out-degree <= 64 -- the k=48 fat-tree and dragonfly shapes).
//
// msbfs packs 64 destinations per mask word, which leaves ndst/64 workgroups
// (18 for the 1,152 k=48 edge switches), each sweeping every edge per level.
// Here one workgroup owns one destination d and loads each vertex's row once:
// dist(., d) lives in LDS (u32, bank-swizzled), the frontier of level L is a
// contiguous range of an LDS queue (every vertex enters once), and expanding
// y loads y's in-row (u16, stride 64: one 128-byte line), gathers the
// in-neighbours' levels, claims the unseen ones for level L+1 with
// ds_cmpswap and appends them with one queue-tail atomic per batch of rows
// (ballot + mbcnt order the slots).  On a symmetric graph the same row is
// y's out-row and its level-(L-1) entries are final, so y's next hop -- the
// smallest out-neighbour one hop closer, the reference's lexicographic
// tie-break -- is the lowest lane of a second ballot over the row already in
// registers; asymmetric graphs run one pass over the out-rows afterwards.
// The tables are written once per destination, coalesced.
// ---------------------------------------------------------------------------
constexpr uint32_t kUnseen = 0xFFFFu;           // == SDNR_DIST_INF
constexpr uint32_t kSentLevel = 0xFFFEu;        // level of the padding vertex V

// LDS words of bfs_dest_kernel: lvl u32 [256-blocks], queue u16, nh u16,
// nh slot u8, 4 control words
__host__ __device__ inline int bfs_dest_qwords(int V) { return ((V + 1) / 2 + 3) & ~3; }
__host__ __device__ inline int bfs_dest_words(int V)
{
    return ((V + 1 + 255) & ~255) + 2 * bfs_dest_qwords(V) + (((V + 3) / 4 + 3) & ~3) + 8;
}

template <int NW, int G, bool SYM>
__global__ __launch_bounds__(NW * 64) void bfs_dest_kernel(
    int V, int W, const uint16_t *__restrict__ adj, const uint16_t *__restrict__ radj,
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ port,
    const int32_t *__restrict__ ell_port, const int32_t *__restrict__ dst, int ndst,
    uint16_t *__restrict__ out_dist, int32_t *__restrict__ out_nh,
    int32_t *__restrict__ out_nh_port)
{
    constexpr int U = 4;                         // flush vertices per thread per step
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const int DWp = (V + 1 + 255) & ~255;
    const int QWp = bfs_dest_qwords(V);
    uint32_t *lvl = lds;                                              // lvl[swz(v)]
    uint16_t *q = reinterpret_cast<uint16_t *>(lvl + DWp);            // BFS order
    uint16_t *nhv = reinterpret_cast<uint16_t *>(lvl + DWp + QWp);    // next hop
    uint8_t *nhs = reinterpret_cast<uint8_t *>(lvl + DWp + 2 * QWp);  // its row slot
    int *ctl = reinterpret_cast<int *>(lds + bfs_dest_words(V) - 8);  // per-wave counts
    const uint16_t *inrow = SYM ? adj : radj;
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    const bool want_nh = out_nh != nullptr;

    for (int di = blockIdx.x; di < ndst; di += gridDim.x) {
        const int d = uniform(dst[di]);
        uint16_t *drow = out_dist + (size_t)di * V;
        int32_t *hrow = want_nh ? out_nh + (size_t)di * V : nullptr;
        int32_t *prow = want_nh ? out_nh_port + (size_t)di * V : nullptr;
        if (d < 0 || d >= V) {                   // unknown destination: empty row
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                drow[v] = (uint16_t)kUnseen;
                if (want_nh) {
                    hrow[v] = -1;
                    prow[v] = -1;
                }
            }
            continue;
        }
        for (int i = threadIdx.x; i <= V; i += blockDim.x)
            lvl[lds_swz(i)] = i == d ? 0u : (i == V ? kSentLevel : kUnseen);
        if (threadIdx.x == 0) q[0] = (uint16_t)d;
        __syncthreads();

        int lo = 0, hi = 1;
        const int slice = ((V + NW * 64 - 1) / (NW * 64)) * 64;   // scan slice per wave
        for (int L = 0; lo < hi; ++L) {
            // ---- expand level L = q[lo, hi): G rows per wave in flight.
            // Unseen in-neighbours take level L+1 with a plain store (every
            // writer stores the same value); no claim round trip, no queue
            // atomic -- the next frontier is collected by the scan below.
            for (int base = lo + w * G; base < hi; base += NW * G) {
                const int n = min(G, hi - base);
                const int mine = lane < n ? (int)q[base + lane] : V;   // past n: sentinel row
                int r[G];
#pragma unroll
                for (int g = 0; g < G; ++g)
                    r[g] = inrow[(size_t)read_lane(mine, g) * 64 + lane];
                uint32_t lv[G];
#pragma unroll
                for (int g = 0; g < G; ++g) lv[g] = lvl[lds_swz(r[g])];
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (lv[g] == kUnseen) lvl[lds_swz(r[g])] = (uint32_t)(L + 1);
                if (SYM && L > 0) {
                    // next hop of each expanded y: the lowest slot one level
                    // closer writes itself (mbcnt on the ballot)
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        if (g < n) {
                            const bool cl = lv[g] == (uint32_t)(L - 1);
                            const uint64_t m = __ballot(cl);
                            if (cl && lanes_below(m) == 0) {
                                const int y = q[base + g];
                                nhv[y] = (uint16_t)r[g];
                                nhs[y] = (uint8_t)lane;
                            }
                        }
                    }
                }
            }
            __syncthreads();                     // level L+1 marked
            // ---- collect level L+1 in ascending vertex order: each wave
            // counts its slice, then writes it after the lower slices
            const int s0 = w * slice, s1 = min(V, s0 + slice);
            int cnt = 0;
            for (int x0 = s0; x0 < s1; x0 += 64) {
                const int x = x0 + lane;
                cnt += __popcll(__ballot(x < s1 && lvl[lds_swz(x)] == (uint32_t)(L + 1)));
            }
            if (lane == 0) ctl[w] = cnt;
            __syncthreads();
            int at = hi, total = 0;
#pragma unroll
            for (int k = 0; k < NW; ++k) {
                const int c = ctl[k];
                at += k < w ? c : 0;
                total += c;
            }
            for (int x0 = s0; x0 < s1; x0 += 64) {
                const int x = x0 + lane;
                const bool hit = x < s1 && lvl[lds_swz(x)] == (uint32_t)(L + 1);
                const uint64_t m = __ballot(hit);
                if (hit) q[at + lanes_below(m)] = (uint16_t)x;
                at += __popcll(m);
            }
            __syncthreads();                     // queue and counts consumed
            lo = hi;
            hi += total;
        }

        if (!SYM && want_nh) {
            // next hop over the out-rows: lowest slot whose level is one less
            for (int base = w * G; base < V; base += NW * G) {
                int r[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int v = base + g < V ? base + g : V;
                    r[g] = adj[(size_t)v * 64 + lane];
                }
                uint32_t lv[G];
#pragma unroll
                for (int g = 0; g < G; ++g) lv[g] = lvl[lds_swz(r[g])];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int v = base + g;
                    if (v < V) {
                        const uint32_t lx = lvl[lds_swz(v)];
                        if (lx != kUnseen && lx != 0u) {
                            const uint64_t m = __ballot(lv[g] + 1u == lx);
                            if (m) {
                                const int sl = __ffsll((unsigned long long)m) - 1;
                                const int nb = read_lane(r[g], sl);
                                if (lane == 0) {
                                    nhv[v] = (uint16_t)nb;
                                    nhs[v] = (uint8_t)sl;
                                }
                            }
                        }
                    }
                }
            }
            __syncthreads();
        }

        // ---- tables: U vertices per thread, port loads in flight together
        for (int v0 = threadIdx.x; v0 < V; v0 += U * blockDim.x) {
            uint32_t lx[U];
            int h[U], sl[U], pt[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                lx[k] = v < V ? lvl[lds_swz(v)] : kUnseen;
                h[k] = -1;
                sl[k] = -1;
                if (want_nh && lx[k] != kUnseen && lx[k] != 0u) {
                    h[k] = nhv[v];
                    sl[k] = nhs[v];
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                pt[k] = -1;
                if (sl[k] >= 0)
                    pt[k] = W > 0 ? ell_port[(size_t)v * W + sl[k]] : port[row_ptr[v] + sl[k]];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                if (v < V) {
                    drow[v] = (uint16_t)lx[k];
                    if (want_nh) {
                        hrow[v] = h[k];
                        prow[v] = pt[k];
                    }
                }
            }
        }
        __syncthreads();
    }
}


// ---------------------------------------------------------------------------
// bfs_dest_lanes_kernel<LPR,NW,G,SYM>: the per-destination BFS for graphs too
// large for bfs_dest_kernel's LDS image (torus 32^3: V = 32,768) with rows of
// at most LPR <= 32 entries.  One workgroup per destination; LDS holds the
// levels (u16), the BFS queue (u16), a claim bitmap and the next-hop row slot
// of every vertex (4 bits if LPR <= 8, else 8).
//  * A row needs only LPR lanes, so one wave instruction expands R = 64/LPR
//    frontier vertices (lane -> row sub = lane/LPR, slot pos = lane%LPR), G
//    such groups in flight per wave.  Symmetric graphs read the compact ELL
//    rows (L2-resident: torus 786 KB instead of 4 MB of 64-wide rows).
//  * An unseen neighbour is claimed with an LDS atomicOr on its bit (exactly
//    one claimant), which sets its level and appends it to the queue (one
//    tail atomic per wave-iteration).
//  * On a symmetric graph the row of a level-L vertex is also its out-row
//    and its level-(L-1) entries are final, so its next hop's slot (the
//    lowest such lane of its group) goes to LDS during the expansion;
//    asymmetric graphs take one pass over the out-rows at the end.
//  * The tables are written once, coalesced: distances from LDS, next hop
//    and port as the row entries at the stored slot.  (Storing the next hops
//    straight to the tables in BFS order scattered 4-byte stores over the
//    rows: 7x write amplification, 185 GB of HBM traffic on the torus.)
// ---------------------------------------------------------------------------
__host__ __device__ constexpr bool lanes_nibble(int LPR) { return LPR <= 8; }

__host__ __device__ inline size_t bfs_lanes_bytes(int V, int LPR)
{
    const size_t lv = (((size_t)V + 1) * 2 + 15) & ~(size_t)15;           // u16 levels [V+1]
    const size_t qb = ((size_t)V * 2 + 15) & ~(size_t)15;                 // u16 queue [V]
    const size_t cb = ((((size_t)V + 1 + 31) / 32) * 4 + 15) & ~(size_t)15;   // claim bits
    const size_t sb = lanes_nibble(LPR) ? ((((size_t)V + 7) / 8) * 4 + 15) & ~(size_t)15
                                        : ((((size_t)V + 3) / 4) * 4 + 15) & ~(size_t)15;
    return lv + qb + cb + sb + 16;
}

template <int LPR, int NW, int G, bool SYM>
__global__ __launch_bounds__(NW * 64) void bfs_dest_lanes_kernel(
    int V, int W, const uint16_t *__restrict__ adj, const uint16_t *__restrict__ radj,
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ port, const int32_t *__restrict__ ell_col,
    const int32_t *__restrict__ ell_port, const int32_t *__restrict__ dst, int ndst,
    uint16_t *__restrict__ out_dist, int32_t *__restrict__ out_nh,
    int32_t *__restrict__ out_nh_port)
{
    constexpr int R = 64 / LPR;
    constexpr bool NIB = lanes_nibble(LPR);
    constexpr int SBITS = NIB ? 4 : 8, SPW = 32 / SBITS;       // slot bits, slots per word
    constexpr uint32_t SNONE = NIB ? 0xFu : 0xFFu;
    constexpr uint16_t kUn = 0xFFFFu, kSent = 0xFFFEu;
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const size_t lvb = (((size_t)V + 1) * 2 + 15) & ~(size_t)15;
    const size_t qbb = ((size_t)V * 2 + 15) & ~(size_t)15;
    const size_t cbb = ((((size_t)V + 1 + 31) / 32) * 4 + 15) & ~(size_t)15;
    const int SW = (V + SPW - 1) / SPW;                         // slot words
    uint8_t *base8 = reinterpret_cast<uint8_t *>(lds);
    uint16_t *lvl = reinterpret_cast<uint16_t *>(base8);
    uint16_t *q = reinterpret_cast<uint16_t *>(base8 + lvb);
    uint32_t *claim = reinterpret_cast<uint32_t *>(base8 + lvb + qbb);
    uint32_t *slotw = reinterpret_cast<uint32_t *>(base8 + lvb + qbb + cbb);
    int *ctl = reinterpret_cast<int *>(slotw + ((SW + 3) & ~3));     // [0] queue tail
    const int CW = (V + 1 + 31) / 32;
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    const int sub = lane / LPR, pos = lane % LPR;
    const uint64_t grp = ((1ull << LPR) - 1ull) << (sub * LPR);
    const bool want_nh = out_nh != nullptr;
    const bool ell = SYM && W > 0;

    // row entry pos of vertex y (y == V: the sentinel row); padding -> V
    auto row_in = [&](int y) -> int {
        if (ell) {
            const int e = (pos < W && y < V) ? ell_col[(size_t)y * W + pos] : -1;
            return e < 0 ? V : e;
        }
        return (int)(SYM ? adj : radj)[(size_t)y * 64 + pos];
    };
    auto set_slot = [&](int y, int sl) {     // slot of y: clear the bits not in sl
        const int sh = (y % SPW) * SBITS;
        atomicAnd(&slotw[y / SPW], ~((SNONE & ~(uint32_t)sl) << sh));
    };

    for (int di = blockIdx.x; di < ndst; di += gridDim.x) {
        const int d = uniform(dst[di]);
        uint16_t *drow = out_dist + (size_t)di * V;
        int32_t *hrow = want_nh ? out_nh + (size_t)di * V : nullptr;
        int32_t *prow = want_nh ? out_nh_port + (size_t)di * V : nullptr;
        if (d < 0 || d >= V) {                   // unknown destination: empty row
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                drow[v] = kUn;
                if (want_nh) {
                    hrow[v] = -1;
                    prow[v] = -1;
                }
            }
            continue;
        }
        for (int i = threadIdx.x; i <= V; i += blockDim.x)
            lvl[i] = i == d ? (uint16_t)0 : (i == V ? kSent : kUn);
        for (int i = threadIdx.x; i < CW; i += blockDim.x) claim[i] = 0u;
        for (int i = threadIdx.x; i < SW; i += blockDim.x) slotw[i] = 0xFFFFFFFFu;
        __syncthreads();
        if (threadIdx.x == 0) {
            claim[d >> 5] |= 1u << (d & 31);
            claim[V >> 5] |= 1u << (V & 31);
            q[0] = (uint16_t)d;
            ctl[0] = 1;
        }
        __syncthreads();

        int lo = 0, hi = 1;
        for (int L = 0; lo < hi; ++L) {
            for (int base = lo + w * (R * G); base < hi; base += NW * R * G) {
                int y[G], r[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int idx = base + g * R + sub;
                    y[g] = idx < hi ? (int)q[idx] : V;         // past hi: sentinel row
                }
#pragma unroll
                for (int g = 0; g < G; ++g) r[g] = row_in(y[g]);
                uint32_t lv[G];
#pragma unroll
                for (int g = 0; g < G; ++g) lv[g] = lvl[r[g]];
                bool won[G];
                int nwon = 0;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    won[g] = false;
                    if (lv[g] == kUn) {
                        const uint32_t bit = 1u << (r[g] & 31);
                        won[g] = (atomicOr(&claim[r[g] >> 5], bit) & bit) == 0u;
                    }
                    nwon += __popcll(__ballot(won[g]));
                }
                if (nwon) {
                    int at = 0;
                    if (lane == 0) at = atomicAdd(&ctl[0], nwon);
                    at = read_lane(at, 0);
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        const uint64_t m = __ballot(won[g]);
                        if (won[g]) {
                            lvl[r[g]] = (uint16_t)(L + 1);
                            q[at + lanes_below(m)] = (uint16_t)r[g];
                        }
                        at += __popcll(m);
                    }
                }
                if (SYM && want_nh && L > 0) {
#pragma unroll
                    for (int g = 0; g < G; ++g) {
                        const bool cl = lv[g] == (uint32_t)(L - 1);
                        const uint64_t m = __ballot(cl) & grp;
                        if (cl && lanes_below(m) == 0 && y[g] < V) set_slot(y[g], pos);
                    }
                }
            }
            __syncthreads();                     // level L+1 claimed and queued
            lo = hi;
            hi = ctl[0];
            __syncthreads();                     // every wave has read the tail
        }

        if (!SYM && want_nh) {
            // next hop over the out-rows: lowest slot whose level is one less
            for (int base = w * (R * G); base < V; base += NW * R * G) {
                int r[G];
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int v = base + g * R + sub;
                    if (W > 0) {
                        const int e = (pos < W && v < V) ? ell_col[(size_t)v * W + pos] : -1;
                        r[g] = e < 0 ? V : e;
                    } else {
                        r[g] = adj[(size_t)(v < V ? v : V) * 64 + pos];
                    }
                }
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    const int v = base + g * R + sub;
                    const uint32_t lx = v < V ? lvl[v] : kUn;
                    const bool cl = lx != kUn && lx != 0u && (uint32_t)lvl[r[g]] + 1u == lx;
                    const uint64_t m = __ballot(cl) & grp;
                    if (cl && lanes_below(m) == 0) set_slot(v, pos);
                }
            }
            __syncthreads();
        }

        // tables once, coalesced; the next hop and its port are the row
        // entries at the stored slot (U vertices per thread, loads in flight
        // together)
        constexpr int U = 4;
        for (int v0 = threadIdx.x; v0 < V; v0 += U * (int)blockDim.x) {
            int h[U], pt[U], e[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                e[k] = -1;
                if (v < V) {
                    const uint16_t lx = lvl[v];
                    drow[v] = lx;
                    const uint32_t sl = (slotw[v / SPW] >> ((v % SPW) * SBITS)) & SNONE;
                    if (want_nh && sl != SNONE && lx != kUn && lx != 0)
                        e[k] = W > 0 ? v * W + (int)sl : row_ptr[v] + (int)sl;
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                h[k] = -1;
                pt[k] = -1;
                if (e[k] >= 0) {
                    h[k] = W > 0 ? ell_col[e[k]] : col[e[k]];
                    pt[k] = W > 0 ? ell_port[e[k]] : port[e[k]];
                }
            }
            if (want_nh) {
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int v = v0 + k * (int)blockDim.x;
                    if (v < V) {
                        hrow[v] = h[k];
                        prow[v] = pt[k];
                    }
                }
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Bit-plane multi-destination BFS with fused next hops (large V: Jellyfish
// 100k, where neither per-destination kernel's LDS state fits).
//
// msbfs_level_kernel + nexthop_kernel spend most of their time in the next
// hop pass: every (destination, vertex) gathers the distances of its W
// neighbours again (1.6e11 gathers for all Jellyfish pairs).  The pull step
// already has what it needs: x joins level L+1 of destination b through the
// first (smallest id = smallest slot, the reference's lexicographic
// tie-break) out-neighbour whose level-L frontier word holds bit b.  So the
// level kernel, walking x's ELL row in slot order, assigns each newly
// reached bit the slot that first supplied it and accumulates, per (batch,
// vertex), bit-sliced planes: 8 planes of the level (L < 256) and
// ceil(log2 W) planes of the slot, next to the visited / frontier words.
// The tables are then written once, coalesced, by a pass that decodes the
// planes for the 64 destinations of a word (dist, nh = row[slot],
// nh_port = port row[slot]).  Destinations run in chunks of 64-destination
// batches so the scratch stays bounded.
// ---------------------------------------------------------------------------
constexpr int kPlVis = 0, kPlFront = 1, kPlNext = 2, kPlDist = 3, kPlSlot = 11;
// planes per batch: vis, front, next, 8 level, SB slot planes (SB =
// ceil(log2 W)); 16 (a 4 MiB batch stride on the torus) up to SB = 5
__host__ __device__ constexpr int plane_count(int sb) { return sb <= 5 ? 16 : kPlSlot + sb; }
// DP: level planes.  8 (levels < 256), or 3 when the BFS is known to end by
// level 7 (the previous call's depth): planes [vis, front, next, 3 level,
// sb slot] -- k=48 12 planes instead of 17, so the init writes, the table
// pass reads and the chunks' footprint shrink with them
__host__ __device__ constexpr int plane_count_dp(int sb, int dp) { return dp == 8 ? plane_count(sb) : 3 + dp + sb; }

__global__ __launch_bounds__(256) void msbfs_plane_seed_kernel(
    int V, int VS, const int32_t *__restrict__ dst, int ndst, uint64_t *__restrict__ pl, int npl,
    int *__restrict__ full)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ndst) return;
    const int d = dst[i];
    if (d < 0 || d >= V) return;
    uint64_t *b = pl + (size_t)(i >> 6) * npl * VS;
    atomicOr((unsigned long long *)&b[(size_t)kPlVis * VS + d], 1ull << (i & 63));
    atomicOr((unsigned long long *)&b[(size_t)kPlFront * VS + d], 1ull << (i & 63));
    // a batch whose destinations are all d (one destination, or repeats)
    // has its (batch, d) word complete already
    if ((i & 63) == 0) {
        bool same = true;
        for (int k = i + 1; same && k < min(ndst, i + 64); ++k) same = dst[k] == d;
        if (same) atomicAdd(full, 1);
    }
}

// the planes of a chunk zeroed, the destinations seeded into the visited and
// frontier planes, the level flags and status words reset -- one launch in
// place of two fills and the seed kernel.  Thread (batch, x) writes column x
// (pad words included) of every plane of its batch.
__global__ __launch_bounds__(256) void msbfs_plane_init_kernel(
    int V, int VS, const int32_t *__restrict__ dst, int ndst, uint64_t *__restrict__ pl, int npl,
    int *__restrict__ flags, int nflags, int *__restrict__ status)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int batch = blockIdx.y;
    const int nb = min(64, ndst - batch * 64);
    const int lane = lane_id();
    const int mine = lane < nb ? dst[batch * 64 + lane] : -1;
    // the batch's id range (wave reductions): a wave outside it skips the
    // 64-step match (destination lists are usually runs of ids)
    int lo = mine >= 0 ? mine : 0x7FFFFFFF, hi = mine;
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    uint64_t seed = 0ull;
    if (x >= lo && x <= hi && x < V)
        for (int k = 0; k < nb; ++k)
            if (__builtin_amdgcn_readlane(mine, k) == x) seed |= 1ull << k;
    if (x < VS) {
        uint64_t *b = pl + (size_t)batch * npl * VS + x;
        for (int p = 0; p < npl; ++p)
            b[(size_t)p * VS] = (p == kPlVis || p == kPlFront) ? seed : 0ull;
    }
    if (batch == 0 && blockIdx.x == 0) {
        for (int i = threadIdx.x; i < nflags; i += blockDim.x) flags[i] = 0;
        __syncthreads();
        // words complete from the start: a batch whose destinations are all
        // one valid vertex d (a last batch of one destination, or repeats)
        // has its (batch, d) word complete before level 1, and the level
        // pass counts only words that become complete -- count these here,
        // behind the reset, so the count still reaches V x batches
        const int nbatch = (ndst + 63) >> 6;
        int seeded = 0;
        for (int bt = threadIdx.x; bt < nbatch; bt += blockDim.x) {
            const int n0 = bt * 64, n1 = min(ndst, n0 + 64);
            const int d = dst[n0];
            bool same = d >= 0 && d < V;
            for (int i = n0 + 1; same && i < n1; ++i) same = dst[i] == d;
            seeded += same;
        }
        if (seeded) atomicAdd(&status[0], seeded);
    }
}

// The init kernel with level 1 folded in.  Level 1
// needs no frontier plane: vertex x is reached at level 1 by destination bit
// b exactly when one of its out-neighbours IS destination b, and the bit takes
// the first such slot (the level kernel's lexicographic rule).  So thread
// (batch, x) computes the seed words of its row's neighbours from the batch's
// destination list itself -- an index test when the batch is an ascending run
// of ids (every benched destination set), else the 64-lane match -- and
// writes the planes as they stand after level 1: visited = seed | new,
// frontier = seed, next = new, level plane 0 = new, slot planes.  The level
// flags and complete-word counters must be zero before it runs (the host
// clears them: this kernel's blocks add into them), and the host starts the
// level sequence at 2.
template <int SB, int DP>
__global__ __launch_bounds__(256) void msbfs_plane_init1_kernel(
    int V, int VS, int W, const int32_t *__restrict__ ell_col, const int32_t *__restrict__ dst,
    int ndst, uint64_t *__restrict__ pl, int *__restrict__ flags, int *__restrict__ status)
{
    constexpr int NPL = plane_count_dp(SB, DP);
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int batch = blockIdx.y;
    const int nb = min(64, ndst - batch * 64);
    const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    const int lane = lane_id();
    const int mine = lane < nb ? dst[batch * 64 + lane] : -1;
    int lo = (lane < nb && mine >= 0 && mine < V) ? mine : 0x7FFFFFFF;
    int hi = lane < nb ? mine : -1;
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    // an ascending run lo, lo + 1, ..., lo + nb - 1 of valid ids
    // (lo is wave-uniform: the ballot runs on every lane or on none)
    const bool run = lo <= V - nb && __ballot(lane < nb && mine != lo + lane) == 0ull;
    auto seed_of = [&](int v) -> uint64_t {
        if (v < lo || v > hi || v >= V) return 0ull;
        if (run) return 1ull << (v - lo);
        uint64_t s = 0ull;
        for (int k = 0; k < nb; ++k)
            if (__builtin_amdgcn_readlane(mine, k) == v) s |= 1ull << k;
        return s;
    };
    uint64_t seed = 0ull, nw = 0ull, rem = 0ull, sp[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) sp[k] = 0ull;
    if (x < V) {
        seed = seed_of(x);
        if ((seed & all) != all) {
            constexpr int WM = 1 << SB;
            const int32_t *r = ell_col + (size_t)x * W;
            int n[WM];
#pragma unroll
            for (int j = 0; j < WM; ++j) n[j] = j < W ? r[j] : -1;
            rem = ~seed & all;
#pragma unroll
            for (int j = 0; j < WM; ++j) {
                if (j < W && n[j] >= 0) {
                    const uint64_t h = seed_of(n[j]) & rem;
                    rem &= ~h;
#pragma unroll
                    for (int k = 0; k < SB; ++k)
                        if ((j >> k) & 1) sp[k] |= h;
                }
            }
            nw = (~seed & all) & ~rem;
        }
    }
    if (x < VS) {
        uint64_t *b = pl + (size_t)batch * NPL * VS + x;
#pragma unroll
        for (int p = 0; p < NPL; ++p) {
            uint64_t w = 0ull;
            if (p == kPlVis) w = seed | nw;
            else if (p == kPlFront) w = seed;
            else if (p == kPlNext || p == kPlDist) w = nw;
            else if (p >= kPlDist + DP && p < kPlDist + DP + SB) w = sp[p - kPlDist - DP];
            b[(size_t)p * VS] = w;
        }
    }
    {
        const uint64_t act = __ballot(true);
        const uint64_t fm = __ballot(nw != 0ull && rem == 0ull), am = __ballot(nw != 0ull);
        if (lane == __builtin_ctzll(act)) {
            if (fm) atomicAdd(&status[16 * (blockIdx.x & 15)], __popcll(fm));
            if (am && flags[1] == 0) flags[1] = 1;   // racing writers all store 1
        }
    }
    if (batch == 0 && blockIdx.x == 0) {
        // words complete from the start (a batch of one repeated valid
        // destination), as msbfs_plane_init_kernel counts them
        const int nbatch = (ndst + 63) >> 6;
        int seeded = 0;
        for (int bt = threadIdx.x; bt < nbatch; bt += blockDim.x) {
            const int n0 = bt * 64, n1 = min(ndst, n0 + 64);
            const int d = dst[n0];
            bool same = d >= 0 && d < V;
            for (int i = n0 + 1; same && i < n1; ++i) same = dst[i] == d;
            seeded += same;
        }
        if (seeded) atomicAdd(&status[0], seeded);
    }
}

// A busy level is a chain of dependent L2 round trips per thread -- visited
// word, row, frontier gathers, then a read-modify-write of the level / slot
// planes.  opt kPlAtomicOr: the plane updates are return-less atomic ORs
// performed in L2 (each (batch, x) word has one writer), so the wave does not
// wait for the old plane values -- 3.5 % off the k=48 and dragonfly steps,
// 7 % slower on the torus, so small graphs only.  (Row loads
// issued beside the visited load were slower on every fabric.)
constexpr int kPlAtomicOr = 2;

// flags[lvl]: level lvl reached something.  status[16 k], k < 16: (batch,
// vertex) words with every destination bit set, counted over 16 words 64 B
// apart -- the BFS is complete when their sum reaches V x batches, so no
// empty level is launched to find out.  Both are hot words: one update per
// wave (the flag only while it is still 0), the count spread over the 16
// (a per-wave store and atomic on two single hot words cost the 32^3 torus
// 12 -> 33 ms; a per-workgroup update behind a barrier 14.7 ms)
constexpr int kStatusWords = 256;
template <int SB, int DP>
__global__ __launch_bounds__(256) void msbfs_plane_level_kernel(
    int V, int VS, int W, const int32_t *__restrict__ ell_col, int ndst, int nbatch, int vpb,
    int lvl, int flip, uint64_t *__restrict__ pl, int *changed, int opt, int *__restrict__ status)
{
    // a block covers vpb vertices of blockDim / vpb batches: with vpb = 64
    // its waves read the same 64 rows (one wave per batch), so the row
    // loads after the first hit the CU's L1
    const int x = blockIdx.x * vpb + (int)threadIdx.x % vpb;
    const int batch = blockIdx.y * ((int)blockDim.x / vpb) + (int)threadIdx.x / vpb;
    if (batch >= nbatch) return;
    // levels are queued ahead of the host's termination check: a level
    // after one that reached nothing has nothing to do
    if (lvl > 1 && __hip_atomic_load(&changed[lvl - 1], __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    if (x >= V) return;
    uint64_t *b = pl + (size_t)batch * plane_count_dp(SB, DP) * VS;
    const uint64_t *front = b + (size_t)(flip ? kPlNext : kPlFront) * VS;
    uint64_t *next = b + (size_t)(flip ? kPlFront : kPlNext) * VS;
    const int nb = min(64, ndst - batch * 64);
    const uint64_t all = nb == 64 ? ~0ull : ((1ull << nb) - 1ull);
    const uint64_t vx = b[(size_t)kPlVis * VS + x];
    if ((vx & all) == all) {                   // every destination reached x already
        next[x] = 0ull;
        return;
    }
    // slot order = ascending neighbour id: a bit takes the first slot whose
    // frontier word has it; W independent loads in flight
    constexpr int WM = 1 << SB;                // row slots this instance handles
    const int32_t *r = ell_col + (size_t)x * W;
    uint64_t f[WM];
#pragma unroll
    for (int j = 0; j < WM; ++j) {
        if (j < W) {
            // [vertex][slot] rows: a transposed u16 copy (coalesced along x)
            // measured slower, k=48 0.110 -> 0.112 ms, dragonfly 0.104 -> 0.111
            const int n = r[j];
            f[j] = n >= 0 ? front[n] : 0ull;
        }
    }
    uint64_t rem = ~vx & all, sp[SB];
#pragma unroll
    for (int k = 0; k < SB; ++k) sp[k] = 0ull;
#pragma unroll
    for (int j = 0; j < WM; ++j) {
        if (j < W) {
            const uint64_t h = f[j] & rem;
            rem &= ~h;
#pragma unroll
            for (int k = 0; k < SB; ++k)
                if ((j >> k) & 1) sp[k] |= h;
        }
    }
    const uint64_t nw = (~vx & all) & ~rem;    // bits reached at this level
    next[x] = nw;
    {
        const uint64_t act = __ballot(true);
        const uint64_t fm = __ballot(nw != 0ull && rem == 0ull), am = __ballot(nw != 0ull);
        if (lane_id() == __builtin_ctzll(act)) {
            if (fm) atomicAdd(&status[16 * (blockIdx.x & 15)], __popcll(fm));
            if (am && changed[lvl] == 0) changed[lvl] = 1;   // racing writers all store 1
        }
    }
    if (nw) {
        b[(size_t)kPlVis * VS + x] = vx | nw;
        if (opt & kPlAtomicOr) {
#pragma unroll
            for (int k = 0; k < DP; ++k)
                if ((lvl >> k) & 1)
                    atomicOr((unsigned long long *)&b[(size_t)(kPlDist + k) * VS + x], nw);
#pragma unroll
            for (int k = 0; k < SB; ++k)
                if (sp[k]) atomicOr((unsigned long long *)&b[(size_t)(kPlDist + DP + k) * VS + x], sp[k]);
        } else {
#pragma unroll
            for (int k = 0; k < DP; ++k)
                if ((lvl >> k) & 1) b[(size_t)(kPlDist + k) * VS + x] |= nw;
#pragma unroll
            for (int k = 0; k < SB; ++k)
                if (sp[k]) b[(size_t)(kPlDist + DP + k) * VS + x] |= sp[k];
        }
    }
}

// decode the planes of one batch into 64 table rows, coalesced along x; the
// block's ELL rows (neighbour ids and ports, 256 vertices) are staged in LDS
// once, transposed to [slot][vertex] so the per-destination lookups of a
// wave hit 32 different banks, instead of two scattered global loads per
// (destination, vertex)
template <int SB, int TB, int Q, int DP>
__global__ __launch_bounds__(TB * Q) void msbfs_plane_tables_kernel(
    int V, int VS, int W, const int32_t *__restrict__ ell_col, const int32_t *__restrict__ ell_port,
    int ndst, const uint64_t *__restrict__ pl, uint16_t *__restrict__ dist,
    int32_t *__restrict__ nh, int32_t *__restrict__ nh_port, const int *__restrict__ status,
    int *hpub, int seq)
{
    // the levels before this launch are done (stream order): hand the host
    // (coherent host memory, system scope) the complete-word count and the
    // last level that reached anything (the highest set level flag), then
    // the sequence number -- no copy on the stream between levels and tables
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 64) {
        const int *flags = status - 256;
        int last = 0, done = threadIdx.x < 16 ? status[16 * threadIdx.x] : 0;
        for (int l = threadIdx.x; l < 256; l += 64)
            if (l > 0 && flags[l]) last = l;
        for (int o = 32; o > 0; o >>= 1) {
            last = max(last, __shfl_xor(last, o));
            done += __shfl_xor(done, o);
        }
        if (threadIdx.x == 0) {
            __hip_atomic_store(&hpub[0], done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hpub[1], last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&hpub[3], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // [2][W][kTabStride]: ids, ports; the odd stride keeps the transposing
    // stores below conflict-free (with 256, a wave's 64 stores -- slots j,
    // j+1, ... of one or two vertices -- fell in one or two banks).  TB
    // vertices per block, each decoded by Q threads (64 / Q destinations
    // each): the decode is ~3.5 k VALU instructions per wave for 64
    // destinations, so on small graphs (k=48: 12 x 18 blocks of 256 for 256
    // CUs, one wave per SIMD) 64-vertex blocks with Q = 4 give each SIMD
    // several waves to hide that latency, with no extra row staging
    constexpr int kTabStride = TB + 1;
    extern __shared__ int32_t lrow[];
    const int x0 = blockIdx.x * TB;
    const int t = threadIdx.x % TB;
    const int q = threadIdx.x / TB;
    const int x = x0 + t;
    const int batch = blockIdx.y;
    const int nx = min(TB, V - x0);
    if (nh) {
        for (int e = threadIdx.x; e < nx * W; e += TB * Q) {   // coalesced reads of the rows
            const int xl = e / W, j = e - xl * W;
            lrow[j * kTabStride + xl] = ell_col[(size_t)x0 * W + e];
            lrow[(W + j) * kTabStride + xl] = ell_port[(size_t)x0 * W + e];
        }
        __syncthreads();
    }
    if (x >= V) return;
    const uint64_t *b = pl + (size_t)batch * plane_count_dp(SB, DP) * VS;
    const uint64_t vx = b[(size_t)kPlVis * VS + x];
    uint64_t d[DP], s[SB];
#pragma unroll
    for (int k = 0; k < DP; ++k) d[k] = b[(size_t)(kPlDist + k) * VS + x];
#pragma unroll
    for (int k = 0; k < SB; ++k) s[k] = b[(size_t)(kPlDist + DP + k) * VS + x];
    const int nb = min(64, ndst - batch * 64);
    // 8 destinations at a time: the planes shifted once per group (32-bit
    // bit extracts after that), the group's 16 LDS lookups issued together
    // before its stores, instead of one dependent lookup per destination
    constexpr int CG = 8;
    const int iend = min(nb, (q + 1) * (64 / Q));
    for (int i0 = q * (64 / Q); i0 < iend; i0 += CG) {
        const uint32_t vv = (uint32_t)(vx >> i0);
        uint32_t dv[DP], sv[SB];
#pragma unroll
        for (int k = 0; k < DP; ++k) dv[k] = (uint32_t)(d[k] >> i0);
#pragma unroll
        for (int k = 0; k < SB; ++k) sv[k] = (uint32_t)(s[k] >> i0);
        uint32_t L[CG];
        int best[CG], bport[CG];
#pragma unroll
        for (int u = 0; u < CG; ++u) {
            L[u] = 0xFFFFu;
            best[u] = -1;
            bport[u] = -1;
            if ((vv >> u) & 1u) {
                uint32_t l = 0;
#pragma unroll
                for (int k = 0; k < DP; ++k) l |= ((dv[k] >> u) & 1u) << k;
                L[u] = l;
                if (l && nh) {
                    int sl = 0;
#pragma unroll
                    for (int k = 0; k < SB; ++k) sl |= (int)((sv[k] >> u) & 1u) << k;
                    best[u] = lrow[sl * kTabStride + t];
                    bport[u] = lrow[(W + sl) * kTabStride + t];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < CG; ++u) {
            if (i0 + u < iend) {
                const size_t row = (size_t)(batch * 64 + i0 + u) * V + x;
                dist[row] = (uint16_t)L[u];
                if (nh) {
                    nh[row] = best[u];
                    nh_port[row] = bport[u];
                }
            }
        }
    }
}

}  // namespace

// SDNROUTE_SP_STRATEGY=msbfs|lanes forces the shortest-mode kernel (tests)
// Shortest tables from all-pairs distances (SDNROUTE_SP_STRATEGY=apsp, and
// the default where it measured faster): D = the min-plus APSP of apsp.hip
// (D[a][b] = hops a -> b), then per requested destination d and vertex x
//   dist[i][x] = D[x][d]   (row d of D when every link has its reverse),
//   nh[i][x]   = the smallest out-neighbour n of x with D[n][d] = D[x][d] - 1,
//   nh_port    = links[x][nh].src.port_no,
// the same values as the BFS tables (the lexicographic rule of
// _find_routes_bfs, reference sdnmpi/util/topology_db.py:86-122).  One
// thread per (vertex, destination); the ELL row of x is scanned in slot
// (= ascending id) order.  SYM: read row d of D (coalesced) instead of
// column d.
template <bool SYM>
__global__ __launch_bounds__(256) void sp_from_apsp_kernel(
    int V, int W, const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ port, const int32_t *__restrict__ ell_col,
    const int32_t *__restrict__ ell_port, const uint16_t *__restrict__ D,
    const int32_t *__restrict__ dst, int ndst, uint16_t *__restrict__ dist,
    int32_t *__restrict__ nh, int32_t *__restrict__ nh_port)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = blockIdx.y;
    if (x >= V || i >= ndst) return;
    const int d = dst[i];
    const size_t o = (size_t)i * V + x;
    if (d < 0 || d >= V) {                      // unknown destination: blank row
        dist[o] = 0xFFFF;
        if (nh) {
            nh[o] = -1;
            nh_port[o] = -1;
        }
        return;
    }
    auto at = [&](int a) -> uint32_t {          // hops a -> d
        return SYM ? D[(size_t)d * V + a] : D[(size_t)a * V + d];
    };
    const uint32_t dx = at(x);
    dist[o] = (uint16_t)dx;
    if (!nh) return;
    int best = -1, bp = -1;
    if (dx != 0u && dx != 0xFFFFu) {
        if (W > 0) {
            for (int j = 0; j < W; ++j) {
                const int n = ell_col[(size_t)x * W + j];
                if (n < 0) break;                   // -1 padding ends the row
                if (at(n) == dx - 1u) {
                    best = n;
                    bp = ell_port[(size_t)x * W + j];
                    break;
                }
            }
        } else {
            for (int e = row_ptr[x]; e < row_ptr[x + 1]; ++e)
                if (at(col[e]) == dx - 1u) {
                    best = col[e];
                    bp = port[e];
                    break;
                }
        }
    }
    nh[o] = best;
    nh_port[o] = bp;
}

static int launch_sp_apsp(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst, uint16_t *d_dist,
                          int32_t *d_nh, int32_t *d_nh_port)
{
    const int V = ctx->V;
    // D in its own buffer (the APSP keeps its pass flags in scratch2 and
    // pads into scratch when V is not a multiple of its tile)
    int rc = sdnr_reserve(&ctx->dmat, &ctx->dmat_bytes, (size_t)V * V * sizeof(uint16_t));
    if (rc) return rc;
    uint16_t *D = static_cast<uint16_t *>(ctx->dmat);
    const bool timed = ctx->timed;
    ctx->timed = false;                          // the caller's events bracket both parts
    rc = sdnr_launch_apsp(ctx, D);
    ctx->timed = timed;
    if (rc) return rc;
    const dim3 grid((V + 255) / 256, ndst);
    if (ctx->symmetric)
        hipLaunchKernelGGL(sp_from_apsp_kernel<true>, grid, dim3(256), 0, ctx->stream, V, ctx->W,
                           ctx->row_ptr, ctx->col, ctx->port, ctx->ell_col, ctx->ell_port, D,
                           d_dst, ndst, d_dist, d_nh, d_nh_port);
    else
        hipLaunchKernelGGL(sp_from_apsp_kernel<false>, grid, dim3(256), 0, ctx->stream, V, ctx->W,
                           ctx->row_ptr, ctx->col, ctx->port, ctx->ell_col, ctx->ell_port, D,
                           d_dst, ndst, d_dist, d_nh, d_nh_port);
    SDNR_HIP(hipGetLastError());
    ctx->last_kernel = "apsp+sp_from_apsp_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}

// the APSP route to the shortest tables pays V^2 distances whatever the
// destination count: only worth it for many destinations of a small graph
// (SDNROUTE_SP_APSP=0|1 overrides the measured rule)
static bool sp_apsp_default(const sdnr_ctx *ctx, int32_t ndst)
{
    if (const char *f = sdnr_tune_env("SDNROUTE_SP_APSP")) return !strcmp(f, "1");
    (void)ctx;
    (void)ndst;
    return false;
}

static const char *sp_strategy()
{
    const char *f = getenv("SDNROUTE_SP_STRATEGY");
    return f ? f : "";
}

// bit-plane BFS (msbfs_plane_*): returns 1 (nothing launched that matters,
// tables to be redone) if a BFS is deeper than the 255 levels the planes hold;
// with compact planes (3 level planes), kPlaneDeeper once a BFS runs past
// level 7 (the caller redoes the call with 8)
constexpr int kPlaneDeeper = 3;
static int launch_plane_dp(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst, uint16_t *d_dist,
                           int32_t *d_nh, int32_t *d_nh_port, bool compact)
{
    const int V = ctx->V, W = ctx->W;
    const int sb = W <= 8 ? 3 : W <= 16 ? 4 : W <= 32 ? 5 : 6;
    const int nbatch = (ndst + 63) / 64;
    // plane stride VS = V + 64 words: with a power-of-two stride (torus 32^3:
    // 256 KiB) the 16 plane streams of a vertex block conflict in the memory
    // channels by a pattern set by where the allocation lands -- 11.4 to 14.0
    // ms across fresh allocations in one process; 11.9-12.2 ms with the 512-B
    // pad (tools/bimodal_settings.py).  SDNROUTE_PLANE_PAD
    // overrides the pad (words).
    int VS = V + 64;
    if (const char *f = getenv("SDNROUTE_PLANE_PAD")) {     // words; a stride below V would
        const int pad = atoi(f);                              // overlap the planes
        if (pad >= 0 && pad <= (1 << 16)) VS = V + pad;
    }
    const int npl = plane_count_dp(sb, compact ? 3 : 8);
    const size_t per_batch = (size_t)npl * VS * sizeof(uint64_t);
    // batches per chunk: the planes one level sweeps stay inside the 256 MiB
    // Infinity Cache (measured: torus 32^3 14.9 -> 12.8 ms with 64 batches of
    // 4 MiB instead of all 512 at once; the 100k Jellyfish 127 -> 119 ms)
    int cb = (int)((size_t)(256ull << 20) / per_batch);
    if (const char *f = getenv("SDNROUTE_PLANE_CHUNK")) {   // batches per chunk (tuning)
        const int k = atoi(f);
        if (k > 0) cb = k;
    }
    if (cb < 1) cb = 1;
    if (cb > nbatch) cb = nbatch;
    // equal chunks: a short last chunk costs a whole level sequence
    const int nchunk = (nbatch + cb - 1) / cb;
    cb = (nbatch + nchunk - 1) / nchunk;
    constexpr int kFlagInts = 256 + kStatusWords;   // level flags + 16 spread counters
    int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes,
                          (size_t)cb * per_batch + kFlagInts * sizeof(int) + 256);
    if (rc) return rc;
    uint64_t *pl = static_cast<uint64_t *>(ctx->scratch);
    int *changed = reinterpret_cast<int *>(reinterpret_cast<char *>(ctx->scratch) +
                                           (size_t)cb * per_batch);   // [256] per level
    int *status = changed + 256;                 // complete-word counters (16, 64 B apart)
    const int gx = (V + 255) / 256;
    // level-pass options: kPlAtomicOr up to 16k vertices (k=48, dragonfly);
    // SDNROUTE_PLANE_OPT=0|2 overrides
    int popt = V <= 16384 ? kPlAtomicOr : 0;
    if (const char *f = getenv("SDNROUTE_PLANE_OPT")) popt = atoi(f) & kPlAtomicOr;
    int levels = 0;
    // levels to queue before the first host check: the last level the
    // previous call on this graph needed (k=48: 4), then what the previous
    // chunk needed; the table pass goes out right behind them, before the
    // host waits, so the host round trip overlaps it.  The check reads the
    // complete-word count and the last busy level: the BFS is done when
    // every (batch, vertex) word is complete (no empty level needed) or a
    // level reached nothing.  A guess too small costs more levels and the
    // table pass again.
    const char *gq = getenv("SDNROUTE_PLANE_GUESS");   // 0: check every kGroup levels
    const bool noguess = gq && !strcmp(gq, "0");
    int guess = noguess ? 0 : ctx->plane_depth;
    // SDNROUTE_PLANE_INIT=0: fills + seed kernel instead of the init kernel
    const char *iq = getenv("SDNROUTE_PLANE_INIT");
    const bool oldinit = iq && !strcmp(iq, "0");
    // level 1 folded into the init kernel (msbfs_plane_init1_kernel);
    // SDNROUTE_PLANE_FUSE1=0 keeps the separate level-1 launch
    const char *fq = getenv("SDNROUTE_PLANE_FUSE1");
    const bool fuse1 = !oldinit && !(fq && !strcmp(fq, "0"));
    const size_t tl = d_nh ? (size_t)2 * W * 257 * sizeof(int32_t) : 0;   // kTabStride, TB 256
    if (sb == 5 && tl > 65536) {  // W = 32 with the padded stride
        sdnr_allow_lds(reinterpret_cast<const void *>(msbfs_plane_tables_kernel<5, 256, 1, 8>), tl);
        sdnr_allow_lds(reinterpret_cast<const void *>(msbfs_plane_tables_kernel<5, 256, 1, 3>), tl);
    }
    if (sb == 6) {
        sdnr_allow_lds(reinterpret_cast<const void *>(msbfs_plane_tables_kernel<6, 256, 1, 8>), tl);
        sdnr_allow_lds(reinterpret_cast<const void *>(msbfs_plane_tables_kernel<6, 256, 1, 3>), tl);
    }
    // small launches (fewer 256-vertex blocks than 2 per CU over the whole
    // destination set): 64-vertex blocks, so every CU gets work
    // (SDNROUTE_PLANE_BLOCK=256|64 overrides)
    bool small = (size_t)gx * nbatch < 2 * (size_t)ctx->num_cus;
    if (const char *f = sdnr_tune_env("SDNROUTE_PLANE_BLOCK")) small = atoi(f) == 64;
    const int lb = small ? 64 : 256;
    // level pass: batches per block on small graphs (SDNROUTE_PLANE_BPB=2|4;
    // 4 measured k=48 0.0917 -> 0.0926 ms, dragonfly 0.0625 -> 0.0608 ms)
    int bpb = 1;
    if (const char *f = sdnr_tune_env("SDNROUTE_PLANE_BPB")) {
        const int k = atoi(f);
        if (small && (k == 1 || k == 2 || k == 4)) bpb = k;
    }
    for (int c0 = 0; c0 < nbatch; c0 += cb) {
        const int nbc = nbatch - c0 < cb ? nbatch - c0 : cb;
        const int nd = ndst - c0 * 64 < nbc * 64 ? ndst - c0 * 64 : nbc * 64;
        // a full chunk's planes end where the level flags begin: one fill
        // for both (one launch fewer per chunk)
        const bool full = nbc == cb;
        if (oldinit) {
            SDNR_HIP(hipMemsetAsync(pl, 0, (size_t)nbc * per_batch + (full ? kFlagInts * sizeof(int) : 0),
                                    ctx->stream));
            if (!full) SDNR_HIP(hipMemsetAsync(changed, 0, kFlagInts * sizeof(int), ctx->stream));
            hipLaunchKernelGGL(msbfs_plane_seed_kernel, dim3((nd + 255) / 256), dim3(256), 0,
                               ctx->stream, V, VS, d_dst + (size_t)c0 * 64, nd, pl, npl,
                               status);
        } else if (fuse1) {
            SDNR_HIP(hipMemsetAsync(changed, 0, kFlagInts * sizeof(int), ctx->stream));
#define SDNR_INIT1(SB_, DP_)                                                                  \
    hipLaunchKernelGGL((msbfs_plane_init1_kernel<SB_, DP_>), dim3((VS + lb - 1) / lb, nbc),       \
                       dim3(lb), 0, ctx->stream, V, VS, W, ctx->ell_col,                          \
                       d_dst + (size_t)c0 * 64, nd, pl, changed, status)
            if (compact) {
                if (sb == 3) SDNR_INIT1(3, 3);
                else if (sb == 4) SDNR_INIT1(4, 3);
                else if (sb == 5) SDNR_INIT1(5, 3);
                else SDNR_INIT1(6, 3);
            } else {
                if (sb == 3) SDNR_INIT1(3, 8);
                else if (sb == 4) SDNR_INIT1(4, 8);
                else if (sb == 5) SDNR_INIT1(5, 8);
                else SDNR_INIT1(6, 8);
            }
#undef SDNR_INIT1
        } else {
            hipLaunchKernelGGL(msbfs_plane_init_kernel, dim3((VS + lb - 1) / lb, nbc), dim3(lb), 0,
                               ctx->stream, V, VS, d_dst + (size_t)c0 * 64, nd, pl, npl,
                               changed, kFlagInts, status);
        }
        SDNR_HIP(hipGetLastError());
        uint16_t *dist = d_dist + (size_t)c0 * 64 * V;
        int32_t *nh = d_nh ? d_nh + (size_t)c0 * 64 * V : nullptr;
        int32_t *nhp = d_nh_port ? d_nh_port + (size_t)c0 * 64 * V : nullptr;
        constexpr int kGroup = 8;
        const long long target = (long long)V * nbc;
        int lvl = fuse1 ? 2 : 1, upto = 0;
        int st[2] = {0, 0};
        for (bool first = true;; first = false) {
            upto = lvl <= guess ? guess : lvl + kGroup - 1;
            // level 1 done by the init: a BFS the previous call finished at
            // level 1 goes straight to the table pass
            if (fuse1 && first && guess == 1) upto = 1;
            if (upto > 255) upto = 255;
            if (compact && upto > 7) upto = 7;
            for (; lvl <= upto; ++lvl) {
#define SDNR_LEVEL(SB_, DP_)                                                                  \
    hipLaunchKernelGGL((msbfs_plane_level_kernel<SB_, DP_>),                                      \
                       dim3((V + lb - 1) / lb, (nbc + bpb - 1) / bpb), dim3(lb * bpb), 0,         \
                       ctx->stream, V, VS, W, ctx->ell_col, nd, nbc, lb, lvl, (lvl - 1) & 1, pl,  \
                       changed, popt, status)
                if (compact) {
                    if (sb == 3) SDNR_LEVEL(3, 3);
                    else if (sb == 4) SDNR_LEVEL(4, 3);
                    else if (sb == 5) SDNR_LEVEL(5, 3);
                    else SDNR_LEVEL(6, 3);
                } else {
                    if (sb == 3) SDNR_LEVEL(3, 8);
                    else if (sb == 4) SDNR_LEVEL(4, 8);
                    else if (sb == 5) SDNR_LEVEL(5, 8);
                    else SDNR_LEVEL(6, 8);
                }
#undef SDNR_LEVEL
                SDNR_HIP(hipGetLastError());
            }
            // the table pass publishes the levels' status to the host as it
            // starts: the host waits for the levels only, and returns while
            // the table pass runs (the next call's launches overlap it)
            const int seq = ++ctx->pub_seq;
            int *hp = ctx->h_pub;
#define SDNR_TABLES(SB_, TB_, Q_, DP_)                                                          \
    hipLaunchKernelGGL((msbfs_plane_tables_kernel<SB_, TB_, Q_, DP_>),                            \
                       dim3((V + TB_ - 1) / TB_, nbc), dim3(TB_ * Q_),                             \
                       (size_t)(nh ? 2 * W * (TB_ + 1) * 4 : 0), ctx->stream, V, VS, W,            \
                       ctx->ell_col, ctx->ell_port, nd, pl, dist, nh, nhp, status, hp, seq)
#define SDNR_TABLES_SB(TB_, Q_, DP_)                                                            \
    do {                                                                                        \
        if (sb == 3) SDNR_TABLES(3, TB_, Q_, DP_);                                              \
        else if (sb == 4) SDNR_TABLES(4, TB_, Q_, DP_);                                         \
        else if (sb == 5) SDNR_TABLES(5, TB_, Q_, DP_);                                         \
        else SDNR_TABLES(6, TB_, Q_, DP_);                                                      \
    } while (0)
            if (small && compact) SDNR_TABLES_SB(64, 4, 3);
            else if (small) SDNR_TABLES_SB(64, 4, 8);
            else if (compact) SDNR_TABLES_SB(256, 1, 3);
            else SDNR_TABLES_SB(256, 1, 8);
#undef SDNR_TABLES_SB
#undef SDNR_TABLES
            SDNR_HIP(hipGetLastError());
            if ((rc = sdnr_wait_published(ctx, seq, 2, st))) return rc;
            if ((long long)st[0] == target || st[1] < upto) break;
            if (compact && upto >= 7) return kPlaneDeeper;   // past the 3 level planes
            if (upto == 255) return 1;           // deeper than 255 levels
        }
        levels += upto;
        // the next chunk / call queues exactly the levels this one needed:
        // up to the completing level, or one more (the empty level) when
        // some word stays incomplete (unreachable pairs)
        guess = (long long)st[0] == target ? st[1] : st[1] + 1;
        if (guess < 1) guess = 1;
        if (c0 == 0) ctx->plane_depth = guess;
        if (noguess) guess = 0;
    }
    ctx->last_launches = levels;
    ctx->last_kernel = "msbfs_plane_level_kernel+msbfs_plane_tables_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}

static int launch_plane(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst, uint16_t *d_dist,
                        int32_t *d_nh, int32_t *d_nh_port)
{
    // compact level planes when the previous call on this graph ended by
    // level 7 (SDNROUTE_PLANE_DP=8 keeps the 8 planes); a deeper BFS redoes
    // the call with 8
    const char *f = getenv("SDNROUTE_PLANE_DP");
    const char *gq = getenv("SDNROUTE_PLANE_GUESS");
    const bool compact = !(f && !strcmp(f, "8")) && !(gq && !strcmp(gq, "0")) &&
                         ctx->plane_depth >= 1 && ctx->plane_depth <= 7;
    int rc = launch_plane_dp(ctx, d_dst, ndst, d_dist, d_nh, d_nh_port, compact);
    if (rc == kPlaneDeeper) {
        ctx->plane_depth = 0;
        rc = launch_plane_dp(ctx, d_dst, ndst, d_dist, d_nh, d_nh_port, false);
    }
    return rc;
}

int sdnr_launch_shortest(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst,
                         uint16_t *d_dist, int32_t *d_nh, int32_t *d_nh_port)
{
    const int V = ctx->V;
    if (ndst == 0 || V == 0) return SDNR_OK;
    const int nbatch = (ndst + 63) / 64;
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    const size_t dlds = (size_t)bfs_dest_words(V) * 4;
    const bool dest_ok = ctx->adj16 != nullptr && ctx->radj16 != nullptr && V < 65534 &&
                         dlds <= 64 * 1024;
    const char *force = sp_strategy();
    // the bit-plane BFS wins wherever its rows fit and the batch is not tiny
    // (dragonfly all-pairs 0.226 -> 0.197 ms, torus 32^3 22.6 -> 16.1 ms, k=48
    // 0.193 -> 0.127 ms; a 32-destination fat-tree k=8 batch is dominated by
    // its per-level syncs);
    // SDNROUTE_SP_STRATEGY=plane|lanes|msbfs forces a kernel family
    // rows of up to 64 slots: k=48 fat-tree (48 slots, 6 slot planes) 0.193 ->
    // 0.127 ms over bfs_dest_kernel, bit-exact
    const bool apsp_ok = V <= 4096;
    if (apsp_ok && (!strcmp(force, "apsp") || (!*force && sp_apsp_default(ctx, ndst))))
        return launch_sp_apsp(ctx, d_dst, ndst, d_dist, d_nh, d_nh_port);
    const bool plane_ok = ctx->W > 0 && ctx->W <= 64;
    // ... and on any batch of a graph of >= 1,024 vertices, where one
    // workgroup walking a destination's whole BFS is slower than the plane
    // BFS's level launches even for a single destination (back-to-back, one
    // box, gpurun_out/r5_absp2/3: k=48 1 / 144 / 576 destinations 123.6 /
    // 125.6 / 150.1 -> 70.2 / 74.8 / 77.3 us -- the N = 8 / N = 2 shares of
    // an all-pairs step were slower than the whole 1,152 (84.8 us); dragonfly
    // a16 h8 144 destinations 88.9 -> 42.6 us; fat-tree k=32 (V = 1,280) 61
    // -> 53 us; below, k=24 (V = 720) 40 vs 46 us and k=8 14 vs 38 us keep
    // the per-destination kernel)
    const bool plane_big = (size_t)ndst * (size_t)V >= ((size_t)1 << 21) || V >= 1024;
    if (plane_ok && (!strcmp(force, "plane") || (!*force && plane_big))) {
        const int rc = launch_plane(ctx, d_dst, ndst, d_dist, d_nh, d_nh_port);
        if (rc <= 0) return rc;
    }
    if (dest_ok && strcmp(force, "msbfs") != 0 && strcmp(force, "lanes") != 0 &&
        strcmp(force, "plane") != 0) {
        const bool sym = ctx->radj16 == ctx->adj16;
        size_t bpc = SDNR_LDS_PER_CU / dlds;
        if (bpc > 8) bpc = 8;
        int grid = (int)((size_t)ctx->num_cus * bpc);
        if (grid > ndst) grid = ndst;
        // SDNROUTE_SP_VARIANT: 0 = 4 waves x 16 rows in flight (default),
        // 1 = 4 x 8, 2 = 8 x 8 (tuning)
        const char *vf = sdnr_tune_env("SDNROUTE_SP_VARIANT");
        const int var = vf ? atoi(vf) : 0;
        static const char *names[2][3] = {
            {"bfs_dest_kernel<4,16,asym>", "bfs_dest_kernel<4,8,asym>", "bfs_dest_kernel<8,8,asym>"},
            {"bfs_dest_kernel<4,16,sym>", "bfs_dest_kernel<4,8,sym>", "bfs_dest_kernel<8,8,sym>"}};
        const int vi = (var == 1 || var == 2) ? var : 0;
        ctx->last_kernel = names[sym ? 1 : 0][vi];
#define SDNR_BFS_DEST(NW_, G_, S_)                                                           \
    do {                                                                                     \
        auto k = bfs_dest_kernel<NW_, G_, S_>;                                               \
        sdnr_allow_lds(reinterpret_cast<const void *>(k), dlds);                             \
        hipLaunchKernelGGL(k, dim3(grid), dim3(NW_ * 64), dlds, ctx->stream, V, ctx->W,      \
                           ctx->adj16, ctx->radj16, ctx->row_ptr, ctx->port, ctx->ell_port,  \
                           d_dst, ndst, d_dist, d_nh, d_nh_port);                            \
    } while (0)
        if (vi == 1) {
            if (sym) SDNR_BFS_DEST(4, 8, true); else SDNR_BFS_DEST(4, 8, false);
        } else if (vi == 2) {
            if (sym) SDNR_BFS_DEST(8, 8, true); else SDNR_BFS_DEST(8, 8, false);
        } else {
            if (sym) SDNR_BFS_DEST(4, 16, true); else SDNR_BFS_DEST(4, 16, false);
        }
#undef SDNR_BFS_DEST
        SDNR_HIP(hipGetLastError());
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    // lane-packed per-destination BFS: rows of <= 32 entries, one workgroup's
    // LDS holds the levels, queue and claim bits
    const int maxrow = ctx->max_deg > ctx->max_indeg ? ctx->max_deg : ctx->max_indeg;
    const int lpr = maxrow <= 4 ? 4 : maxrow <= 8 ? 8 : maxrow <= 16 ? 16 : 32;
    const size_t llds = bfs_lanes_bytes(V, lpr);
    const bool lanes_ok = ctx->adj16 != nullptr && ctx->radj16 != nullptr && V < 65534 &&
                          maxrow <= 32 && llds <= SDNR_MAX_LDS_PER_BLOCK - 1024;
    if (lanes_ok && strcmp(force, "msbfs") != 0 && strcmp(force, "plane") != 0) {
        const bool sym = ctx->radj16 == ctx->adj16;
        size_t bpc = SDNR_LDS_PER_CU / llds;
        if (bpc > 2) bpc = 2;
        if (bpc < 1) bpc = 1;
        int grid = (int)((size_t)ctx->num_cus * bpc);
        if (grid > ndst) grid = ndst;
        static const char *names[2][4] = {
            {"bfs_dest_lanes_kernel<4,asym>", "bfs_dest_lanes_kernel<8,asym>",
             "bfs_dest_lanes_kernel<16,asym>", "bfs_dest_lanes_kernel<32,asym>"},
            {"bfs_dest_lanes_kernel<4,sym>", "bfs_dest_lanes_kernel<8,sym>",
             "bfs_dest_lanes_kernel<16,sym>", "bfs_dest_lanes_kernel<32,sym>"}};
        const int li = maxrow <= 4 ? 0 : maxrow <= 8 ? 1 : maxrow <= 16 ? 2 : 3;
        ctx->last_kernel = names[sym ? 1 : 0][li];
        // SDNROUTE_SP_LANES_G=1|2|4|8: frontier groups in flight per wave
        // (tuning; torus 32^3: 1 24.6 ms, 2 22.5 ms, 4 24.4 ms, 8 29.6 ms)
        const char *gf = sdnr_tune_env("SDNROUTE_SP_LANES_G");
        const int gsel = gf ? atoi(gf) : 2;
#define SDNR_BFS_LANES_G(LPR_, S_, G_)                                                       \
    do {                                                                                     \
        auto k = bfs_dest_lanes_kernel<LPR_, 16, G_, S_>;                                    \
        sdnr_allow_lds(reinterpret_cast<const void *>(k), llds);                             \
        hipLaunchKernelGGL(k, dim3(grid), dim3(16 * 64), llds, ctx->stream, V, ctx->W,       \
                           ctx->adj16, ctx->radj16, ctx->row_ptr, ctx->col, ctx->port,       \
                           ctx->ell_col, ctx->ell_port, d_dst, ndst, d_dist, d_nh,           \
                           d_nh_port);                                                       \
    } while (0)
#define SDNR_BFS_LANES(LPR_, S_)                                                             \
    do {                                                                                     \
        if (gsel == 1) SDNR_BFS_LANES_G(LPR_, S_, 1);                                        \
        else if (gsel == 2) SDNR_BFS_LANES_G(LPR_, S_, 2);                                   \
        else if (gsel == 4) SDNR_BFS_LANES_G(LPR_, S_, 4);                                   \
        else SDNR_BFS_LANES_G(LPR_, S_, 8);                                                  \
    } while (0)
#define SDNR_BFS_LANES_S(LPR_)                                                               \
    do {                                                                                     \
        if (sym) SDNR_BFS_LANES(LPR_, true); else SDNR_BFS_LANES(LPR_, false);               \
    } while (0)
        if (li == 0) SDNR_BFS_LANES_S(4);
        else if (li == 1) SDNR_BFS_LANES_S(8);
        else if (li == 2) SDNR_BFS_LANES_S(16);
        else SDNR_BFS_LANES_S(32);
#undef SDNR_BFS_LANES_S
#undef SDNR_BFS_LANES
#undef SDNR_BFS_LANES_G
        SDNR_HIP(hipGetLastError());
        if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    const size_t lds = (size_t)V * 3 * sizeof(uint64_t);
    // large graphs with ELL rows: the bit-plane BFS with fused next hops
    // (SDNROUTE_SP_STRATEGY=msbfs keeps the level + next-hop pair)
    if (lds > 150 * 1024 && ctx->W > 0 && ctx->W <= 32 && strcmp(force, "msbfs") != 0) {
        const int rc = launch_plane(ctx, d_dst, ndst, d_dist, d_nh, d_nh_port);
        if (rc <= 0) return rc;                  // else: too deep, redo below
    }
    SDNR_HIP(hipMemsetAsync(d_dist, 0xFF, (size_t)ndst * V * sizeof(uint16_t), ctx->stream));
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
        ctx->last_launches = 0;
        for (int lvl = 1; lvl < 0xFFFF && h_changed; ++lvl) {
            ctx->last_launches = lvl;
            SDNR_HIP(hipMemsetAsync(changed, 0, sizeof(int), ctx->stream));
            hipLaunchKernelGGL(msbfs_level_kernel, dim3((V + 255) / 256, nbatch), dim3(256),
                               0, ctx->stream, V, ctx->W, ctx->row_ptr, ctx->col, ctx->ell_col,
                               ndst, lvl, front, next, vis, d_dist, changed);
            SDNR_HIP(hipGetLastError());
            int rc2 = sdnr_fetch_ints(ctx, changed, 1, &h_changed);
            if (rc2) return rc2;
            uint64_t *t = front;
            front = next;
            next = t;
        }
    }
    if (d_nh && d_nh_port) {
        const int stage = (size_t)V * 2 <= 64 * 1024;
        int grid = ctx->num_cus * 8;
        if (grid > ndst) grid = ndst;
        auto k = nexthop_kernel;
        if (stage) sdnr_allow_lds(reinterpret_cast<const void *>(k), (size_t)V * 2);
        hipLaunchKernelGGL(k, dim3(grid), dim3(1024), stage ? (size_t)V * 2 : 0, ctx->stream, V,
                           ctx->W, ndst, ctx->row_ptr, ctx->col, ctx->port, ctx->ell_col,
                           ctx->ell_port, d_dist, d_nh, d_nh_port, stage);
        SDNR_HIP(hipGetLastError());
    }
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
