// dfs_bits.hip -- default-route tables, the search chain in registers.
//
// Reference: TopologyDB._find_route_dfs (sdnmpi/util/topology_db.py:59-84):
// LIFO search, a switch is marked when it is PUSHED (:78-82), neighbours are
// pushed in ascending dpid order (:76); one full traversal from s answers
// every destination (the tree of first pushes, dfs.hip's header).
//
// LIFO with ascending pushes is the recursion explore(u): C = N(u) \ visited;
// mark C; for c in C, descending: explore(c) -- the children of one pop form
// a FRAME, popped from the highest id down.  dfs_async_kernel keeps the
// visited bits, the stack of vertices and the counts in LDS, and a candidate
// costs 4-5 dependent LDS round trips (visited gather, count gather behind
// the stack / ring / parent writes, the skip's stack and count reads).  For
// graphs of up to 4,096 switches this kernel holds the whole visited set in
// the search wave's REGISTERS -- lane l owns bits 64l..64l+63, one u64 -- and
// the switch rows as BITMAPS in the same layout (512 B per row, L2
// resident), so exploring u is
//     fresh = row(u) & ~visited; visited |= fresh        (lane-local VALU)
// and a frame is the u64 of each lane (sparse: only lanes with children are
// logged).  Leaf pops are skipped with a bitmap of non-leaves NL (bit v set
// while v may still have an unvisited out-neighbour), maintained by the
// decrement workers from the same counts as dfs_async_kernel (stale-set NL
// bits only cost a candidate that finds no fresh child; a bit is cleared only
// when the count reaches 0, and counts are never low).  The next candidate is
// the highest bit of (frame & NL): one 8-byte LDS read per lane -- the only
// LDS round trip on the chain of a child-first candidate -- while the row of
// the highest fresh child is already in flight.
//
// State per source (LDS): counts (u32, swizzled as dfs_async_kernel's, plus
// one dummy word per lane for the in-row padding), NL (64 x u64), the frame
// log (per logged lane: its u64 bits + lane | parent << 6 | parent depth <<
// 18), frame headers (first log entry | entries << 16), the stack of saved
// frames (frame | cursor << 16: the frame's bits below the cursor remain);
// log, headers and stack spill to a global area past their LDS capacity.
// Workers take logged lanes round-robin, expand their bits into children and
// decrement each child's in-neighbours (radjx: count index | vertex << 16,
// padding -> a dummy word and vertex 0xFFFF), clearing NL bits at zero.  The
// epilogue turns the log into parent | slot << 16 per vertex (slot = rank of
// v in the parent's row: prefix popcount of the bitmap row) and writes the
// tables as dfs_async_kernel does.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr int kBitsEmax = 768;           // log entries in LDS
constexpr int kBitsFmax = 384;           // frame headers in LDS
constexpr int kBitsDmax = 192;           // stack entries in LDS
constexpr int kBitsG = 8;                // children per worker step
constexpr int kBitsK = 4;                // candidates tested together
constexpr unsigned kBitsSpin = 1u << 22;
constexpr int kBitsFlagPrio = 1;         // search wave at raised issue priority
constexpr int kBitsFlagHops16 = 32;      // hop counts as u16 (0xFFFF unreached)
constexpr unsigned kBitsDummyInit = 0x40000000u;

#ifdef SDNR_STAMPS
// diagnostic build only (tools/build_stamps.sh): per-phase cycle and event
// counts of the search wave, summed over sources (sdnr_debug_bits_stamps)
__device__ unsigned long long g_bits_stamp[16];
#define BITS_STAMP(i, v) atomicAdd(&g_bits_stamp[i], (unsigned long long)(v))
#else
#define BITS_STAMP(i, v) do { (void)(v); } while (0)
#endif

__device__ __forceinline__ uint64_t read_lane64(uint64_t x, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), l);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ int bswz(int x) { return x ^ ((x >> 3) & 31); }

// LDS words per source; shared with the launcher
struct BitsLayout {
    int CW, NLw, LMw, LTw, FHw, STw, DPw, CTw, total;
    __host__ __device__ BitsLayout(int V, bool hops)
    {
        CW = ((V + 31) & ~31) + 64;          // counts (swizzled) + 64 dummies; ps later
        CW = (CW + 1) & ~1;                  // keep what follows 8-byte aligned
        NLw = 128;                           // 64 x u64
        LMw = 2 * kBitsEmax;                 // u64 bits per entry
        LTw = kBitsEmax;                     // u32 meta per entry
        FHw = kBitsFmax;
        STw = kBitsDmax;
        DPw = hops ? ((V + 1) >> 1) : 0;     // u16 depth per vertex
        CTw = 4;
        total = CW + NLw + LMw + LTw + FHw + STw + DPw + CTw;
    }
};

template <int NW, bool HOPS, bool PACKED>
__global__ __launch_bounds__(NW * 64) void dfs_bits_kernel(
    int V, const uint64_t *__restrict__ adjb, const uint8_t *__restrict__ adjp,
    const uint32_t *__restrict__ radjx, const uint32_t *__restrict__ deg,
    const int32_t *__restrict__ row_ptr, const int32_t *__restrict__ port, int W,
    const int32_t *__restrict__ ell_port, const int32_t *__restrict__ src, int nsrc,
    int32_t *__restrict__ out_parent, int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops,
    uint64_t *__restrict__ spill, int *__restrict__ err, int flags)
{
    static_assert(NW >= 2, "wave 0 searches, the others decrement");
    constexpr int S = NW - 1;
    constexpr int U = 4;                     // epilogue vertices per thread per step
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const BitsLayout lay(V, HOPS);
    uint32_t *cnt = lds;                                        // cnt[bswz(v)]; later ps[v]
    uint64_t *NL = reinterpret_cast<uint64_t *>(lds + lay.CW);
    uint64_t *lm = NL + 64;
    uint32_t *lt = reinterpret_cast<uint32_t *>(lm + kBitsEmax);
    uint32_t *fh = lt + kBitsEmax;
    uint32_t *st = fh + kBitsFmax;
    uint16_t *dep = reinterpret_cast<uint16_t *>(st + kBitsDmax);
    int *ctl = reinterpret_cast<int *>(st + kBitsDmax + lay.DPw);   // [0] published [1] done
    uint32_t *ps = cnt;
    const int dummy = (V + 31) & ~31;
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    // spill area of this workgroup: entries (u64 bits, u32 meta), headers, stack
    uint64_t *gm = spill + (size_t)blockIdx.x * (size_t)V * 3;
    uint32_t *gt = reinterpret_cast<uint32_t *>(gm + V);
    uint32_t *gfh = gt + V;
    uint32_t *gst = gfh + V;

    for (int si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int s = uniform(src[si]);
        int32_t *prow = out_parent + (size_t)si * V;
        int32_t *trow = PACKED ? nullptr : out_port + (size_t)si * V;
        const size_t hb = (size_t)si * V;
        auto put_hop = [&](size_t e, int h) {
            if (flags & kBitsFlagHops16) reinterpret_cast<uint16_t *>(out_hops)[e] = (uint16_t)h;
            else out_hops[e] = h;
        };
        if (s < 0 || s >= V) {
            for (int v = threadIdx.x; v < V; v += blockDim.x) {
                prow[v] = -1;                    // packed: 0xFFFFFFFF
                if (!PACKED) trow[v] = -1;
                if (HOPS) put_hop(hb + v, -1);
            }
            continue;
        }
        // counts start at the out-degrees, dummies high; NL = out-degree > 0
        for (int i0 = threadIdx.x; i0 < V; i0 += U * blockDim.x) {
            uint32_t dg[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int i = i0 + k * (int)blockDim.x;
                dg[k] = deg[i < V ? i : V];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int i = i0 + k * (int)blockDim.x;
                if (i < V) cnt[bswz(i)] = dg[k];
            }
        }
        if (threadIdx.x < 64) cnt[dummy + threadIdx.x] = kBitsDummyInit;
        for (int l = w; l < 64; l += NW) {
            const int v = 64 * l + lane;
            const uint64_t m = __ballot(v < V && deg[v < V ? v : V] != 0u);
            if (lane == 0) NL[l] = m;
        }
        if (threadIdx.x < 4) ctl[threadIdx.x] = 0;
        __syncthreads();

        if (w == 0) {
            // ------------------------------------------------ the search
            if (flags & kBitsFlagPrio) __builtin_amdgcn_s_setprio(3);
            auto log_put = [&](int e, uint64_t m, uint32_t t) {
                if (e < kBitsEmax) {
                    lm[e] = m;
                    lt[e] = t;
                } else {
                    gm[e - kBitsEmax] = m;
                    gt[e - kBitsEmax] = t;
                }
            };
            // frame 0 = {s}, already popped: its cursor s leaves nothing
            uint64_t vis = lane == (s >> 6) ? 1ull << (s & 63) : 0ull;
            if (lane == 0) {
                lm[0] = 1ull << (s & 63);
                lt[0] = (uint32_t)(s >> 6) | ((uint32_t)s << 6);
                fh[0] = 0u | (1u << 16);
                __hip_atomic_store(&ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            int fidx = 0, fdep = 0, nf = 1, ne = 1, sp = 0;
            int Lid = -1;
            uint64_t M = 0;
            int u = s, du = 0;
            int pfu = -1;
            uint64_t pfrow = 0ull;
            uint64_t rb = adjb[(size_t)s * 64 + lane];   // row of the vertex to explore
            bool spilled = false;
#ifdef SDNR_STAMPS
            unsigned long long z0 = __builtin_readcyclecounter(), za, zb, z_ex = 0, z_sel = 0;
            unsigned long long n_ex = 0, n_false = 0, n_ret = 0, n_miss = 0;
#endif
            // frame & NL below the cursor x: drop x and every bit above it
            auto below = [&](uint64_t &mm, int x) {
                const int xl = x >> 6;
                if (Lid > xl) mm = 0ull;
                else if (Lid == xl) mm &= (1ull << (x & 63)) - 1ull;
            };
            for (;;) {
                // ---- explore u (its row in rb, its fresh children non-empty
                // unless u is the source)
#ifdef SDNR_STAMPS
                za = __builtin_readcyclecounter();
                n_ex++;
#endif
                const uint64_t fresh = rb & ~vis;
                const uint64_t fm = __ballot(fresh != 0ull);
                if (fm) {
                    vis |= fresh;
                    const int k = __popcll(fm);
                    const int rank = lanes_below(fm);
                    // the current frame, u popped from it, goes on the stack
                    const uint32_t se = (uint32_t)fidx | ((uint32_t)u << 16);
                    if (lane == 0) {
                        if (sp < kBitsDmax) st[sp] = se;
                        else gst[sp - kBitsDmax] = se;
                        if (nf < kBitsFmax) fh[nf] = (uint32_t)ne | ((uint32_t)k << 16);
                        else gfh[nf - kBitsFmax] = (uint32_t)ne | ((uint32_t)k << 16);
                    }
                    ++sp;
                    if (fresh)
                        log_put(ne + rank, fresh,
                                (uint32_t)lane | ((uint32_t)u << 6) | ((uint32_t)du << 18));
                    fidx = nf++;
                    fdep = du;
                    Lid = fresh ? lane : -1;
                    M = fresh;
                    if (ne + k > kBitsEmax) spilled = true;
                    ne += k;
                    // announce the entries: one wave's LDS ops execute in
                    // issue order (the empty asm keeps the compiler from
                    // hoisting the store); spilled entries need a real release
                    if (spilled) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                        spilled = false;
                    }
                    __asm__ volatile("" ::: "memory");
                    if (lane == 0) __hip_atomic_store(&ctl[0], ne, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    // the highest fresh child is the next candidate most of
                    // the time: its row goes in flight now
                    const int h = highest_lane(fm);
                    const int c1 = 64 * h + 63 - __clzll(read_lane64(fresh, h));
                    pfu = c1;
                    pfrow = adjb[(size_t)c1 * 64 + lane];
                }
#ifdef SDNR_STAMPS
                else {
                    n_false++;
                }
                zb = __builtin_readcyclecounter();
                z_ex += zb - za;
#endif
                // ---- the next vertex to explore: among the highest bits of
                // frame & NL (NL may be stale-set: a candidate may be a leaf
                // after all), up to K at a time are tested exactly -- their
                // rows loaded together, the first with a fresh child wins
                bool done = false;
                for (;;) {
                    const uint64_t nl = Lid >= 0 ? __hip_atomic_load(&NL[Lid], __ATOMIC_RELAXED,
                                                                      __HIP_MEMORY_SCOPE_WORKGROUP)
                                                 : 0ull;
                    uint64_t cand = M & nl;
                    int cv[kBitsK];
                    int nc = 0;
#pragma unroll
                    for (int q = 0; q < kBitsK; ++q) {
                        cv[q] = -1;
                        const uint64_t cm = __ballot(cand != 0ull);
                        if (cm) {
                            const int h = highest_lane(cm);
                            const int b = 63 - __clzll(read_lane64(cand, h));
                            cv[q] = 64 * read_lane(Lid, h) + b;
                            if (lane == h) cand &= ~(1ull << b);
                            ++nc;
                        }
                    }
                    if (nc) {
                        uint64_t rk[kBitsK];
#pragma unroll
                        for (int q = 0; q < kBitsK; ++q)
                            if (q < nc) rk[q] = cv[q] == pfu ? pfrow : adjb[(size_t)cv[q] * 64 + lane];
                        int pick = -1;
#pragma unroll
                        for (int q = 0; q < kBitsK; ++q) {
                            if (pick < 0 && q < nc) {
                                if (__ballot((rk[q] & ~vis) != 0ull)) {
                                    pick = q;
                                    rb = rk[q];
                                }
                            }
                        }
#ifdef SDNR_STAMPS
                        n_false += pick < 0 ? nc : pick;
                        if (cv[0] != pfu) n_miss++;
#endif
                        if (pick >= 0) {
                            // the picked vertex and every bit above it leave
                            // the frame (the ones above are leaf pops)
                            int x = cv[0];
#pragma unroll
                            for (int q = 0; q < kBitsK; ++q)
                                if (q == pick) x = cv[q];
                            below(M, x);
                            u = x;
                            du = fdep + 1;
                            break;
                        }
                        below(M, cv[nc - 1]);    // all leaves: popped
                        continue;
                    }
                    // frame exhausted: back to the saved one below
                    if (sp == 0) {
                        done = true;
                        break;
                    }
#ifdef SDNR_STAMPS
                    n_ret++;
#endif
                    --sp;
                    // the spill area is reused across sources: this wave's own
                    // stores must be done and no stale line read (rare path)
                    if (sp >= kBitsDmax || ne > kBitsEmax || nf > kBitsFmax)
                        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
                    const uint32_t se = sp < kBitsDmax ? st[sp] : gst[sp - kBitsDmax];
                    fidx = (int)(se & 0xFFFFu);
                    const int cur = (int)(se >> 16);
                    const uint32_t hd = fidx < kBitsFmax ? fh[fidx] : gfh[fidx - kBitsFmax];
                    const int start = (int)(hd & 0xFFFFu), k = (int)(hd >> 16);
                    M = 0ull;
                    Lid = -1;
                    uint32_t t = 0u;
                    if (lane < k) {
                        const int e = start + lane;
                        if (e < kBitsEmax) {
                            M = lm[e];
                            t = lt[e];
                        } else {
                            M = gm[e - kBitsEmax];
                            t = gt[e - kBitsEmax];
                        }
                        Lid = (int)(t & 63u);
                    }
                    fdep = (int)(read_lane((int)t, 0) >> 18);
                    below(M, cur);
                }
#ifdef SDNR_STAMPS
                z_sel += __builtin_readcyclecounter() - zb;
#endif
                if (done) break;
            }
#ifdef SDNR_STAMPS
            if (lane == 0) {
                BITS_STAMP(0, __builtin_readcyclecounter() - z0);   // search wave life
                BITS_STAMP(1, n_ex);                                  // explores (candidates)
                BITS_STAMP(2, n_false);                               // ... with no fresh child
                BITS_STAMP(3, n_ret);                                 // frame returns
                BITS_STAMP(4, z_ex);                                  // cycles: explore
                BITS_STAMP(5, z_sel);                                 // cycles: select + returns
                BITS_STAMP(6, n_miss);                                // row prefetch misses
                BITS_STAMP(7, 1);                                     // sources
            }
#endif
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&ctl[1], ne, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (flags & kBitsFlagPrio) __builtin_amdgcn_s_setprio(0);
        } else {
            // ------------------------------------------------ the decrements
            // every worker reads every log entry and takes the children whose
            // ordinal (over the whole log) is its own mod S: a frame's
            // children are decremented by all workers at once
            int j = 0, ord = 0;                  // next log entry, its first child's ordinal
            const int q = w - 1;
            for (unsigned spin = 0;;) {
                const int P = __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (j >= P) {
                    const int fin = __hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (fin && j >= fin) break;
                    if (++spin > kBitsSpin) {
                        if (lane == 0) atomicOr(err, 32);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                spin = 0;
                uint64_t m;
                uint32_t t;
                if (j < kBitsEmax) {
                    m = lm[j];
                    t = lt[j];
                } else {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    m = gm[j - kBitsEmax];
                    t = gt[j - kBitsEmax];
                }
                m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)m)) |
                    ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(m >> 32)) << 32);
                const int base = 64 * (int)(__builtin_amdgcn_readfirstlane((int)t) & 63);
                // skip to this worker's first child of the entry
                int skip = (q - ord) % S;
                if (skip < 0) skip += S;
                ord += __popcll(m);
                for (int i = 0; i < skip && m; ++i) m &= m - 1ull;
                while (m) {
                    int c[kBitsG];
                    int n = 0;
#pragma unroll
                    for (int g = 0; g < kBitsG; ++g) {
                        c[g] = V;                // the sentinel row: all padding
                        if (m) {
                            c[g] = base + __builtin_ctzll(m);
                            ++n;
                            for (int i = 0; i < S && m; ++i) m &= m - 1ull;   // next own child
                        }
                    }
                    uint32_t r[kBitsG];
#pragma unroll
                    for (int g = 0; g < kBitsG; ++g) r[g] = radjx[(size_t)c[g] * 64 + lane];
                    uint32_t old[kBitsG];
#pragma unroll
                    for (int g = 0; g < kBitsG; ++g)
                        old[g] = g < n ? atomicSub(&cnt[r[g] & 0xFFFFu], 1u) : 2u;
#pragma unroll
                    for (int g = 0; g < kBitsG; ++g) {
                        const uint32_t v = r[g] >> 16;
                        if (old[g] == 1u && v != 0xFFFFu)
                            atomicAnd(reinterpret_cast<unsigned long long *>(&NL[v >> 6]),
                                      ~(1ull << (v & 63)));
                    }
                }
                ++j;
            }
        }
        __syncthreads();

        // ---------------------------------------------------- the tables
        const int ne = ctl[1];
        if (ne > kBitsEmax) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        for (int v = threadIdx.x; v < V; v += blockDim.x) ps[v] = 0xFFFFFFFFu;
        __syncthreads();
        if (threadIdx.x == 0) {
            ps[s] = (uint32_t)s | (0xFFFFu << 16);
            if (HOPS) dep[s] = 0;
        }
        // log entries (frame 0 = the root excluded): parent | slot << 16 and
        // depth of every logged bit; slot = rank of v in the parent's row
        for (int e = 1 + (int)threadIdx.x; e < ne; e += blockDim.x) {
            uint64_t m;
            uint32_t t;
            if (e < kBitsEmax) {
                m = lm[e];
                t = lt[e];
            } else {
                m = gm[e - kBitsEmax];
                t = gt[e - kBitsEmax];
            }
            const int L = (int)(t & 63u), p = (int)((t >> 6) & 0xFFFu), d = (int)(t >> 18);
            const uint64_t rw = adjb[(size_t)p * 64 + L];
            const uint32_t pre = adjp[(size_t)p * 64 + L];
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1ull;
                const int v = 64 * L + b;
                const uint32_t slot = pre + (uint32_t)__popcll(rw & ((1ull << b) - 1ull));
                ps[v] = (uint32_t)p | (slot << 16);
                if (HOPS) dep[v] = (uint16_t)(d + 1);
            }
        }
        __syncthreads();
        for (int v0 = threadIdx.x; v0 < V; v0 += U * blockDim.x) {
            int p[U], sl[U], pt[U];
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                p[k] = -1;
                sl[k] = -1;
                if (v < V) {
                    const uint32_t xx = ps[v];
                    if (xx != 0xFFFFFFFFu) {
                        p[k] = (int)(xx & 0xFFFFu);
                        if (v != s) sl[k] = (int)(xx >> 16);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                pt[k] = -1;
                if (sl[k] >= 0)
                    pt[k] = W > 0 ? ell_port[(size_t)p[k] * W + sl[k]] : port[row_ptr[p[k]] + sl[k]];
            }
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int v = v0 + k * (int)blockDim.x;
                if (v < V) {
                    if (PACKED) {                // parent | port << 16, -1 -> 0xFFFF
                        prow[v] = (int32_t)(((uint32_t)p[k] & 0xFFFFu) | ((uint32_t)pt[k] << 16));
                    } else {
                        prow[v] = p[k];
                        trow[v] = pt[k];
                    }
                    if (HOPS) put_hop(hb + v, p[k] < 0 ? -1 : (v == s ? 0 : (int)dep[v]));
                }
            }
        }
        __syncthreads();
    }
}

template <typename Kern>
void allow_lds_bits(Kern k, size_t bytes)
{
    sdnr_allow_lds(reinterpret_cast<const void *>(k), bytes);
}

}  // namespace

#ifdef SDNR_STAMPS
extern "C" int sdnr_debug_bits_stamps(unsigned long long *out16)
{
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_bits_stamp), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -5;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_bits_stamp), z, sizeof z) == hipSuccess ? 0 : -5;
}
#endif

bool sdnr_dfs_bits_ok(const sdnr_ctx *ctx)
{
    return ctx->adjb && ctx->adjp && ctx->radjx && ctx->deg32 && ctx->V > 0 && ctx->V <= 4096;
}

int sdnr_launch_dfs_bits(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                         int32_t *d_port, int32_t *d_hops, uint32_t *d_tree, bool hops16)
{
    const int V = ctx->V;
    if (!sdnr_dfs_bits_ok(ctx))
        return sdnr_fail(SDNR_ERR_INVAL, "dfs bits: needs V <= 4096 and rows of <= 64 links");
    const bool hops = d_hops != nullptr, packed = d_tree != nullptr;
    const size_t lds = (size_t)BitsLayout(V, hops).total * 4;
    // waves: 1 search + workers; more workers where few sources share a CU
    int nw = nsrc <= 2 * ctx->num_cus ? 6 : 4;
    if (const char *f = getenv("SDNROUTE_DFS_BITS_WAVES")) {
        const int k = atoi(f);
        if (k == 2 || k == 3 || k == 4 || k == 6 || k == 8) nw = k;
    }
    size_t per_cu = SDNR_LDS_PER_CU / lds;
    if (per_cu > (size_t)(32 / nw)) per_cu = 32 / nw;
    if (per_cu < 1) per_cu = 1;
    int grid = (int)((size_t)ctx->num_cus * per_cu);
    if (grid > nsrc) grid = nsrc;
    int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes,
                          (size_t)grid * (size_t)V * 3 * sizeof(uint64_t) + 256);
    if (rc) return rc;
    uint64_t *spill = static_cast<uint64_t *>(ctx->scratch);
    int flags = kBitsFlagPrio | (hops && hops16 ? kBitsFlagHops16 : 0);
    if (const char *f = getenv("SDNROUTE_DFS_BITS_FLAGS")) flags = atoi(f) | (flags & kBitsFlagHops16);
    int32_t *par = packed ? reinterpret_cast<int32_t *>(d_tree) : d_parent;
    static const char *names[2][2] = {{"dfs_bits_kernel", "dfs_bits_kernel<hops>"},
                                      {"dfs_bits_kernel<packed>", "dfs_bits_kernel<packed,hops>"}};
    ctx->last_kernel = names[packed][hops];
#define SDNR_BITS(N_, H_, P_)                                                                \
    do {                                                                                     \
        auto k = dfs_bits_kernel<N_, H_, P_>;                                                \
        allow_lds_bits(k, lds);                                                              \
        hipLaunchKernelGGL(k, dim3(grid), dim3(N_ * 64), lds, ctx->stream, V, ctx->adjb,      \
                           ctx->adjp, ctx->radjx, ctx->deg32, ctx->row_ptr, ctx->port, ctx->W,\
                           ctx->ell_port, d_src, nsrc, par, d_port, d_hops, spill, ctx->d_err,\
                           flags);                                                           \
    } while (0)
#define SDNR_BITS_HP(N_)                                                                     \
    do {                                                                                     \
        if (hops) { if (packed) SDNR_BITS(N_, true, true); else SDNR_BITS(N_, true, false); }\
        else { if (packed) SDNR_BITS(N_, false, true); else SDNR_BITS(N_, false, false); }   \
    } while (0)
    if (nw == 2) SDNR_BITS_HP(2);
    else if (nw == 3) SDNR_BITS_HP(3);
    else if (nw == 6) SDNR_BITS_HP(6);
    else if (nw == 8) SDNR_BITS_HP(8);
    else SDNR_BITS_HP(4);
#undef SDNR_BITS_HP
#undef SDNR_BITS
    SDNR_HIP(hipGetLastError());
    return SDNR_OK;
}
