// dfs_runs.hip -- default-route tables with the switch rows held in LDS.
//
// Reference: TopologyDB._find_route_dfs (sdnmpi/util/topology_db.py:59-84):
// LIFO search, a switch is marked when it is PUSHED (:78-82), neighbours are
// pushed in ascending dpid order (:76); one full traversal from s answers
// every destination (the tree of first pushes, dfs.hip's header).
//
// This is dfs_async_kernel's search (dfs.hip: leaf pops skipped through
// per-vertex counts of unvisited out-neighbours, decrement workers off the
// chain) with the last global-memory access on the chain removed.  There,
// every candidate pop fetched the popped switch's 128-B row from L2: 600-800
// cycles under load, half of the ~1,250 cycles a candidate costs.  Here the
// rows live in LDS, compressed:
//
//  * a sorted row is cut into arithmetic runs (start, stride, count) -- the
//    structured fabrics need few: fat-tree rows 1-2 (a core's aggregation
//    neighbours are h apart, an aggregation switch's are two contiguous
//    ranges), dragonfly rows 2-4 -- and a row is R run words (R = 2 or 4):
//        start (bits 0-15) | stride (16-24) | count (25-31, 0 = no run);
//    lane i of a wavefront decodes the row's i-th neighbour with a few VALU
//    ops from the R words (uniform: one broadcast LDS read);
//  * the k=48 rows take 23 KB, once per workgroup, so a workgroup runs
//    several sources ("slots"), each with its own search wave, decrement
//    workers, visited bits, u16 counts, u16 stack, u16 parents and ring;
//    slots per workgroup = sources per CU (k=48 on one GPU: 5; at 8 GPUs: 1);
//  * the chain per candidate is LDS only: the row words of every stack entry
//    are gathered together with its count (skip path), and those of every
//    new child at the push (the next candidate is a child 4 times in 5), so
//    a candidate costs the visited gather and the push;
//  * decrement workers load the children's u16 in-rows from L2 as before
//    (off the chain; a load is one instruction, an LDS run decode ~25 per
//    child, measured 2x slower in all) and ds_sub u16 count halves;
//  * the epilogue recovers each vertex's slot in its parent's row from the
//    parent's runs, looks the port up in the ELL port table and writes the
//    tables coalesced.
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr int kRunsRing = 512;          // children in flight per slot (u16)
constexpr int kRunsG = 32;              // children per worker step (most)
constexpr unsigned kRunsSpin = 1u << 22;
constexpr int kRunsFlagPrio = 1;        // search waves at raised issue priority
constexpr int kRunsU = 4;               // epilogue vertices per thread per step

// LDS words of one slot and of the rows; shared with the launcher
struct RunsLayout {
    int VWp, CWp, SWp, PWp, DWp, slot_words, row_words;
    __host__ __device__ RunsLayout(int V, int R, bool hops)
    {
        VWp = (((V + 1 + 31) >> 5) + 3) & ~3;             // visited bits of 0..V
#ifndef SDNR_RUNS_C16
        CWp = (V + 1 + 255) & ~255;                       // u32 counts of 0..V, swizzled
#else
        CWp = ((((V + 2) >> 1)) + 255) & ~255;            // u16 counts of 0..V, swizzled words
#endif
        SWp = ((((V + 2) >> 1)) + 3) & ~3;                // u16 stack
        PWp = ((V + 255) & ~255) >> 1;                    // u16 parents, swizzled ids
        DWp = hops ? ((((V + 2) >> 1)) + 3) & ~3 : 0;      // u16 depths
        slot_words = VWp + CWp + SWp + PWp + DWp + kRunsRing / 2 + 16;
        row_words = (((V + 1) * R) + 3) & ~3;
    }
};

template <int R>
__device__ __forceinline__ void load_desc(const uint32_t *rows, int v, uint32_t (&d)[R])
{
    if constexpr (R == 2) {
        const uint2 t = *reinterpret_cast<const uint2 *>(rows + (size_t)v * 2);
        d[0] = t.x;
        d[1] = t.y;
    } else {
        const uint4 t = *reinterpret_cast<const uint4 *>(rows + (size_t)v * 4);
        d[0] = t.x;
        d[1] = t.y;
        d[2] = t.z;
        d[3] = t.w;
    }
}

// i-th neighbour of the row (V past its end)
template <int R>
__device__ __forceinline__ int run_at(const uint32_t (&d)[R], int i, int V)
{
    int x = V, base = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int c = (int)(d[k] >> 25);
        const int off = i - base;
        if ((unsigned)off < (unsigned)c)
            x = (int)(d[k] & 0xFFFFu) + off * (int)((d[k] >> 16) & 0x1FFu);
        base += c;
    }
    return x;
}

// position of v in the row (v is in it)
template <int R>
__device__ __forceinline__ int run_slot(const uint32_t (&d)[R], int v)
{
    int slot = -1, base = 0;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int c = (int)(d[k] >> 25);
        const int st = (int)((d[k] >> 16) & 0x1FFu);
        const int off = v - (int)(d[k] & 0xFFFFu);
        int q = -1;
        if (off == 0) q = 0;
        else if (off > 0 && st > 0) q = (int)__fdividef((float)off + 0.5f, (float)st);
        if (slot < 0 && q >= 0 && q < c && q * st == off) slot = base + q;
        base += c;
    }
    return slot;
}

__device__ __forceinline__ int rswz(int x) { return lds_swz(x); }   // common.h

// scheduling fences between the search phases: the compiler otherwise
// interleaves the phases and the chain gets longer (measured 134 vs 91 us
// for one k=48 source)
#define RSCHED() __builtin_amdgcn_sched_barrier(0)

#ifdef SDNR_STAMPS
// diagnostic build only (tools/stamps_runs.py): search anatomy summed over
// every source; never in the real kernel
__device__ unsigned long long g_rstamp[16];
#define RSTAMP(t) \
    do { __builtin_amdgcn_sched_barrier(0); \
         asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory"); \
         __builtin_amdgcn_sched_barrier(0); } while (0)
#define RCOUNT(i, v) do { if (lane == 0) atomicAdd(&g_rstamp[i], (unsigned long long)(v)); } while (0)
#else
#define RSTAMP(t) do { (void)(t); } while (0)
#define RCOUNT(i, v) do { } while (0)
#endif

#ifndef SDNR_RUNS_C16
__device__ __forceinline__ uint32_t cnt_get(uint32_t *cntw, int v)
{
    return __hip_atomic_load(&cntw[rswz(v)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cnt_dec(uint32_t *cntw, int v) { atomicSub(&cntw[rswz(v)], 1u); }
#else
__device__ __forceinline__ void cnt_dec(uint32_t *cntw, int v)
{
    atomicSub(&cntw[rswz(v >> 1)], 1u << ((v & 1) << 4));
}
__device__ __forceinline__ uint32_t cnt_get(uint32_t *cntw, int v)
{
    const uint32_t w = __hip_atomic_load(&cntw[rswz(v >> 1)], __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_WORKGROUP);
    return (w >> ((v & 1) << 4)) & 0xFFFFu;
}
#endif

template <int S, int R, bool HOPS, bool PACKED>
__global__ __launch_bounds__(1024) void dfs_runs_kernel(
    int V, int nslot, const uint32_t *__restrict__ g_rows, const uint16_t *__restrict__ radj,
    const uint32_t *__restrict__ deg, const int32_t *__restrict__ row_ptr,
    const int32_t *__restrict__ port, int W, const int32_t *__restrict__ ell_port,
    const int32_t *__restrict__ src, int nsrc, int32_t *__restrict__ out_parent,
    int32_t *__restrict__ out_port, int32_t *__restrict__ out_hops, int *__restrict__ err,
    int flags)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    const RunsLayout L(V, R, HOPS);
    uint32_t *rows = lds;
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    const int nthr = (int)blockDim.x;

    // rows -> LDS, once for every round of this workgroup
    for (int i0 = threadIdx.x; i0 < L.row_words / 4; i0 += kRunsU * nthr) {
        uint4 t[kRunsU];
#pragma unroll
        for (int k = 0; k < kRunsU; ++k) {
            const int i = i0 + k * nthr;
            t[k] = i < L.row_words / 4 ? reinterpret_cast<const uint4 *>(g_rows)[i] : uint4{};
        }
#pragma unroll
        for (int k = 0; k < kRunsU; ++k) {
            const int i = i0 + k * nthr;
            if (i < L.row_words / 4) reinterpret_cast<uint4 *>(rows)[i] = t[k];
        }
    }

    // role: waves 0..nslot-1 search slot w; the rest decrement for slot
    // (w - nslot) / S
    const bool searcher = w < nslot;
    const int q = searcher ? w : (w - nslot) / S;
    const int wk = searcher ? -1 : (w - nslot) % S;           // worker index
    const int role = searcher ? 0 : 1 + wk;                   // epilogue share
    uint32_t *slot = lds + L.row_words + (size_t)q * L.slot_words;
    uint32_t *vis = slot;
    uint32_t *cntw = vis + L.VWp;
    uint16_t *stk = reinterpret_cast<uint16_t *>(cntw + L.CWp);
    uint16_t *ps = reinterpret_cast<uint16_t *>(cntw + L.CWp + L.SWp);
    uint16_t *dep = reinterpret_cast<uint16_t *>(cntw + L.CWp + L.SWp + L.PWp);
    uint16_t *ring = reinterpret_cast<uint16_t *>(cntw + L.CWp + L.SWp + L.PWp + L.DWp);
    int *ctl = reinterpret_cast<int *>(cntw + L.CWp + L.SWp + L.PWp + L.DWp + kRunsRing / 2);
    const int nW = (V + 2) >> 1;                              // count words

    for (int base = blockIdx.x * nslot; base < nsrc; base += gridDim.x * nslot) {
        // -------------------------------------------------------- init
        for (int qq = 0; qq < nslot; ++qq) {
            if (base + qq >= nsrc) break;
            uint32_t *sl = lds + L.row_words + (size_t)qq * L.slot_words;
            uint32_t *cw = sl + L.VWp;
            for (int i = threadIdx.x; i < L.VWp; i += nthr) sl[i] = 0u;
            // counts start at the out-degrees, U word loads in flight
            for (int i0 = threadIdx.x; i0 < nW; i0 += kRunsU * nthr) {
                uint2 dg[kRunsU];
#pragma unroll
                for (int k = 0; k < kRunsU; ++k) {
                    const int i = i0 + k * nthr;
                    dg[k] = i < nW ? reinterpret_cast<const uint2 *>(deg)[i] : uint2{};
                }
#pragma unroll
                for (int k = 0; k < kRunsU; ++k) {
                    const int i = i0 + k * nthr;
#ifndef SDNR_RUNS_C16
                    if (i < nW) {
                        cw[rswz(2 * i)] = dg[k].x;
                        if (2 * i + 1 <= V) cw[rswz(2 * i + 1)] = dg[k].y;
                    }
#else
                    if (i < nW) cw[rswz(i)] = dg[k].x | (dg[k].y << 16);
#endif
                }
            }
            int *ct = reinterpret_cast<int *>(cw + L.CWp + L.SWp + L.PWp + L.DWp + kRunsRing / 2);
            if (threadIdx.x < 2 + S) ct[threadIdx.x] = 0;
        }
        __syncthreads();

        const int si = base + q;
        const int s = si < nsrc ? src[si] : -1;
        int32_t *prow = si < nsrc ? out_parent + (size_t)si * V : nullptr;
        int32_t *trow = (!PACKED && si < nsrc) ? out_port + (size_t)si * V : nullptr;
        int32_t *hrow = (HOPS && si < nsrc) ? out_hops + (size_t)si * V : nullptr;
        const int st = role * 64 + lane, sn = (1 + S) * 64;   // slot-local thread
        if (si >= nsrc) {
            // idle slot
        } else if (s < 0 || s >= V) {
            for (int v = st; v < V; v += sn) {
                prow[v] = -1;                    // packed: 0xFFFFFFFF
                if (!PACKED) trow[v] = -1;
                if (HOPS) hrow[v] = -1;
            }
        } else {
            if (searcher) {
                // ------------------------------------------------ the search
                if (flags & kRunsFlagPrio) __builtin_amdgcn_s_setprio(3);
                if (lane == 0) {
                    vis[s >> 5] |= 1u << (s & 31);
                    vis[V >> 5] |= 1u << (V & 31);
                    ps[rswz(s)] = (uint16_t)s;
                    if (HOPS) dep[s] = 0;
                    stk[0] = (uint16_t)s;
                    ring[0] = (uint16_t)s;           // s's in-neighbours lose one
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_store(&ctl[0], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                int pub = 1, sp = 1, lo = 0;
#ifdef SDNR_STAMPS
                unsigned long long t0 = 0, ta = 0, tb = 0, tc = 0, c_find = 0, c_row = 0,
                                   c_push = 0, n_cand = 0, n_false = 0, n_skip = 0, n_child = 0,
                                   n_lag = 0;
                RSTAMP(t0);
                tc = t0;
#endif
                int nu = -1;                         // next candidate: a new child ...
                uint32_t nd[R];                      // ... and its row words
#pragma unroll
                for (int k = 0; k < R; ++k) nd[k] = 0u;
                for (;;) {
                    int u;
                    uint32_t d[R];
                    if (nu >= 0) {
                        u = nu;
#pragma unroll
                        for (int k = 0; k < R; ++k) d[k] = nd[k];
                        nu = -1;
#ifdef SDNR_STAMPS
                        n_child++;
#endif
                    } else {
                        uint64_t m = 0;
                        int e = V;
                        uint32_t de[R];
#pragma unroll
                        for (int k = 0; k < R; ++k) de[k] = 0u;
                        while (sp > 0) {
#ifdef SDNR_STAMPS
                            n_skip++;
#endif
                            const int kk = sp < 64 ? sp : 64;
                            const int at = sp - 1 - lane;
                            e = stk[at < 0 ? 0 : at];
                            e = lane < kk ? e : V;
                            const uint32_t c = cnt_get(cntw, e);
                            load_desc<R>(rows, e, de);
                            m = __ballot(c != 0u);
                            if (m) break;
                            sp -= kk;
                        }
                        if (!m) break;
                        const int first = __ffsll((unsigned long long)m) - 1;
                        u = read_lane(e, first);
#pragma unroll
                        for (int k = 0; k < R; ++k) d[k] = (uint32_t)read_lane((int)de[k], first);
                        sp -= first + 1;
                    }
                    RSCHED();
#ifdef SDNR_STAMPS
                    RSTAMP(ta);
                    c_find += ta - tc;
                    n_cand++;
                    {
                        int lw = 0x7FFFFFFF;
                        for (int k = 0; k < S; ++k)
                            lw = min(lw, __hip_atomic_load(&ctl[2 + k], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP));
                        n_lag += (unsigned long long)(pub - lw);
                    }
#endif
                    const int x = run_at<R>(d, lane, V);
                    const uint32_t wv = vis[x >> 5];
                    const bool fresh = ((wv >> (x & 31)) & 1u) == 0u;
                    const uint64_t mm = __ballot(fresh);
                    RSCHED();
#ifdef SDNR_STAMPS
                    RSTAMP(tb);
                    c_row += tb - ta;
                    if (mm == 0) {
                        n_false++;
                        tc = tb;
                    }
#endif
                    if (mm == 0) continue;           // stale count: a leaf pop after all
                    const int c = __popcll(mm);
                    const int rank = lanes_below(mm);
                    int du = 0;
                    if (HOPS) du = uniform((int)dep[u]);
                    // back-pressure: ring slots below every worker's progress are free
                    for (unsigned spin = 0; pub + c - lo > kRunsRing; ++spin) {
                        lo = 0x7FFFFFFF;
#pragma unroll
                        for (int k = 0; k < S; ++k)
                            lo = min(lo, __hip_atomic_load(&ctl[2 + k], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP));
                        if (pub + c - lo <= kRunsRing) break;
                        if (spin > kRunsSpin) {
                            if (lane == 0) atomicOr(err, 1);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                    }
                    uint32_t cc = 0u;
                    uint32_t dd[R];
#pragma unroll
                    for (int k = 0; k < R; ++k) dd[k] = 0u;
                    if (fresh) {
                        atomicOr(&vis[x >> 5], 1u << (x & 31));
                        ps[rswz(x)] = (uint16_t)u;
                        if (HOPS) dep[x] = (uint16_t)(du + 1);
                        stk[sp + rank] = (uint16_t)x;
                        ring[(pub + rank) & (kRunsRing - 1)] = (uint16_t)x;
                        // children-first: the new stack top is these children
                        // (highest id on top); their counts and rows now
                        cc = cnt_get(cntw, x);
                        load_desc<R>(rows, x, dd);
                    }
                    const uint64_t mc = __ballot(cc != 0u);
                    pub += c;
                    // the count gather waited for the ring writes (LDS ops
                    // complete in order): an LDS-only release suffices
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                    if (lane == 0) __hip_atomic_store(&ctl[0], pub, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (mc) {
                        // children above the highest one with a count are
                        // leaves (counts are never low): popped; it is next
                        const int hl = highest_lane(mc);
                        nu = read_lane(x, hl);
#pragma unroll
                        for (int k = 0; k < R; ++k) nd[k] = (uint32_t)read_lane((int)dd[k], hl);
                        sp += read_lane(rank, hl);
                    }
                    RSCHED();
#ifdef SDNR_STAMPS
                    RSTAMP(tc);
                    c_push += tc - tb;
#endif
                }
#ifdef SDNR_STAMPS
                RSTAMP(ta);
                RCOUNT(0, ta - t0);
                RCOUNT(1, n_cand);
                RCOUNT(2, n_false);
                RCOUNT(3, n_skip);
                RCOUNT(4, n_child);
                RCOUNT(5, c_find);
                RCOUNT(6, c_row);
                RCOUNT(7, c_push);
                RCOUNT(8, n_lag);
#endif
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_store(&ctl[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (flags & kRunsFlagPrio) __builtin_amdgcn_s_setprio(0);
            } else {
                // ------------------------------------------------ the decrements
                int j = wk;                          // next child index of this worker
                int gmax = (flags >> 8) & 0xFF;         // tuning: children per step
                gmax = gmax == 0 || gmax > kRunsG ? kRunsG : gmax;
                for (unsigned spin = 0;;) {
                    const int P = __hip_atomic_load(&ctl[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                        break;
                    if (j >= P) {
                        // the search is over: the remaining decrements are moot
                        if (__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
                            break;
                        if (++spin > kRunsSpin) {
                            if (lane == 0) atomicOr(err, 2);
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    spin = 0;
                    int n = (P - j + S - 1) / S;
                    if (n > gmax) n = gmax;
                    const int mine = lane < n ? (int)ring[(j + lane * S) & (kRunsRing - 1)] : V;
                    // the in-rows come from L2 (u16, 128 B each, G in flight):
                    // off the search chain, and a load is one instruction
                    // where an LDS run decode is ~25 per child
                    int r[kRunsG];
#pragma unroll
                    for (int g = 0; g < kRunsG; ++g)
                        r[g] = radj[(size_t)read_lane(mine, g) * 64 + lane];   // past n: row V
#pragma unroll
                    for (int g = 0; g < kRunsG; ++g)
                        if (g < n && r[g] != V) cnt_dec(cntw, r[g]);
                    j += n * S;
                    if (lane == 0) __hip_atomic_store(&ctl[2 + wk], j, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                // wait for the search (its visited bits, parents, depths)
                while (!__hip_atomic_load(&ctl[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP))
                    __builtin_amdgcn_s_sleep(2);
            }

            // ---------------------------------------------------- tables
            // the slot's waves: parent, slot (from the parent's runs), port
            // (ELL port table), U vertices per thread in flight
            for (int v0 = st; v0 < V; v0 += kRunsU * sn) {
                int p[kRunsU], sl[kRunsU], pt[kRunsU];
#pragma unroll
                for (int k = 0; k < kRunsU; ++k) {
                    const int v = v0 + k * sn;
                    p[k] = -1;
                    sl[k] = -1;
                    if (v < V && ((vis[v >> 5] >> (v & 31)) & 1u)) {
                        p[k] = (int)ps[rswz(v)];
                        if (v != s) {
                            uint32_t dp[R];
                            load_desc<R>(rows, p[k], dp);
                            sl[k] = run_slot<R>(dp, v);
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < kRunsU; ++k) {
                    pt[k] = -1;
                    if (sl[k] >= 0)
                        pt[k] = W > 0 ? ell_port[(size_t)p[k] * W + sl[k]] : port[row_ptr[p[k]] + sl[k]];
                }
#pragma unroll
                for (int k = 0; k < kRunsU; ++k) {
                    const int v = v0 + k * sn;
                    if (v < V) {
                        if (PACKED) {            // parent | port << 16, -1 -> 0xFFFF
                            prow[v] = (int32_t)(((uint32_t)p[k] & 0xFFFFu) | ((uint32_t)pt[k] << 16));
                        } else {
                            prow[v] = p[k];
                            trow[v] = pt[k];
                        }
                        if (HOPS) hrow[v] = p[k] < 0 ? -1 : (v == s ? 0 : (int)dep[v]);
                    }
                }
            }
        }
        __syncthreads();
    }
}

}  // namespace

// ---------------------------------------------------------------- launcher --

// slots per workgroup and workers per slot: SDNROUTE_DFS_RUNS_SLOTS=1..8,
// SDNROUTE_DFS_RUNS_S=1..3 override (tuning / tests)
static int env_int(const char *name, int lo, int hi, int dflt)
{
    if (const char *f = getenv(name)) {
        const int k = atoi(f);
        if (k >= lo && k <= hi) return k;
    }
    return dflt;
}

bool sdnr_dfs_runs_ok(const sdnr_ctx *ctx, bool hops)
{
    if (!ctx->runs || ctx->V <= 0 || ctx->V >= 65535 || !ctx->deg32 || !ctx->radj16) return false;
    const RunsLayout L(ctx->V, ctx->runs_R, hops);
    return (size_t)(L.row_words + L.slot_words) * 4 <= SDNR_MAX_LDS_PER_BLOCK;
}

int sdnr_launch_dfs_runs(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                         int32_t *d_port, int32_t *d_hops, uint32_t *d_tree)
{
    const int V = ctx->V, R = ctx->runs_R;
    const bool hops = d_hops != nullptr, packed = d_tree != nullptr;
    if (!sdnr_dfs_runs_ok(ctx, hops))
        return sdnr_fail(SDNR_ERR_INVAL, "dfs runs: graph rows do not fit the LDS (V=%d)", V);
    if (packed && !ctx->port16)
        return sdnr_fail(SDNR_ERR_INVAL, "dfs runs: packed tables need 16-bit ports");
    const RunsLayout L(V, R, hops);
    const int lds_slots = (SDNR_LDS_PER_CU / 4 - L.row_words) / L.slot_words;
    // workers per slot: in-rows of <= 32 neighbours need fewer (dfs.hip's
    // dfs_async_waves); slots: the sources each CU must hold at once
    int S = env_int("SDNROUTE_DFS_RUNS_S", 1, 7, ctx->max_indeg <= 32 ? 2 : 3);
    if (S == 4) S = 3;
    if (S == 6) S = 5;
    int ns = (nsrc + ctx->num_cus - 1) / ctx->num_cus;
    ns = env_int("SDNROUTE_DFS_RUNS_SLOTS", 1, 8, ns);
    if (ns > lds_slots) ns = lds_slots;
    if (ns < 1) ns = 1;
    while (ns * (1 + S) > 16 && S > 1) S = S == 7 ? 5 : (S == 5 ? 3 : S - 1);
    if (ns * (1 + S) > 16) ns = 16 / (1 + S);
    const size_t lds = (size_t)(L.row_words + ns * L.slot_words) * 4;
    int bpc = (int)(SDNR_LDS_PER_CU / lds);
    const int wpb = ns * (1 + S);
    if (bpc > 32 / wpb) bpc = 32 / wpb;
    if (bpc < 1) bpc = 1;
    int grid = (nsrc + ns - 1) / ns;
    if (grid > ctx->num_cus * bpc) grid = ctx->num_cus * bpc;
    const int flags = env_int("SDNROUTE_DFS_FLAGS", 0, 1 << 20, kRunsFlagPrio);
    static const char *names[3] = {"dfs_runs_kernel", "dfs_runs_kernel<packed>",
                                   "dfs_runs_kernel<hops>"};
    ctx->last_kernel = packed ? names[1] : (hops ? names[2] : names[0]);
    int32_t *par = packed ? reinterpret_cast<int32_t *>(d_tree) : d_parent;
#define SDNR_RUNS(S_, R_, H_, P_)                                                            \
    do {                                                                                     \
        auto k = dfs_runs_kernel<S_, R_, H_, P_>;                                            \
        sdnr_allow_lds(reinterpret_cast<const void *>(k), lds);                              \
        hipLaunchKernelGGL(k, dim3(grid), dim3(wpb * 64), lds, ctx->stream, V, ns, ctx->runs, \
                           ctx->radj16, ctx->deg32, ctx->row_ptr, ctx->port, ctx->W,          \
                           ctx->ell_port, d_src, nsrc, par, d_port, d_hops, ctx->d_err,      \
                           flags);                                                           \
    } while (0)
#define SDNR_RUNS_L(S_, R_)                                                                  \
    do {                                                                                     \
        if (packed) SDNR_RUNS(S_, R_, false, true);                                          \
        else if (hops) SDNR_RUNS(S_, R_, true, false);                                       \
        else SDNR_RUNS(S_, R_, false, false);                                                \
    } while (0)
#define SDNR_RUNS_R(S_)                                                                      \
    do {                                                                                     \
        if (R == 2) SDNR_RUNS_L(S_, 2); else SDNR_RUNS_L(S_, 4);                             \
    } while (0)
    if (S == 1) SDNR_RUNS_R(1);
    else if (S == 2) SDNR_RUNS_R(2);
    else if (S == 3) SDNR_RUNS_R(3);
    else if (S == 5) SDNR_RUNS_R(5);
    else SDNR_RUNS_R(7);
#undef SDNR_RUNS_R
#undef SDNR_RUNS_L
#undef SDNR_RUNS
    SDNR_HIP(hipGetLastError());
    return SDNR_OK;
}

#ifdef SDNR_STAMPS
extern "C" int sdnr_debug_stamps_runs(unsigned long long *out16)
{
    if (hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_rstamp), 16 * sizeof(unsigned long long)) !=
        hipSuccess)
        return -5;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rstamp), z, sizeof z) == hipSuccess ? 0 : -5;
}
#endif
