// routes.hip -- flow-entry emission from the default-route tables.
//
// SURVEY.md 8(f) 1.  The router installs, for a (src, dst) host pair, one
// OFPFlowMod per switch of find_route(src, dst) (reference
// sdnmpi/router.py:83-104, _add_flows_for_path), and find_route's fdb is the
// tree path of the source's table turned into (switch, out port) pairs by
// _route_to_fdb (sdnmpi/util/topology_db.py:127-138): one entry per hop with
// the port toward the next switch, then the destination switch with the
// host's port (or OFPP_LOCAL).  Batched over many pairs -- every MPI rank
// pair of a job -- that is a ragged array:
//   offsets[i] .. offsets[i+1]   entries of pair i (0 if unreachable),
//   hop_switch[j], hop_port[j]   dense switch id and out port of entry j.
// Pass 1 (route_len_kernel + a three-phase scan) sizes every pair from the
// hop table; pass 2 walks each pair's tree path from the destination up,
// writing entries back to front: route_jump_kernel<16> splits every walk over
// 16 lanes with a 16th-ancestor table (four compositions of the parent
// table), so the lanes of a pair store 16 consecutive entries per step and a
// path of h hops costs ~k + h/16 dependent loads (k < 16: the lane's start);
// route_jump_packed_kernel<16> (the default when V <= 65535 and ports are
// 16-bit) walks a packed copy of the trees (parent | port << 16: one gather
// per entry) with u16 2^j-th-ancestor tables, so lane k reaches its start in
// popcount(k) loads; route_walk_kernel (one lane per pair,
// SDNROUTE_ROUTE_WALK=serial) is the plain form.  The tree rows stay L2 / Infinity-Cache resident; the output is
// written once.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "common.h"

namespace {

constexpr int kScanThreads = 1024;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__global__ __launch_bounds__(256) void route_len_kernel(
    int V, const int32_t *__restrict__ hops, const int32_t *__restrict__ rows,
    const int32_t *__restrict__ dsts, int npairs, int64_t *__restrict__ len)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += gridDim.x * blockDim.x) {
        const int r = rows[i], d = dsts[i];
        int h = -1;
        if (r >= 0 && d >= 0 && d < V) h = hops[(size_t)r * V + d];
        len[i] = h < 0 ? 0 : (int64_t)h + 1;
    }
}

// block-wide exclusive scan of kScanTile values in place; block total out.
// Each thread's kScanItems serially, the thread totals by a wave scan (six
// shuffles), the 16 wave totals through LDS -- two barriers per tile (a
// Hillis-Steele pass over the 1,024 thread totals took twenty).
__device__ int64_t block_scan(int64_t (&v)[kScanItems], int64_t *sh)
{
    int64_t t = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t x = v[k];
        v[k] = t;
        t += x;
    }
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    int64_t incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    constexpr int kWaves = kScanThreads / 64;
    if (lane == 63) sh[wv] = incl;                 // wave totals
    __syncthreads();
    if (wv == 0) {
        int64_t w = lane < kWaves ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < kWaves; o <<= 1) {
            const int64_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < kWaves) sh[kWaves + lane] = w;   // inclusive wave prefixes
    }
    __syncthreads();
    const int64_t wave_excl = wv == 0 ? 0 : sh[kWaves + wv - 1];
    const int64_t total = sh[2 * kWaves - 1];
    const int64_t excl = wave_excl + incl - t;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) v[k] += excl;
    __syncthreads();                               // sh reusable by the caller
    return total;
}

// The same exclusive scan over a tile laid out wave-striped: wave w's lane
// l holds items w * 64 * kScanItems + k * 64 + l, k = 0 .. kScanItems - 1, so
// every load and store instruction of the caller touches 64 consecutive
// elements (with kScanItems consecutive items per thread, each instruction
// spans kScanItems times as many cache lines and the L2 sees as many more
// requests: 8.6 M per 16.7 M-pair chunk of the offsets pass, measured).  Each
// k is a wave scan with a running carry; the wave totals go through LDS.
__device__ int64_t block_scan_striped(int64_t (&v)[kScanItems], int64_t *sh)
{
    const int lane = lane_id(), wv = (int)(threadIdx.x >> 6);
    int64_t carry = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        int64_t incl = v[k];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(incl, o, 64);
            if (lane >= o) incl += y;
        }
        const int64_t x = v[k];
        v[k] = carry + incl - x;
        carry += __shfl(incl, 63, 64);
    }
    constexpr int kWaves = kScanThreads / 64;
    if (lane == 0) sh[wv] = carry;                 // wave totals
    __syncthreads();
    if (wv == 0) {
        int64_t w = lane < kWaves ? sh[lane] : 0;
#pragma unroll
        for (int o = 1; o < kWaves; o <<= 1) {
            const int64_t y = __shfl_up(w, o, 64);
            if (lane >= o) w += y;
        }
        if (lane < kWaves) sh[kWaves + lane] = w;   // inclusive wave prefixes
    }
    __syncthreads();
    const int64_t wave_excl = wv == 0 ? 0 : sh[kWaves + wv - 1];
    const int64_t total = sh[2 * kWaves - 1];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) v[k] += wave_excl;
    __syncthreads();                               // sh reusable by the caller
    return total;
}

// phase 1: scan each tile, tile totals to sums[]
__global__ __launch_bounds__(kScanThreads) void scan_tiles_kernel(int64_t *__restrict__ a, int64_t n,
                                                                  int64_t *__restrict__ sums)
{
    __shared__ int64_t sh[kScanThreads];
    const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
    int64_t v[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) v[k] = base + k < n ? a[base + k] : 0;
    const int64_t tot = block_scan(v, sh);
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + k < n) a[base + k] = v[k];
    if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// phase 2: one block scans the tile totals (any count), grand total to *total
__global__ __launch_bounds__(kScanThreads) void scan_sums_kernel(int64_t *__restrict__ sums, int64_t n,
                                                                 int64_t *__restrict__ total)
{
    __shared__ int64_t sh[kScanThreads];
    int64_t carry = 0;
    for (int64_t t0 = 0; t0 < n; t0 += kScanTile) {
        const int64_t base = t0 + (int64_t)threadIdx.x * kScanItems;
        int64_t v[kScanItems];
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) v[k] = base + k < n ? sums[base + k] : 0;
        const int64_t tot = block_scan(v, sh);
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (base + k < n) sums[base + k] = v[k] + carry;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

// phase 3: add each tile's prefix
__global__ __launch_bounds__(256) void scan_add_kernel(int64_t *__restrict__ a, int64_t n,
                                                       const int64_t *__restrict__ sums)
{
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        a[i] += sums[i / kScanTile];
}

// Offsets in ONE pass (the default): lengths gathered from the hop table,
// scanned per tile, and the tile prefixes chained by a decoupled look-back --
// route_len + scan_tiles + scan_sums + scan_add made four passes over the
// int64 offsets (k=48 all-pairs: 0.23 ms of every 16.7 M-pair chunk).  Tiles
// are numbered by an arrival ticket, so a tile only ever waits for tiles that
// already run; a tile's status word is flag << 62 | value (flag 1: the
// tile's own total, 2: the inclusive prefix through it).  Wave 0 looks back
// 64 tiles at a time.  Every spin is bounded (watchdog code kErrScan).
constexpr uint64_t kStAgg = 1ull << 62, kStPre = 2ull << 62, kStVal = (1ull << 62) - 1;

__global__ __launch_bounds__(kScanThreads) void route_offsets_fused_kernel(
    int V, const int32_t *__restrict__ hops, const int32_t *__restrict__ rows,
    const int32_t *__restrict__ dsts, int64_t n, int64_t *__restrict__ off,
    uint64_t *__restrict__ st, int *__restrict__ err)
{
    __shared__ int64_t sh[kScanThreads];
    __shared__ int64_t s_prefix;
    __shared__ int64_t s_tile;
    if (threadIdx.x == 0)
        s_tile = (int64_t)atomicAdd(reinterpret_cast<unsigned long long *>(&st[0]), 1ull);
    __syncthreads();
    const int64_t tile = s_tile;
    // wave-striped items (block_scan_striped): item k of this lane is base + 64 k
    const int64_t base = tile * kScanTile + (int64_t)(threadIdx.x >> 6) * (64 * kScanItems) +
                         lane_id();
    int64_t v[kScanItems];
    int r[kScanItems], d[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {        // every request load in flight first
        const int64_t i = base + 64 * k;
        r[k] = i < n ? rows[i] : -1;
        d[k] = i < n ? dsts[i] : -1;
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        int h = -1;
        if (r[k] >= 0 && d[k] >= 0 && d[k] < V) h = hops[(size_t)r[k] * V + d[k]];
        v[k] = h < 0 ? 0 : (int64_t)h + 1;
    }
    const int64_t total = block_scan_striped(v, sh);
    uint64_t *status = st + 1;
    if (threadIdx.x < SDNR_WAVE) {
        const int lane = (int)threadIdx.x;
        int64_t prefix = 0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(&status[0], kStPre | (uint64_t)total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&status[tile], kStAgg | (uint64_t)total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = tile - 1;
            for (unsigned spin = 0;;) {
                const int64_t idx = j - lane;
                const uint64_t w = idx >= 0 ? __hip_atomic_load(&status[idx], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_AGENT)
                                            : kStPre;               // before tile 0: prefix 0
                const uint64_t mp = __ballot((w >> 62) == 2u);
                const int fp = mp ? __ffsll((unsigned long long)mp) - 1 : SDNR_WAVE;
                const uint64_t below = fp >= SDNR_WAVE ? ~0ull : ((2ull << fp) - 1ull);
                if (__ballot((w >> 62) == 0u) & below) {            // a needed tile not published
                    if (++spin > (1u << 22)) {
                        if (lane == 0) atomicOr(err, kErrScan);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                int64_t x = lane <= fp ? (int64_t)(w & kStVal) : 0;
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
                prefix += x;
                if (fp < SDNR_WAVE) break;
                j -= SDNR_WAVE;
            }
            if (lane == 0)
                __hip_atomic_store(&status[tile], kStPre | (uint64_t)(prefix + total),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_prefix = prefix;
    }
    __syncthreads();
    const int64_t prefix = s_prefix;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k)
        if (base + 64 * k < n) off[base + 64 * k] = prefix + v[k];
    if (threadIdx.x == 0 && (tile + 1) * kScanTile >= n) off[n] = prefix + total;
}

// anc_out[r][v] = a[r][b[r][v]] (-1 stays -1): composing the parent table
// with itself by doubling gives the 2^j-th ancestor table of every tree
__global__ __launch_bounds__(256) void tree_compose_kernel(int V, size_t n,
                                                           const int32_t *__restrict__ a,
                                                           const int32_t *__restrict__ b,
                                                           int32_t *__restrict__ out)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int32_t x = b[i];
        out[i] = x < 0 ? -1 : a[(i / (size_t)V) * V + x];
    }
}

// P lanes per pair: lane k starts at the k-th ancestor of the destination
// (k parent steps) and then jumps P ancestors at a time, writing the entry of
// each ancestor's parent.  The P lanes of a pair write P consecutive entries
// per step (one 4*P-byte segment per output array instead of P scattered
// words), and a path of h hops takes about k + h/P dependent loads instead of
// h.
template <int P>
__global__ __launch_bounds__(256) void route_jump_kernel(
    int V, const int32_t *__restrict__ parent, const int32_t *__restrict__ port,
    const int32_t *__restrict__ ancP, const int32_t *__restrict__ rows,
    const int32_t *__restrict__ dsts, const int32_t *__restrict__ last_port, int npairs,
    const int64_t *__restrict__ off, int32_t *__restrict__ hop_switch,
    int32_t *__restrict__ hop_port)
{
    const int64_t nthr = (int64_t)npairs * P;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nthr;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(t / P), k = (int)(t % P);
        const int64_t lo = off[i], hi = off[i + 1];
        if (hi <= lo) continue;               // unreachable: no entries
        const int64_t h = hi - lo - 1;        // hops; entry h is the destination
        const size_t rb = (size_t)rows[i] * V;
        int y = dsts[i];
        if (k == 0) {
            hop_switch[lo + h] = y;
            hop_port[lo + h] = last_port[i];
        }
        for (int s = 0; s < k && s < h; ++s) y = parent[rb + y];
        // y = x_u, the ancestor u steps above the destination: its parent's
        // entry (switch, port toward y) goes to index h - u - 1
        for (int64_t u = k; u < h; u += P) {
            hop_switch[lo + h - u - 1] = parent[rb + y];
            hop_port[lo + h - u - 1] = port[rb + y];
            if (u + P < h) y = ancP[rb + y];
        }
    }
}

// Packed form of the walk for V <= 65535 and 16-bit ports: the int32 trees
// are first packed to parent | port << 16 (one 4-byte gather per entry
// instead of two, half the cache footprint) and the 16th-ancestor table is
// u16 (0xFFFF: none).
__global__ __launch_bounds__(256) void tree_pack_kernel(size_t n, const int32_t *__restrict__ parent,
                                                        const int32_t *__restrict__ port,
                                                        uint32_t *__restrict__ tree,
                                                        uint16_t *__restrict__ par16)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const int32_t p = parent[i];
        tree[i] = p < 0 ? 0xFFFFFFFFu : ((uint32_t)p | ((uint32_t)port[i] & 0xFFFFu) << 16);
        par16[i] = p < 0 ? (uint16_t)0xFFFFu : (uint16_t)p;
    }
}

// out[r][v] = a[r][b[r][v]] on u16 ancestor tables (0xFFFF stays 0xFFFF)
__global__ __launch_bounds__(256) void tree_compose16_kernel(int V, size_t n,
                                                             const uint16_t *__restrict__ a,
                                                             const uint16_t *__restrict__ b,
                                                             uint16_t *__restrict__ out)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint16_t x = b[i];
        out[i] = x == 0xFFFFu ? (uint16_t)0xFFFFu : a[(i / (size_t)V) * V + x];
    }
}

struct Anc16 {
    const uint16_t *a[5];    // a[j]: the 2^j-th ancestor (a[0] unused: tree)
};

template <int P>
__global__ __launch_bounds__(256) void route_jump_packed_kernel(
    int V, const uint32_t *__restrict__ tree, Anc16 anc,
    const int32_t *__restrict__ rows, const int32_t *__restrict__ dsts,
    const int32_t *__restrict__ last_port, int npairs, const int64_t *__restrict__ off,
    int32_t *__restrict__ hop_switch, int32_t *__restrict__ hop_port)
{
    const int64_t nthr = (int64_t)npairs * P;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nthr;
         t += (int64_t)gridDim.x * blockDim.x) {
        const int i = (int)(t / P), k = (int)(t % P);
        const int64_t lo = off[i], hi = off[i + 1];
        if (hi <= lo) continue;               // unreachable: no entries
        const int64_t h = hi - lo - 1;        // hops; entry h is the destination
        const size_t rb = (size_t)rows[i] * V;
        int y = dsts[i];
        if (k == 0) {
            hop_switch[lo + h] = y;
            hop_port[lo + h] = last_port[i];
        }
        if (k >= h) continue;
        // k-th ancestor by binary jumps: popcount(k) dependent loads
        if (k & 1) y = (int)(tree[rb + y] & 0xFFFFu);
#pragma unroll
        for (int j = 1; (1 << j) < P; ++j)
            if (k & (1 << j)) y = anc.a[j][rb + y];
        const uint16_t *__restrict__ ancP = anc.a[__builtin_ctz(P)];
        for (int64_t u = k; u < h; u += P) {
            const uint32_t e = tree[rb + y];
            hop_switch[lo + h - u - 1] = (int32_t)(e & 0xFFFFu);
            hop_port[lo + h - u - 1] = (int32_t)(e >> 16);
            if (u + P < h) y = ancP[rb + y];
        }
    }
}

// inclusive prefix sum across the 64 lanes of a wave
__device__ __forceinline__ int wave_incl_scan(int x)
{
    const int lane = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(x, o, 64);
        if (lane >= o) x += t;
    }
    return x;
}

// Entries a run stores one by one before its 16-B body: up to the next
// 128-B line of the output when both arrays share the line phase (the u32
// form: one array), else up to the next 16 B.  A body that starts on a line
// makes every full wave of 16-B stores cover 8 whole lines instead of 9
// partial ones (store probe)
__device__ __forceinline__ int store_head(const uint32_t *o, const uint32_t *op, int total)
{
    const uint32_t m = (op == nullptr || ((((uintptr_t)o ^ (uintptr_t)op) & 127u) == 0)) ? 127u : 15u;
    return min(total, (int)((((m + 1u) - ((uint32_t)(uintptr_t)o & m)) & m) >> 2));
}

// Output-centric expansion (the default for packed trees).  Consecutive
// pairs very often ask for the same (tree row, destination switch) -- every
// host on a switch has the same route from a given source switch, and the
// requests of an all-pairs or rank-pair set come ordered by source, then
// destination -- and then their entries are identical except the last one
// (the destination host's port).  Each wave takes up to 64 consecutive pairs
// (as many as their DISTINCT paths fit its CAP-entry LDS buffer), walks each
// distinct path once into LDS (16 lanes per path, the 2^j-th-ancestor jumps
// of route_jump_packed_kernel), then writes the pairs' entries in order: the
// output range of the group [off[first], off[last + 1]) is contiguous, so the
// stores fill whole cache lines, and the tree gathers drop from one per entry
// to one per distinct path entry.  A pair whose path alone exceeds CAP is
// walked straight to global memory (16 lanes, as the jump kernel).
// OUTP: entries as one u32 each, switch | port << 16 (the tree word layout:
// the LDS buffer is copied as is) instead of two int32 arrays.  V4: a run's
// entries go out as 16-B stores, 4 consecutive entries per lane (per array),
// after a head of single entries to the line (or 16-B) boundary (store_head)
template <int CAP, bool NT, bool OUTP, bool V4 = false>
__global__ __launch_bounds__(256) void route_seg_packed_kernel(
    int V, const uint32_t *__restrict__ tree, Anc16 anc,
    const int32_t *__restrict__ rows, const int32_t *__restrict__ dsts,
    const int32_t *__restrict__ last_port, int npairs, const int64_t *__restrict__ off,
    int32_t *__restrict__ hop_switch, int32_t *__restrict__ hop_port, int *__restrict__ err,
    int diag)
{
    __shared__ uint32_t seg_lds[4][CAP];
    __shared__ int lp_lds[4][64];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    uint32_t *buf = seg_lds[wv];
    int *lps = lp_lds[wv];
    const int groups = (npairs + 63) >> 6;
    const int nwaves = gridDim.x * 4;
    const uint16_t *__restrict__ anc16 = anc.a[4];
    for (int g = blockIdx.x * 4 + wv; g < groups; g += nwaves) {
        const int gend = min(npairs, (g + 1) * 64);
        for (int base = g * 64; base < gend;) {
            const int i = base + lane;
            const bool valid = i < gend;
            int r = -1, d = -1, lp = 0;
            int64_t lo = 0;
            int L = 0;
            if (valid) {
                r = rows[i];
                d = dsts[i];
                lp = last_port[i];
                lo = off[i];
                L = (int)(off[i + 1] - lo);
            }
            // u32 entries hold a 16-bit port: a last (host) port outside
            // [0, 0xFFFF] cannot be written -- fail the call (watchdog code
            // kErrLastPort, reported by sdnr_synchronize) instead of keeping
            // its low bits
            if (OUTP && __ballot(L > 0 && (uint32_t)lp > 0xFFFFu) && lane == 0)
                atomicOr(err, kErrLastPort);
            const int pl = L > 0 ? L - 1 : 0;       // path entries before the last
            const int pr = __shfl_up(r, 1, 64), pd = __shfl_up(d, 1, 64);
            const bool head = valid && (lane == 0 || pr != r || pd != d);
            const int c = head ? pl : 0;
            const int incl = wave_incl_scan(c);
            const int segoff = head ? incl - c : incl - pl;   // followers share the head's
            const uint64_t fit = __ballot(valid && incl <= CAP);
            int n = fit == ~0ull ? 64 : __builtin_ctzll(~fit);   // leading lanes that fit
            if (n == 0) {
                // one pair longer than the buffer: walk it straight to global
                const int64_t lo0 = (int64_t)(uint32_t)read_lane((int)lo, 0) |
                                    ((int64_t)read_lane((int)(lo >> 32), 0) << 32);
                const int h = read_lane(pl, 0);
                const int r0 = read_lane(r, 0);
                const size_t rb = (size_t)r0 * V;
                if (lane < 16) {
                    const int k = lane;
                    int y = read_lane(d, 0);
                    uint32_t *ent = reinterpret_cast<uint32_t *>(hop_switch);
                    if (k == 0) {
                        if (OUTP) {
                            ent[lo0 + h] = (uint32_t)y | ((uint32_t)read_lane(lp, 0) << 16);
                        } else {
                            hop_switch[lo0 + h] = y;
                            hop_port[lo0 + h] = read_lane(lp, 0);
                        }
                    }
                    if (k < h) {
                        if (k & 1) y = (int)(tree[rb + y] & 0xFFFFu);
#pragma unroll
                        for (int j = 1; j < 4; ++j)
                            if (k & (1 << j)) y = anc.a[j][rb + y];
                        for (int u = k; u < h; u += 16) {
                            const uint32_t e = tree[rb + y];
                            if (OUTP) {
                                ent[lo0 + h - u - 1] = e;
                            } else {
                                hop_switch[lo0 + h - u - 1] = (int32_t)(e & 0xFFFFu);
                                hop_port[lo0 + h - u - 1] = (int32_t)(e >> 16);
                            }
                            if (u + 16 < h) y = anc16[rb + y];
                        }
                    }
                }
                base += 1;
                continue;
            }
            // distinct paths of the n pairs, 4 at a time (16 lanes each)
            // diag 1 (timing diagnostic, SDNROUTE_ROUTE_DIAG): no route walks
            uint64_t heads = (diag & 1) ? 0ull : __ballot(head && lane < n && pl > 0);
            while (heads) {
                // the q-th lowest head for lane group q
                const int q = lane >> 4, k = lane & 15;
                uint64_t hm = heads;
                for (int t = 0; t < q && hm; ++t) hm &= hm - 1;
                const int hl = hm ? __builtin_ctzll(hm) : -1;
                const int src_lane = hl < 0 ? 0 : hl;
                const int hr = __shfl(r, src_lane, 64), hd = __shfl(d, src_lane, 64);
                const int h = __shfl(pl, src_lane, 64), so = __shfl(segoff, src_lane, 64);
                if (hl >= 0 && k < h) {
                    const size_t rb = (size_t)hr * V;
                    int y = hd;
                    if (k & 1) y = (int)(tree[rb + y] & 0xFFFFu);
#pragma unroll
                    for (int j = 1; j < 4; ++j)
                        if (k & (1 << j)) y = anc.a[j][rb + y];
                    for (int u = k; u < h; u += 16) {
                        buf[so + h - u - 1] = tree[rb + y];
                        if (u + 16 < h) y = anc16[rb + y];
                    }
                }
                for (int t = 0; t < 4 && heads; ++t) heads &= heads - 1;
            }
            lps[lane] = lp;                          // last ports, read by entry
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // the pairs' entries, in output order, one run of equal (row,
            // destination) pairs at a time: the run's entries are cnt copies
            // of one L-entry route, contiguous, so the lanes stream them with
            // full-wave stores (pair q, entry k of flat index t = q L + k)
            // diag 2 (timing diagnostic): no entry stores
            uint64_t runs = (diag & 2) ? 0ull : __ballot(head && lane < n);
            while (runs) {
                const int p0 = __builtin_ctzll(runs);
                runs &= runs - 1;
                const int p1 = runs ? __builtin_ctzll(runs) : n;
                const int Lr = read_lane(L, p0);
                if (Lr <= 0) continue;
                const int64_t lop = (int64_t)(uint32_t)read_lane((int)lo, p0) |
                                    ((int64_t)read_lane((int)(lo >> 32), p0) << 32);
                const int sop = read_lane(segoff, p0), dp = read_lane(d, p0);
                const int total = (p1 - p0) * Lr;
                const float inv = 1.0f / (float)Lr;
                // (a run shorter than one 16-B pass -- random pairs, one pair
                // per run -- keeps the 4-B stores: head + body + tail would be
                // three partly empty store passes; 1,024-rank flows measured
                // 0.48 -> 0.61 ms with 16-B stores everywhere)
                if (V4 && total >= 256) {
                    // entry at flat index t of the run: pair q = t / Lr, hop k
                    auto qk = [&](int t, int &q, int &k) {
                        q = (int)((float)t * inv);
                        k = t - q * Lr;
                        if (k >= Lr) { ++q; k -= Lr; }
                        if (k < 0) { --q; k += Lr; }
                    };
                    auto word = [&](int q, int k) -> uint32_t {
                        return k < Lr - 1 ? buf[sop + k] : (uint32_t)dp | ((uint32_t)lps[p0 + q] << 16);
                    };
                    // u32 entries, or the switch / port int32 arrays (same
                    // offsets, so one alignment for both)
                    uint32_t *o = reinterpret_cast<uint32_t *>(hop_switch) + lop;
                    uint32_t *op = OUTP ? nullptr : reinterpret_cast<uint32_t *>(hop_port) + lop;
                    // int32 form: switch and port of entry (q, k); the last
                    // entry's port is the request's, any int32
                    auto sw_of = [&](int k) -> uint32_t {
                        return k < Lr - 1 ? (buf[sop + k] & 0xFFFFu) : (uint32_t)dp;
                    };
                    auto pt_of = [&](int q, int k) -> uint32_t {
                        return k < Lr - 1 ? (buf[sop + k] >> 16) : (uint32_t)lps[p0 + q];
                    };
                    auto put1 = [&](int t, int q, int k) {
                        if (OUTP) {
                            o[t] = word(q, k);
                        } else {
                            o[t] = sw_of(k);
                            op[t] = pt_of(q, k);
                        }
                    };
                    const int head = store_head(o, op, total);
                    if (lane < head) {
                        int q, k;
                        qk(lane, q, k);
                        put1(lane, q, k);
                    }
                    const int bend = head + ((total - head) & ~3);
                    for (int t0 = head; t0 < bend; t0 += 256) {
                        const int t = t0 + 4 * lane;
                        if (t < bend) {
                            int q, k;
                            qk(t, q, k);
                            uint32_t a[4], b[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (OUTP) {
                                    a[u] = word(q, k);
                                } else {
                                    a[u] = sw_of(k);
                                    b[u] = pt_of(q, k);
                                }
                                if (++k == Lr) { k = 0; ++q; }
                            }
                            // 16-B aligned (o and op share the offset)
                            *reinterpret_cast<uint4 *>(o + t) = make_uint4(a[0], a[1], a[2], a[3]);
                            if (!OUTP)
                                *reinterpret_cast<uint4 *>(op + t) = make_uint4(b[0], b[1], b[2], b[3]);
                        }
                    }
                    if (bend + lane < total) {
                        int q, k;
                        qk(bend + lane, q, k);
                        put1(bend + lane, q, k);
                    }
                    continue;
                }
                for (int t0 = 0; t0 < total; t0 += 64) {
                    const int t = t0 + lane;
                    if (t < total) {
                        int q = (int)((float)t * inv);
                        int k = t - q * Lr;
                        if (k >= Lr) { ++q; k -= Lr; }
                        if (k < 0) { --q; k += Lr; }
                        int sw, pt;
                        if (OUTP) {
                            const uint32_t e = k < Lr - 1 ? buf[sop + k]
                                                          : (uint32_t)dp | ((uint32_t)lps[p0 + q] << 16);
                            reinterpret_cast<uint32_t *>(hop_switch)[lop + t] = e;
                            continue;
                        }
                        if (k < Lr - 1) {
                            const uint32_t e = buf[sop + k];
                            sw = (int)(e & 0xFFFFu);
                            pt = (int)(e >> 16);
                        } else {
                            sw = dp;
                            pt = lps[p0 + q];
                        }
                        if (NT) {                // streaming: never re-read here
                            __builtin_nontemporal_store(sw, &hop_switch[lop + t]);
                            __builtin_nontemporal_store(pt, &hop_port[lop + t]);
                        } else {
                            hop_switch[lop + t] = sw;
                            hop_port[lop + t] = pt;
                        }
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();        // buffer reused by the next group
            base += n;
        }
    }
}

// Walkers and storers (the default u32 / int32 expansion on packed trees).
// A GCN / CDNA wave's vector-memory counter retires loads AND stores in
// issue order, so in route_seg_packed_kernel every load of the next group
// (its pairs, then each step of a route walk) first waited for the previous
// group's entry stores to be acknowledged -- at the all-pairs write rate,
// microseconds per group (diagnostic: walks alone 9 ms, stores alone 51 ms,
// both 73 ms on k=48).  Here the roles are separate waves of one workgroup:
// NWK walker waves take the 64-pair groups (pairs, distinct routes walked
// into an LDS slot, run descriptors) and never store; NST storer waves take
// full slots and only read LDS and store, so neither kind of wave ever waits
// on the other's memory traffic.  Walker w owns NSL slots (a ring with
// produced / consumed counters in LDS); storer j serves walkers j, j + NST,
// ...  A pair whose route outgrows a slot is walked straight to global
// memory by its walker, as before.  Bounded spins (watchdog kErrSeg).
template <int CAP>
struct SegSlot {
    uint32_t buf[CAP];            // the distinct routes' entries
    int lps[64];                  // last (host) port per pair
    int dlo[64], dhi[64];         // run descriptors by head lane: output offset,
    int dso[64], dL[64], dd[64];  //   route offset in buf, entries per pair, destination
    uint32_t mlo, mhi;            // run heads (lane mask)
    int n;                        // pairs in the slot
};

template <int CAP, bool OUTP, int NWK, int NST, int NSL>
__global__ __launch_bounds__((NWK + NST) * 64) void route_seg_pipe_kernel(
    int V, const uint32_t *__restrict__ tree, Anc16 anc,
    const int32_t *__restrict__ rows, const int32_t *__restrict__ dsts,
    const int32_t *__restrict__ last_port, int npairs, const int64_t *__restrict__ off,
    int32_t *__restrict__ hop_switch, int32_t *__restrict__ hop_port, int *__restrict__ err,
    int diag)
{
    static_assert(NWK % NST == 0, "each storer serves NWK / NST walkers");
    constexpr unsigned kSpin = 1u << 24;
    __shared__ SegSlot<CAP> slots[NWK * NSL];
    __shared__ int prod[NWK], cons[NWK], done[NWK];
    const int lane = lane_id();
    const int w = uniform((int)(threadIdx.x >> 6));
    if (threadIdx.x < NWK) {
        prod[threadIdx.x] = 0;
        cons[threadIdx.x] = 0;
        done[threadIdx.x] = 0;
    }
    __syncthreads();
    const int groups = (npairs + 63) >> 6;
    const uint16_t *__restrict__ anc16 = anc.a[4];
    if (w < NWK) {
        // ------------------------------------------------------ a walker
        int P = 0;
        for (int g = blockIdx.x * NWK + w; g < groups; g += gridDim.x * NWK) {
            const int gend = min(npairs, (g + 1) * 64);
            for (int base = g * 64; base < gend;) {
                const int i = base + lane;
                const bool valid = i < gend;
                int r = -1, d = -1, lp = 0;
                int64_t lo = 0;
                int L = 0;
                if (valid) {
                    r = rows[i];
                    d = dsts[i];
                    lp = last_port[i];
                    lo = off[i];
                    L = (int)(off[i + 1] - lo);
                }
                if (OUTP && __ballot(L > 0 && (uint32_t)lp > 0xFFFFu) && lane == 0)
                    atomicOr(err, kErrLastPort);
                const int pl = L > 0 ? L - 1 : 0;
                const int pr = __shfl_up(r, 1, 64), pd = __shfl_up(d, 1, 64);
                const bool head = valid && (lane == 0 || pr != r || pd != d);
                const int c = head ? pl : 0;
                const int incl = wave_incl_scan(c);
                const int segoff = head ? incl - c : incl - pl;
                const uint64_t fit = __ballot(valid && incl <= CAP);
                const int n = fit == ~0ull ? 64 : __builtin_ctzll(~fit);
                if (n == 0) {
                    // one pair longer than a slot: walked straight to global
                    // memory here (these stores are the walker's own)
                    const int64_t lo0 = (int64_t)(uint32_t)read_lane((int)lo, 0) |
                                        ((int64_t)read_lane((int)(lo >> 32), 0) << 32);
                    const int h = read_lane(pl, 0);
                    const size_t rb = (size_t)read_lane(r, 0) * V;
                    if (lane < 16) {
                        const int k = lane;
                        int y = read_lane(d, 0);
                        uint32_t *ent = reinterpret_cast<uint32_t *>(hop_switch);
                        if (k == 0) {
                            if (OUTP) {
                                ent[lo0 + h] = (uint32_t)y | ((uint32_t)read_lane(lp, 0) << 16);
                            } else {
                                hop_switch[lo0 + h] = y;
                                hop_port[lo0 + h] = read_lane(lp, 0);
                            }
                        }
                        if (k < h) {
                            if (k & 1) y = (int)(tree[rb + y] & 0xFFFFu);
#pragma unroll
                            for (int j = 1; j < 4; ++j)
                                if (k & (1 << j)) y = anc.a[j][rb + y];
                            for (int u = k; u < h; u += 16) {
                                const uint32_t e = tree[rb + y];
                                if (OUTP) {
                                    ent[lo0 + h - u - 1] = e;
                                } else {
                                    hop_switch[lo0 + h - u - 1] = (int32_t)(e & 0xFFFFu);
                                    hop_port[lo0 + h - u - 1] = (int32_t)(e >> 16);
                                }
                                if (u + 16 < h) y = anc16[rb + y];
                            }
                        }
                    }
                    base += 1;
                    continue;
                }
                // a free slot of this walker's ring
                for (unsigned spin = 0;
                     P - __hip_atomic_load(&cons[w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= NSL;
                     ++spin) {
                    if (spin > kSpin) {
                        if (lane == 0) atomicOr(err, kErrSeg);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                SegSlot<CAP> &sl = slots[w * NSL + P % NSL];
                // distinct paths of the n pairs, 4 at a time (16 lanes each)
                // (diag 1, timing only: no route walks)
                uint64_t heads = (diag & 1) ? 0ull : __ballot(head && lane < n && pl > 0);
                while (heads) {
                    const int q = lane >> 4, k = lane & 15;
                    uint64_t hm = heads;
                    for (int t = 0; t < q && hm; ++t) hm &= hm - 1;
                    const int hl = hm ? __builtin_ctzll(hm) : -1;
                    const int src_lane = hl < 0 ? 0 : hl;
                    const int hr = __shfl(r, src_lane, 64), hd = __shfl(d, src_lane, 64);
                    const int h = __shfl(pl, src_lane, 64), so = __shfl(segoff, src_lane, 64);
                    if (hl >= 0 && k < h) {
                        const size_t rb = (size_t)hr * V;
                        int y = hd;
                        if (k & 1) y = (int)(tree[rb + y] & 0xFFFFu);
#pragma unroll
                        for (int j = 1; j < 4; ++j)
                            if (k & (1 << j)) y = anc.a[j][rb + y];
                        for (int u = k; u < h; u += 16) {
                            sl.buf[so + h - u - 1] = tree[rb + y];
                            if (u + 16 < h) y = anc16[rb + y];
                        }
                    }
                    for (int t = 0; t < 4 && heads; ++t) heads &= heads - 1;
                }
                sl.lps[lane] = lp;
                const uint64_t runs = __ballot(head && lane < n);
                if (head && lane < n) {
                    sl.dlo[lane] = (int)(uint32_t)lo;
                    sl.dhi[lane] = (int)(lo >> 32);
                    sl.dso[lane] = segoff;
                    sl.dL[lane] = L;
                    sl.dd[lane] = d;
                }
                if (lane == 0) {
                    sl.mlo = (uint32_t)runs;
                    sl.mhi = (uint32_t)(runs >> 32);
                    sl.n = n;
                }
                ++P;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
                if (lane == 0) __hip_atomic_store(&prod[w], P, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                base += n;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) __hip_atomic_store(&done[w], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    // ---------------------------------------------------------- a storer
    constexpr int PER = NWK / NST;                // walkers served
    const int js = w - NWK;
    int C[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) C[q] = 0;
    for (unsigned spin = 0;;) {
        bool progress = false, finished = true;
#pragma unroll
        for (int q = 0; q < PER; ++q) {
            const int ww = js + q * NST;
            const int dn = __hip_atomic_load(&done[ww], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int Pw = __hip_atomic_load(&prod[ww], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (C[q] >= Pw) {
                finished = finished && dn;
                continue;
            }
            finished = false;
            progress = true;
            const SegSlot<CAP> &sl = slots[ww * NSL + C[q] % NSL];
            const int n = sl.n;
            // (diag 2, timing only: no entry stores)
            uint64_t runs = (diag & 2) ? 0ull : ((uint64_t)sl.mlo | ((uint64_t)sl.mhi << 32));
            while (runs) {
                const int p0 = __builtin_ctzll(runs);
                runs &= runs - 1;
                const int p1 = runs ? __builtin_ctzll(runs) : n;
                const int Lr = sl.dL[p0];
                if (Lr <= 0) continue;
                const int64_t lop = (int64_t)(uint32_t)sl.dlo[p0] | ((int64_t)sl.dhi[p0] << 32);
                const int sop = sl.dso[p0], dp = sl.dd[p0];
                const int total = (p1 - p0) * Lr;
                const float inv = 1.0f / (float)Lr;
                auto qk = [&](int t, int &q2, int &k) {
                    q2 = (int)((float)t * inv);
                    k = t - q2 * Lr;
                    if (k >= Lr) { ++q2; k -= Lr; }
                    if (k < 0) { --q2; k += Lr; }
                };
                auto sw_of = [&](int k) -> uint32_t {
                    return k < Lr - 1 ? (sl.buf[sop + k] & 0xFFFFu) : (uint32_t)dp;
                };
                auto pt_of = [&](int q2, int k) -> uint32_t {
                    return k < Lr - 1 ? (sl.buf[sop + k] >> 16) : (uint32_t)sl.lps[p0 + q2];
                };
                auto word = [&](int q2, int k) -> uint32_t {
                    return k < Lr - 1 ? sl.buf[sop + k] : (uint32_t)dp | ((uint32_t)sl.lps[p0 + q2] << 16);
                };
                uint32_t *o = reinterpret_cast<uint32_t *>(hop_switch) + lop;
                uint32_t *op = OUTP ? nullptr : reinterpret_cast<uint32_t *>(hop_port) + lop;
                auto put1 = [&](int t) {
                    int q2, k;
                    qk(t, q2, k);
                    if (OUTP) {
                        o[t] = word(q2, k);
                    } else {
                        o[t] = sw_of(k);
                        op[t] = pt_of(q2, k);
                    }
                };
                // 16-B stores of 4 entries per lane when the run fills a
                // pass and both arrays share the 16-B phase (int32 form)
                const bool v4 = total >= 256 &&
                                (OUTP || ((((uintptr_t)o ^ (uintptr_t)op) & 15u) == 0));
                if (v4) {
                    const int hd = store_head(o, op, total);
                    if (lane < hd) put1(lane);
                    const int bend = hd + ((total - hd) & ~3);
                    for (int t0 = hd; t0 < bend; t0 += 256) {
                        const int t = t0 + 4 * lane;
                        if (t < bend) {
                            int q2, k;
                            qk(t, q2, k);
                            uint32_t a[4], b[4];
#pragma unroll
                            for (int u = 0; u < 4; ++u) {
                                if (OUTP) {
                                    a[u] = word(q2, k);
                                } else {
                                    a[u] = sw_of(k);
                                    b[u] = pt_of(q2, k);
                                }
                                if (++k == Lr) { k = 0; ++q2; }
                            }
                            *reinterpret_cast<uint4 *>(o + t) = make_uint4(a[0], a[1], a[2], a[3]);
                            if (!OUTP)
                                *reinterpret_cast<uint4 *>(op + t) = make_uint4(b[0], b[1], b[2], b[3]);
                        }
                    }
                    if (bend + lane < total) put1(bend + lane);
                } else {
                    for (int t0 = 0; t0 < total; t0 += 64)
                        if (t0 + lane < total) put1(t0 + lane);
                }
            }
            ++C[q];
            // the slot's LDS reads are done (their values are in the store
            // registers): hand it back
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
            if (lane == 0) __hip_atomic_store(&cons[ww], C[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (finished) break;
        if (progress) {
            spin = 0;
        } else {
            if (++spin > kSpin) {
                if (lane == 0) atomicOr(err, kErrSeg);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

__global__ __launch_bounds__(256) void route_walk_kernel(
    int V, const int32_t *__restrict__ parent, const int32_t *__restrict__ port,
    const int32_t *__restrict__ rows, const int32_t *__restrict__ dsts,
    const int32_t *__restrict__ last_port, int npairs, const int64_t *__restrict__ off,
    int32_t *__restrict__ hop_switch, int32_t *__restrict__ hop_port)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npairs; i += gridDim.x * blockDim.x) {
        int64_t lo = off[i], j = off[i + 1] - 1;
        if (j < lo) continue;                 // unreachable: no entries
        const size_t rb = (size_t)rows[i] * V;
        int x = dsts[i];
        hop_switch[j] = x;
        hop_port[j] = last_port[i];
        // parent and port of x: the switch before x and its port toward x
        while (j > lo) {
            const int p = parent[rb + x];
            const int pt = port[rb + x];
            --j;
            hop_switch[j] = p;
            hop_port[j] = pt;
            x = p;
        }
    }
}

// Flood-port test of TopologyManager._is_edge_port (reference
// sdnmpi/topology.py:150-155, used by _do_broadcast :157-177): a switch port
// is an edge port iff it is neither end of any link.  Keys are (dense switch
// id << 32 | port_no); the link ends arrive sorted, so each port is one
// binary search instead of the reference's scan over every link.
__global__ __launch_bounds__(256) void edge_port_kernel(const uint64_t *__restrict__ ends, int nends,
                                                         const uint64_t *__restrict__ ports,
                                                         int nports, uint8_t *__restrict__ is_edge)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nports; i += gridDim.x * blockDim.x) {
        const uint64_t k = ports[i];
        int lo = 0, hi = nends;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (ends[mid] < k) lo = mid + 1; else hi = mid;
        }
        is_edge[i] = (lo < nends && ends[lo] == k) ? 0 : 1;
    }
}

}  // namespace

int sdnr_launch_route_offsets(sdnr_ctx *ctx, const int32_t *d_hops, const int32_t *d_rows,
                              const int32_t *d_dsts, int32_t npairs, int64_t *d_off)
{
    // offsets[0..npairs]: lengths into off[0..npairs), exclusive scan, the
    // total into off[npairs]
    const int V = ctx->V;
    const int64_t n = npairs;
    if (n == 0) {
        SDNR_HIP(hipMemsetAsync(d_off, 0, sizeof(int64_t), ctx->stream));
        return SDNR_OK;
    }
    const int64_t tiles = (n + kScanTile - 1) / kScanTile;
    int rc = sdnr_reserve(&ctx->scratch, &ctx->scratch_bytes, (size_t)(tiles + 1) * 8);
    if (rc) return rc;
    // one pass (SDNROUTE_ROUTE_SCAN=4: the four-kernel form, A/B)
    const char *sf = getenv("SDNROUTE_ROUTE_SCAN");
    if (!(sf && !strcmp(sf, "4"))) {
        uint64_t *st = static_cast<uint64_t *>(ctx->scratch);
        SDNR_HIP(hipMemsetAsync(st, 0, (size_t)(tiles + 1) * 8, ctx->stream));
        hipLaunchKernelGGL(route_offsets_fused_kernel, dim3((unsigned)tiles), dim3(kScanThreads), 0,
                           ctx->stream, V, d_hops, d_rows, d_dsts, n, d_off, st, ctx->d_err);
        SDNR_HIP(hipGetLastError());
        return SDNR_OK;
    }
    int64_t *sums = static_cast<int64_t *>(ctx->scratch);
    int g = (int)((n + 255) / 256);
    if (g > ctx->num_cus * 16) g = ctx->num_cus * 16;
    hipLaunchKernelGGL(route_len_kernel, dim3(g), dim3(256), 0, ctx->stream, V, d_hops, d_rows,
                       d_dsts, npairs, d_off);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)tiles), dim3(kScanThreads), 0, ctx->stream,
                       d_off, n, sums);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanThreads), 0, ctx->stream, sums, tiles,
                       d_off + n);
    hipLaunchKernelGGL(scan_add_kernel, dim3(g), dim3(256), 0, ctx->stream, d_off, n, sums);
    SDNR_HIP(hipGetLastError());
    return SDNR_OK;
}

int sdnr_launch_route_expand(sdnr_ctx *ctx, const int32_t *d_parent, const int32_t *d_port,
                             int32_t nrows, const int32_t *d_rows, const int32_t *d_dsts,
                             const int32_t *d_last_port, int32_t npairs, const int64_t *d_off,
                             int32_t *d_switch, int32_t *d_hport, uint32_t *d_entries,
                             bool same_tables)
{
    if (npairs == 0) return SDNR_OK;
    if (d_entries && !(ctx->V <= 0xFFFF && ctx->port16))
        return sdnr_fail(SDNR_ERR_INVAL, "route entries as u32 need V <= 65535 and 16-bit ports");
    const char *f = getenv("SDNROUTE_ROUTE_WALK");      // "serial": one lane per pair
    const bool serial = f && !strcmp(f, "serial");
    const size_t n = (size_t)nrows * (size_t)ctx->V;
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    const char *pk = getenv("SDNROUTE_ROUTE_PACKED");          // "0": int32 tables
    const bool packed = d_entries ||
                        (!serial && ctx->V <= 0xFFFF && ctx->port16 && !(pk && !strcmp(pk, "0")));
    if (packed) {
        // walk tables (14n bytes, a buffer of their own): tree u32 [n] | u16
        // ancestor tables a1..a16 [n]; rebuilt unless the caller says the
        // tables are the previous call's (SDNR_SAME_TABLES) and they match
        const bool reuse = same_tables && ctx->anc_valid && ctx->anc_parent == d_parent &&
                           ctx->anc_port == d_port && ctx->anc_n == n;
        if (!reuse) {
            // invalid until the rebuild below is launched: a failed reserve
            // (which frees the old buffer) or launch must not leave a later
            // SDNR_SAME_TABLES call matching the old tables
            ctx->anc_valid = false;
            int rc = sdnr_reserve(&ctx->anc, &ctx->anc_bytes, 14 * n + 64);
            if (rc) return rc;
        }
        uint32_t *tree = static_cast<uint32_t *>(ctx->anc);
        uint16_t *a16 = reinterpret_cast<uint16_t *>(tree + n);
        const int cg = ctx->num_cus * 8;
        Anc16 tabs{};
        for (int j = 1; j <= 4; ++j) tabs.a[j] = a16 + (size_t)j * n;
        if (!reuse) {
            hipLaunchKernelGGL(tree_pack_kernel, dim3(cg), dim3(256), 0, ctx->stream, n, d_parent,
                               d_port, tree, a16);
            for (int j = 1; j <= 4; ++j) {
                const uint16_t *prev = a16 + (size_t)(j - 1) * n;
                hipLaunchKernelGGL(tree_compose16_kernel, dim3(cg), dim3(256), 0, ctx->stream,
                                   ctx->V, n, prev, prev, a16 + (size_t)j * n);
            }
            SDNR_HIP(hipGetLastError());
            ctx->anc_parent = d_parent;
            ctx->anc_port = d_port;
            ctx->anc_n = n;
            ctx->anc_valid = true;
        }
        const char *sg = getenv("SDNROUTE_ROUTE_SEG");        // "0": per-entry jump walks
        if (d_entries || !(sg && !strcmp(sg, "0"))) {
            // 4 waves per workgroup, one 64-pair group per wave at a time
            int64_t g = (((int64_t)npairs + 63) / 64 + 3) / 4;
            int wpc = 8;                                  // workgroups per CU
            if (const char *gf = sdnr_tune_env("SDNROUTE_ROUTE_WGS")) wpc = atoi(gf) > 0 ? atoi(gf) : 8;
            if (g > ctx->num_cus * wpc) g = ctx->num_cus * wpc;
            const char *nt = sdnr_tune_env("SDNROUTE_ROUTE_NT");       // "1": non-temporal stores
            // 16-B stores of 4 entries per lane (SDNROUTE_ROUTE_V4=0: 4-B stores)
            const char *v4 = getenv("SDNROUTE_ROUTE_V4");
#ifdef SDNR_DIAG_VARIANTS
            // timing only (the entries are then wrong): 1 no walks, 2 no stores
            const char *dg = getenv("SDNROUTE_ROUTE_DIAG");
            const int diag = dg ? atoi(dg) : 0;
#else
            const int diag = 0;                 // never in the product library
#endif
            // walker / storer waves (route_seg_pipe_kernel): SDNROUTE_ROUTE_PIPE=0
            // keeps the one-role kernel, "W,S,N" picks walkers, storers and
            // slots per walker among the compiled shapes
            // k=48 all-pairs u32 entries, same box (gpurun_out/r5_f, r5_h): 2,2,4
            // 69.1-69.3 ms, 2,2,3 69.1-69.5; one-role 73.6-73.9; 4,4,2 73.3-73.6;
            // 8,4,2 72.2; 2,2,2 78.8; 3,3,2 79.6; 2,1,3 79.8; 4,2,2 92.3;
            // 1,1,4 91.8; 6,2,2 91.5; 6,3,2 107.6; 4,2,3 144.7.  The int32 form
            // gains nothing (116.4 one-role, 115.6 at 2,2,4) and short runs of
            // random rank pairs lose (1,024-rank flows 0.50 -> 0.61 ms), so the
            // pipeline serves large u32 batches only
            int pw = 2, ps = 2, pn = 4;
            bool pipe = d_entries && npairs >= (1 << 22) && !(v4 && !strcmp(v4, "0")) &&
                        !(nt && !strcmp(nt, "1")) && !diag;
            if (const char *pp = getenv("SDNROUTE_ROUTE_PIPE")) {
                if (!strcmp(pp, "0")) pipe = false;
                else if (sscanf(pp, "%d,%d,%d", &pw, &ps, &pn) == 3) pipe = true;   // diag too
            }
            if (pipe) {
                bool launched = false;
#define SDNR_PIPE(W_, S_, N_)                                                                 \
    if (!launched && pw == W_ && ps == S_ && pn == N_) {                                     \
        constexpr size_t kL = sizeof(SegSlot<512>) * W_ * N_;                                \
        size_t per_cu = SDNR_LDS_PER_CU / (kL + 256);                                        \
        if (per_cu > (size_t)(32 / (W_ + S_))) per_cu = 32 / (W_ + S_);                       \
        if (per_cu < 1) per_cu = 1;                                                          \
        int64_t pg = (((int64_t)npairs + 63) / 64 + W_ - 1) / W_;                            \
        if (pg > (int64_t)ctx->num_cus * (int64_t)per_cu) pg = (int64_t)ctx->num_cus * per_cu; \
        if (d_entries)                                                                       \
            hipLaunchKernelGGL((route_seg_pipe_kernel<512, true, W_, S_, N_>), dim3((unsigned)pg), \
                               dim3((W_ + S_) * 64), 0, ctx->stream, ctx->V, tree, tabs, d_rows, \
                               d_dsts, d_last_port, npairs, d_off,                           \
                               reinterpret_cast<int32_t *>(d_entries), nullptr, ctx->d_err, diag); \
        else                                                                                 \
            hipLaunchKernelGGL((route_seg_pipe_kernel<512, false, W_, S_, N_>), dim3((unsigned)pg), \
                               dim3((W_ + S_) * 64), 0, ctx->stream, ctx->V, tree, tabs, d_rows, \
                               d_dsts, d_last_port, npairs, d_off, d_switch, d_hport, ctx->d_err, diag); \
        launched = true;                                                                     \
    }
                SDNR_PIPE(4, 2, 2)
                SDNR_PIPE(4, 4, 2)
                SDNR_PIPE(6, 2, 2)
                SDNR_PIPE(4, 2, 3)
                SDNR_PIPE(2, 2, 3)
                SDNR_PIPE(8, 4, 2)
                SDNR_PIPE(6, 3, 2)
                SDNR_PIPE(2, 2, 2)
                SDNR_PIPE(2, 2, 4)
                SDNR_PIPE(1, 1, 4)
                SDNR_PIPE(3, 3, 2)
                SDNR_PIPE(2, 1, 3)
#undef SDNR_PIPE
                if (!launched) return sdnr_fail(SDNR_ERR_INVAL, "SDNROUTE_ROUTE_PIPE=%d,%d,%d: no such shape", pw, ps, pn);
                ctx->last_kernel = d_entries ? "route_seg_pipe_kernel<u32>" : "route_seg_pipe_kernel<int32>";
                SDNR_HIP(hipGetLastError());
                if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
                return SDNR_OK;
            }
            if (d_entries) {
                ctx->last_kernel = "route_seg_packed_kernel<1024,u32>";
                if (v4 && !strcmp(v4, "0"))
                    hipLaunchKernelGGL((route_seg_packed_kernel<1024, false, true, false>),
                                       dim3((unsigned)g), dim3(256), 0, ctx->stream, ctx->V, tree,
                                       tabs, d_rows, d_dsts, d_last_port, npairs, d_off,
                                       reinterpret_cast<int32_t *>(d_entries), nullptr, ctx->d_err, diag);
                else
                    hipLaunchKernelGGL((route_seg_packed_kernel<1024, false, true, true>),
                                       dim3((unsigned)g), dim3(256), 0, ctx->stream, ctx->V, tree,
                                       tabs, d_rows, d_dsts, d_last_port, npairs, d_off,
                                       reinterpret_cast<int32_t *>(d_entries), nullptr, ctx->d_err, diag);
            } else {
                ctx->last_kernel = "route_seg_packed_kernel<1024>";
                if (nt && !strcmp(nt, "1"))
                    hipLaunchKernelGGL((route_seg_packed_kernel<1024, true, false>), dim3((unsigned)g),
                                       dim3(256), 0, ctx->stream, ctx->V, tree, tabs, d_rows, d_dsts,
                                       d_last_port, npairs, d_off, d_switch, d_hport, nullptr, diag);
                else if ((((uintptr_t)d_switch ^ (uintptr_t)d_hport) & 15u) == 0 && !(v4 && !strcmp(v4, "0")))
                    // both arrays share their 16-B phase: 16-B stores into each
                    hipLaunchKernelGGL((route_seg_packed_kernel<1024, false, false, true>),
                                       dim3((unsigned)g), dim3(256), 0, ctx->stream, ctx->V, tree,
                                       tabs, d_rows, d_dsts, d_last_port, npairs, d_off, d_switch,
                                       d_hport, nullptr, diag);
                else
                    hipLaunchKernelGGL((route_seg_packed_kernel<1024, false, false>), dim3((unsigned)g),
                                       dim3(256), 0, ctx->stream, ctx->V, tree, tabs, d_rows, d_dsts,
                                       d_last_port, npairs, d_off, d_switch, d_hport, nullptr, diag);
            }
        } else {
            int64_t g = ((int64_t)npairs * 16 + 255) / 256;
            if (g > ctx->num_cus * 16) g = ctx->num_cus * 16;
            ctx->last_kernel = "route_jump_packed_kernel<16>";
            hipLaunchKernelGGL(route_jump_packed_kernel<16>, dim3((unsigned)g), dim3(256), 0,
                               ctx->stream, ctx->V, tree, tabs, d_rows, d_dsts, d_last_port,
                               npairs, d_off, d_switch, d_hport);
        }
    } else if (serial) {
        int g = (npairs + 255) / 256;
        if (g > ctx->num_cus * 16) g = ctx->num_cus * 16;
        ctx->last_kernel = "route_walk_kernel";
        hipLaunchKernelGGL(route_walk_kernel, dim3(g), dim3(256), 0, ctx->stream, ctx->V, d_parent,
                           d_port, d_rows, d_dsts, d_last_port, npairs, d_off, d_switch, d_hport);
    } else {
        // int32 ancestor tables in scratch2 (2 x n int32)
        int rc = sdnr_reserve(&ctx->scratch2, &ctx->scratch2_bytes, 8 * n + 64);
        if (rc) return rc;
        int32_t *anc = static_cast<int32_t *>(ctx->scratch2);
        int32_t *tmp = anc + n;
        // P-th ancestors by doubling: p2 = p o p, p4 = p2 o p2, ...
        // SDNROUTE_ROUTE_P=4|8|16 lanes per pair (default 16: k=48 1M rank
        // pairs 0.57 ms at 8, 0.54 ms at 16, 0.75 ms at 4)
        const char *pf = getenv("SDNROUTE_ROUTE_P");
        const int P = pf && (atoi(pf) == 4 || atoi(pf) == 8) ? atoi(pf) : 16;
        const int cg = ctx->num_cus * 8;
        const int32_t *cur = d_parent;
        int32_t *bufs[2] = {tmp, anc};
        int which = 0;
        for (int q = 1; q < P; q <<= 1) {
            hipLaunchKernelGGL(tree_compose_kernel, dim3(cg), dim3(256), 0, ctx->stream, ctx->V,
                               n, cur, cur, bufs[which]);
            cur = bufs[which];
            which ^= 1;
        }
        int64_t g = ((int64_t)npairs * P + 255) / 256;
        if (g > ctx->num_cus * 16) g = ctx->num_cus * 16;
#define SDNR_JUMP(P_)                                                                        \
    hipLaunchKernelGGL(route_jump_kernel<P_>, dim3((unsigned)g), dim3(256), 0, ctx->stream,  \
                       ctx->V, d_parent, d_port, cur, d_rows, d_dsts, d_last_port, npairs,   \
                       d_off, d_switch, d_hport)
        if (P == 4) {
            ctx->last_kernel = "route_jump_kernel<4>";
            SDNR_JUMP(4);
        } else if (P == 8) {
            ctx->last_kernel = "route_jump_kernel<8>";
            SDNR_JUMP(8);
        } else {
            ctx->last_kernel = "route_jump_kernel<16>";
            SDNR_JUMP(16);
        }
#undef SDNR_JUMP
    }
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}

int sdnr_launch_edge_ports(sdnr_ctx *ctx, const uint64_t *d_ends, int32_t nends,
                           const uint64_t *d_ports, int32_t nports, uint8_t *d_is_edge)
{
    if (nports == 0) return SDNR_OK;
    int g = (nports + 255) / 256;
    if (g > ctx->num_cus * 8) g = ctx->num_cus * 8;
    ctx->last_kernel = "edge_port_kernel";
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
    hipLaunchKernelGGL(edge_port_kernel, dim3(g), dim3(256), 0, ctx->stream, d_ends, nends, d_ports,
                       nports, d_is_edge);
    SDNR_HIP(hipGetLastError());
    if (ctx->timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
    return SDNR_OK;
}
