// common.h -- shared device helpers and the context layout of libsdnroute.
// gfx950 (CDNA4) only: 64-lane wavefronts, 160 KiB LDS per CU, 256 CUs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/sdnroute.h"

#define SDNR_WAVE 64
#define SDNR_LDS_PER_CU (160 * 1024)
#define SDNR_MAX_LDS_PER_BLOCK (160 * 1024)

// ---------------------------------------------------------------- device --

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// number of set bits of m strictly below this lane
__device__ __forceinline__ int lanes_below(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int uniform(int x) {
    return __builtin_amdgcn_readfirstlane(x);
}

__device__ __forceinline__ int read_lane(int x, int lane) {
    return __builtin_amdgcn_readlane(x, lane);
}

__device__ __forceinline__ int highest_lane(uint64_t m) { return 63 - __clzll(m); }

// LDS bank swizzle for per-vertex u32 arrays indexed by neighbour ids: rows of
// structured fabrics hold strided ids (a fat-tree core's neighbours are 24
// apart: 8-way bank conflicts); x ^ ((x >> 3) & 31) is a bijection inside
// every 256-entry block and spreads those rows over all 32 banks.  Arrays
// indexed this way are sized in whole 256-entry blocks.
__device__ __forceinline__ int lds_swz(int x) { return x ^ ((x >> 3) & 31); }

// ------------------------------------------------------------------ host --

struct sdnr_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;

    // graph (device)
    int32_t V = -1, E = 0, max_deg = 0;
    int32_t max_indeg = 0x7FFFFFFF;     // maximum in-degree (set with adj16/radj16)
    int32_t W = 0;                      // ELL row width (0: CSR only)
    int32_t *row_ptr = nullptr, *col = nullptr, *port = nullptr;
    int32_t *ell_col = nullptr, *ell_port = nullptr;
    uint16_t *ell16 = nullptr;          // ELL ids as u16 (low 16 bits when V > 65535), 0xFFFF pad
    uint32_t *ell_hi = nullptr;         // per row: the 17th id bit of each slot (65535 <= V < 131071)
    // dictionary rows for the split DFS (V <= 65535, rows of <= 8 slots):
    // row u = u + dict_off[p(u) * 8 + slot], p(u) = byte (u & 31) of block
    // tuple dict_bt[b(u)] (32 pattern bytes = 8 u32 words), b(u) = byte
    // u >> 5 of dict_bp (4 block ids per u32 word, dict_bpw words); dict_off
    // dict_P x 8 int32 offsets (padding slots: kDictPad)
    uint32_t *dict_bp = nullptr;
    uint32_t *dict_bt = nullptr;
    int32_t *dict_off = nullptr;
    int32_t dict_P = 0, dict_NB = 0, dict_bpw = 0;
    uint16_t *adj16 = nullptr;          // (V+1) rows x 64 u16, sentinel V (V < 65535)
    uint16_t *radj16 = nullptr;         // in-neighbour rows, same layout (== adj16 if symmetric)
    uint32_t *deg32 = nullptr;          // out-degrees of 0..V (sentinel V: 0)
    uint16_t *radjw = nullptr;          // radj16 as swizzled count indices (async DFS workers)
    uint16_t *radjc = nullptr;          // ... for the compact-LDS form (word << 1 | half)
    bool radj_owned = false;
    // in-degree <= 32: the pre-swizzled rows (radjw / radjc) repeat their 32
    // entries in lanes 32..63, so one 64-lane load + ds_sub covers 2 children
    bool radj_pair = false;
    // out-rows as arithmetic runs (dfs_runs.hip): (V+1) rows x runs_R words
    // of start | stride << 16 | count << 25
    uint32_t *runs = nullptr;
    int32_t runs_R = 0;
    // bitmap rows for the register-visited DFS (dfs_bits.hip, V <= 4096):
    // adjb[u * 64 + l] = bits of u's out-neighbours 64l..64l+63, adjp the
    // exclusive prefix popcount of lane blocks (u8), radjx[v * 64 + i] =
    // swizzled count index | in-neighbour << 16 (padding: dummy | 0xFFFF << 16;
    // row V all padding)
    uint64_t *adjb = nullptr;
    uint8_t *adjp = nullptr;
    uint32_t *radjx = nullptr;

    // grow-only device scratch / staging
    void *scratch = nullptr;
    size_t scratch_bytes = 0;
    void *stage = nullptr;
    size_t stage_bytes = 0;
    void *scratch2 = nullptr;           // int32 tables behind a packed-table call
    size_t scratch2_bytes = 0;
    void *wq = nullptr;                 // source work queue of the split DFS (kFlagCuMap)
    size_t wq_bytes = 0;
    void *dmat = nullptr;               // V x V distances behind APSP-derived shortest tables
    size_t dmat_bytes = 0;
    // the route expansion's walk tables (packed trees + u16 ancestor tables)
    // and what they were built from (SDNR_SAME_TABLES reuses them)
    void *anc = nullptr;
    size_t anc_bytes = 0;
    const void *anc_parent = nullptr, *anc_port = nullptr;
    size_t anc_n = 0;
    bool anc_valid = false;
    bool port16 = false;                // every port fits the packed layout (< 0xFFFF)
    bool symmetric = false;             // every link (u, v) has its reverse (v, u)

    // timing of the main kernel(s) of the last SDNR_TIMING call
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    const char *last_kernel = "";       // variant launched by the last table call
    int32_t last_launches = 0;          // main-kernel launches of the last table call
    int32_t last_sweeps = 0;            // Bellman-Ford sweeps of the last APSP call
    int32_t plane_depth = 0;            // levels the bit-plane BFS last needed on this graph
    int *d_err = nullptr;               // kernel watchdog word (0 = ok)
    int *h_flag = nullptr;              // pinned host words for level-loop checks
    int *h_pub = nullptr;               // coherent host words a kernel publishes into
    int pub_seq = 0;                    // sequence number of the last publication
    hipEvent_t ev_flag = nullptr;       // ... and the event the host spins on

    // multi-device context (sdnr_create_multi): this context is shard 0 on
    // the primary device; peers[k] own shard k+1 (own device, stream, graph
    // copy and scratch).  fork/join events order the peers' streams after /
    // before the primary stream.
    sdnr_ctx **peers = nullptr;
    int npeers = 0;
    hipEvent_t ev_fork = nullptr;       // recorded on the primary stream
    hipEvent_t ev_join = nullptr;       // per context: recorded on its own stream
};

// Raise a kernel's dynamic-LDS limit; a refusal (e.g. static LDS + bytes >
// 160 KiB) is cleared so it cannot surface later as hipGetLastError().
inline void sdnr_allow_lds(const void *fn, size_t bytes)
{
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes) !=
        hipSuccess)
        (void)hipGetLastError();
}

// watchdog-word codes a kernel ORs into ctx->d_err (dfs.hip uses 1..16 for
// bounded waits that ran out, and 32 for the split kernel's CU-numbering spin,
// split_cu_number); sdnr_synchronize turns a nonzero word into an error, the
// specific INVAL causes below tested bit by bit (a word may hold several)
// A/B tuning knobs that only select non-default shapes (worker widths,
// block shapes, store hints): read by the diagnostic build alone
// (tools/diag/build_diag.sh, -DSDNR_DIAG_VARIANTS); the product library
// always takes its measured defaults (knob sprawl)
inline const char *sdnr_tune_env(const char *name)
{
#ifdef SDNR_DIAG_VARIANTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

constexpr int kDictPad = 0x40000000;   // dictionary-row padding offset (u + pad >= V)
constexpr int kDictMaxP = 255;         // pattern ids are bytes
constexpr int kErrLastPort = 256;   // sdnr_route_expand_packed: a last port outside [0, 0xFFFF]
constexpr int kErrTreeClimb = 512;  // sdnr_dfs_rows_affected: a tree climb outran V steps
constexpr int kErrScan = 1024;      // sdnr_route_offsets: a look-back wait ran out
constexpr int kErrSeg = 2048;       // route expansion: a walker / storer hand-off wait ran out

// error plumbing (capi.hip)
int sdnr_fail(int code, const char *fmt, ...);
int sdnr_hip_fail(hipError_t e, const char *what);
int sdnr_reserve(void **buf, size_t *cur, size_t need);
int sdnr_check_watchdog(sdnr_ctx *ctx);   // after a stream sync
// copy n (<= 4) ints from the device into out and wait for them with a
// busy spin on an event: a level loop's termination check costs a few
// microseconds instead of a blocking stream synchronize's wake-up
int sdnr_fetch_ints(sdnr_ctx *ctx, const int *d_src, int n, int *out);
// the same in two halves: the copy + event go on the stream, more work may
// follow them, then the host waits for the event (the words as of then)
int sdnr_wait_published(sdnr_ctx *ctx, int seq, int n, int *out);

#define SDNR_HIP(call)                                           \
    do {                                                         \
        hipError_t _e = (call);                                  \
        if (_e != hipSuccess) return sdnr_hip_fail(_e, #call);   \
    } while (0)

// kernel launchers (dfs.hip, shortest.hip, apsp.hip); device pointers,
// asynchronous on ctx->stream
int sdnr_launch_dfs(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc,
                    int32_t *d_parent, int32_t *d_port, int32_t *d_hops,
                    uint32_t *d_tree,         // d_tree: packed layout instead of the three
                    bool slots = false,       // d_tree as parent | slot << 26
                    bool hops16 = false);     // d_hops as u16 (0xFFFF unreached)
// int32 trees -> parent | port << 16 or parent | slot << 26 (dfs.hip)
int sdnr_launch_tree_pack(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port, size_t n,
                          uint32_t *tree, bool slots);
#ifdef SDNR_DIAG_VARIANTS
// the diagnostic build's losing DFS variants (tools/diag/)
// register-visited DFS (dfs_bits.hip): V <= 4096 with bitmap rows uploaded
bool sdnr_dfs_bits_ok(const sdnr_ctx *ctx);
int sdnr_launch_dfs_bits(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                         int32_t *d_port, int32_t *d_hops, uint32_t *d_tree, bool hops16);
// LDS-row DFS (dfs_runs.hip): usable when the run-encoded rows plus one
// source's state fit a workgroup's LDS
bool sdnr_dfs_runs_ok(const sdnr_ctx *ctx, bool hops);
int sdnr_launch_dfs_runs(sdnr_ctx *ctx, const int32_t *d_src, int32_t nsrc, int32_t *d_parent,
                         int32_t *d_port, int32_t *d_hops, uint32_t *d_tree);
#endif
int sdnr_launch_shortest(sdnr_ctx *ctx, const int32_t *d_dst, int32_t ndst,
                         uint16_t *d_dist, int32_t *d_nh, int32_t *d_nh_port);
int sdnr_launch_apsp(sdnr_ctx *ctx, uint16_t *d_dist);
int sdnr_launch_ecmp_counts(sdnr_ctx *ctx, const uint16_t *d_dist, int32_t ndst,
                            uint64_t *d_paths);
int sdnr_launch_ecmp_unrank(sdnr_ctx *ctx, const uint16_t *d_dist, const uint64_t *d_paths,
                            const int32_t *d_rows, const int32_t *d_srcs, const uint64_t *d_ranks,
                            int32_t nroutes, int32_t max_len, int32_t *d_out);
int sdnr_launch_route_offsets(sdnr_ctx *ctx, const int32_t *d_hops, const int32_t *d_rows,
                              const int32_t *d_dsts, int32_t npairs, int64_t *d_off);
int sdnr_launch_route_expand(sdnr_ctx *ctx, const int32_t *d_parent, const int32_t *d_port,
                             int32_t nrows, const int32_t *d_rows, const int32_t *d_dsts,
                             const int32_t *d_last_port, int32_t npairs, const int64_t *d_off,
                             int32_t *d_switch, int32_t *d_hport, uint32_t *d_entries = nullptr,
                             bool same_tables = false);
// rows of cached default-route trees a link change alters (incremental.hip)
int sdnr_launch_dfs_rows_affected(sdnr_ctx *ctx, const uint32_t *d_tree, const void *d_depth,
                                  int32_t layout, int32_t depth_bytes, int32_t nrows,
                                  const int32_t *d_row_src, const int32_t *d_links, int32_t nrm,
                                  int32_t nadd, uint8_t *d_affected);
int sdnr_launch_edge_ports(sdnr_ctx *ctx, const uint64_t *d_ends, int32_t nends,
                           const uint64_t *d_ports, int32_t nports, uint8_t *d_is_edge);
