// capi.hip -- extern "C" boundary of libsdnroute.so (include/sdnroute.h).
//
// Host side of the drop-in: validates and uploads the CSR the Python
// TopologyDB exports from its dicts (reference sdnmpi/util/topology_db.py:
// 14-18 state, :20-42 mutators), derives the ELL layout the DFS kernel reads,
// stages host buffers when the caller passes host pointers, and forwards to
// the kernel launchers (dfs.hip, shortest.hip, apsp.hip).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <array>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

static thread_local char g_err[512] = "";

int sdnr_fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

int sdnr_hip_fail(hipError_t e, const char *what)
{
    const int code = (e == hipErrorOutOfMemory) ? SDNR_ERR_NOMEM
                     : (e == hipErrorInvalidDevice || e == hipErrorNoDevice) ? SDNR_ERR_NODEV
                                                                             : SDNR_ERR_HIP;
    return sdnr_fail(code, "%s: %s", what, hipGetErrorString(e));
}

// A kernel whose bounded spin ran out sets *d_err instead of hanging; report
// it once (and clear it) after the work has been waited for.
int sdnr_check_watchdog(sdnr_ctx *ctx)
{
    int h = 0;
    SDNR_HIP(hipMemcpy(&h, ctx->d_err, sizeof(int), hipMemcpyDeviceToHost));
    if (h) {
        SDNR_HIP(hipMemset(ctx->d_err, 0, sizeof(int)));
        // bit tests: a word may hold several codes (e.g. a bad last port and
        // a hand-off wait of the same expansion); the specific cause wins
        if (h & kErrTreeClimb)
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: a tree row is not a tree "
                             "(a parent chain longer than V, or a reached vertex without a "
                             "reached parent)");
        if (h & kErrLastPort)
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand_packed: a last port outside "
                             "[0, 0xFFFF] (u32 entries hold 16-bit ports): entries invalid");
        return sdnr_fail(SDNR_ERR_HIP, "kernel watchdog tripped (code %d): results invalid", h);
    }
    return SDNR_OK;
}

int sdnr_reserve(void **buf, size_t *cur, size_t need)
{
    if (need <= *cur && *buf) return SDNR_OK;
    if (*buf) {
        (void)hipFree(*buf);
        *buf = nullptr;
        *cur = 0;
    }
    size_t n = need < 4096 ? 4096 : need;
    hipError_t e = hipMalloc(buf, n);
    if (e != hipSuccess) {
        *buf = nullptr;
        return sdnr_hip_fail(e, "hipMalloc(scratch)");
    }
    *cur = n;
    return SDNR_OK;
}

int sdnr_wait_published(sdnr_ctx *ctx, int seq, int n, int *out)
{
    volatile int *h = ctx->h_pub;
    for (unsigned k = 0;; ++k) {
        if (__atomic_load_n(&h[3], __ATOMIC_ACQUIRE) == seq) break;
        if ((k & 63) == 63) {                    // the stream drained without publishing: fault
            const hipError_t e = hipStreamQuery(ctx->stream);
            if (e == hipSuccess && __atomic_load_n(&h[3], __ATOMIC_ACQUIRE) != seq)
                return sdnr_fail(SDNR_ERR_HIP, "sdnr_wait_published: stream idle, word %d not "
                                                "published", seq);
            if (e != hipSuccess && e != hipErrorNotReady) return sdnr_hip_fail(e, "sdnr_wait_published");
        }
    }
    for (int i = 0; i < n; ++i) out[i] = h[i];
    return SDNR_OK;
}

int sdnr_fetch_ints(sdnr_ctx *ctx, const int *d_src, int n, int *out)
{
    if (n < 1 || n > 4) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_fetch_ints: %d words", n);
    SDNR_HIP(hipMemcpyAsync(ctx->h_flag, d_src, (size_t)n * sizeof(int), hipMemcpyDeviceToHost,
                            ctx->stream));
    SDNR_HIP(hipEventRecord(ctx->ev_flag, ctx->stream));
    for (;;) {
        const hipError_t e = hipEventQuery(ctx->ev_flag);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) return sdnr_hip_fail(e, "sdnr_fetch_ints");
    }
    for (int i = 0; i < n; ++i) out[i] = reinterpret_cast<volatile int *>(ctx->h_flag)[i];
    return SDNR_OK;
}

static void free_graph(sdnr_ctx *c)
{
    int32_t **bufs[] = {&c->row_ptr, &c->col, &c->port, &c->ell_col, &c->ell_port};
    for (int32_t **b : bufs) {
        if (*b) (void)hipFree(*b);
        *b = nullptr;
    }
    if (c->radj16 && c->radj_owned) (void)hipFree(c->radj16);
    if (c->runs) (void)hipFree(c->runs);
    c->runs = nullptr;
    c->runs_R = 0;
    if (c->adjb) (void)hipFree(c->adjb);
    if (c->adjp) (void)hipFree(c->adjp);
    if (c->radjx) (void)hipFree(c->radjx);
    c->adjb = nullptr;
    c->adjp = nullptr;
    c->radjx = nullptr;
    if (c->adj16) (void)hipFree(c->adj16);
    if (c->deg32) (void)hipFree(c->deg32);
    if (c->radjw) (void)hipFree(c->radjw);
    c->radjw = nullptr;
    if (c->radjc) (void)hipFree(c->radjc);
    c->radjc = nullptr;
    if (c->dict_bp) (void)hipFree(c->dict_bp);
    if (c->dict_bt) (void)hipFree(c->dict_bt);
    if (c->dict_off) (void)hipFree(c->dict_off);
    c->dict_bp = nullptr;
    c->dict_bt = nullptr;
    c->dict_off = nullptr;
    c->dict_P = 0;
    c->dict_NB = 0;
    c->dict_bpw = 0;
    if (c->ell16) (void)hipFree(c->ell16);
    if (c->ell_hi) (void)hipFree(c->ell_hi);
    c->ell16 = nullptr;
    c->ell_hi = nullptr;
    c->adj16 = nullptr;
    c->radj16 = nullptr;
    c->deg32 = nullptr;
    c->radj_owned = false;
    c->radj_pair = false;
    c->V = -1;
    c->E = 0;
    c->anc_valid = false;                // derived walk tables follow the graph
    c->W = 0;
    c->max_deg = 0;
}

static constexpr size_t kPad = SDNR_WAVE;

#ifdef SDNR_DIAG_VARIANTS
// Sorted rows (stride-64 u16 rows padded with the sentinel V) as arithmetic
// runs for dfs_runs.hip: greedy longest progression from each position,
// strides <= 511, counts <= 64, a run word = start | stride << 16 | count <<
// 25.  Returns the most runs a row needs; out gets R words per row.
static int encode_runs(int32_t V, const std::vector<uint16_t> &rows, int R,
                       std::vector<uint32_t> *out)
{
    int most = 0;
    if (out) out->assign((((size_t)V + 1) * R + 3) & ~(size_t)3, 0u);
    for (int32_t u = 0; u < V; ++u) {
        const uint16_t *r = rows.data() + (size_t)u * SDNR_WAVE;
        int n = 0;
        while (n < SDNR_WAVE && r[n] != (uint16_t)V) ++n;
        int nr = 0;
        for (int i = 0; i < n;) {
            int j = i, st = 0;
            if (i + 1 < n && r[i + 1] - r[i] <= 511) {
                st = r[i + 1] - r[i];
                j = i + 1;
                while (j + 1 < n && r[j + 1] - r[j] == st) ++j;
            }
            if (out && nr < R)
                (*out)[(size_t)u * R + nr] = (uint32_t)r[i] | ((uint32_t)st << 16) |
                                             ((uint32_t)(j - i + 1) << 25);
            ++nr;
            i = j + 1;
        }
        most = nr > most ? nr : most;
    }
    return most;
}

#endif

// device copy of `bytes` plus `pad` int32 entries of -1 behind them
static int upload(int32_t **dst, const void *src, size_t bytes, size_t pad, hipStream_t s)
{
    const size_t total = bytes + pad * sizeof(int32_t);
    SDNR_HIP(hipMalloc(reinterpret_cast<void **>(dst), total < 4 ? 4 : total));
    if (bytes) SDNR_HIP(hipMemcpyAsync(*dst, src, bytes, hipMemcpyHostToDevice, s));
    if (pad) SDNR_HIP(hipMemsetAsync(reinterpret_cast<char *>(*dst) + bytes, 0xFF,
                                     pad * sizeof(int32_t), s));
    return SDNR_OK;
}

// build identity: SHA-256 of the sources, headers and flags this library was
// compiled from (sdnmpi_amd/_buildinfo.py passes it; a file scan finds the
// marker without loading the library)
#ifndef SDNR_BUILD_ID
#define SDNR_BUILD_ID "unversioned"
#endif
static const char k_build_marker[] __attribute__((used)) = "SDNR_BUILD_ID:" SDNR_BUILD_ID;

#define CHECK_CTX(c) \
    if (!(c)) return sdnr_fail(SDNR_ERR_INVAL, "%s: null context", __func__)

extern "C" {

int sdnr_abi_version(void) { return SDNR_ABI_VERSION; }

const char *sdnr_build_id(void) { return k_build_marker + sizeof("SDNR_BUILD_ID:") - 1; }

const char *sdnr_last_error(void) { return g_err; }

int sdnr_device_count(int *count)
{
    if (!count) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_device_count: null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice) n = 0;
    else if (e != hipSuccess) return sdnr_hip_fail(e, "hipGetDeviceCount");
    *count = n;
    return SDNR_OK;
}

int sdnr_create(int device, sdnr_ctx **out)
{
    if (!out) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_create: null out");
    *out = nullptr;
    int n = 0;
    int rc = sdnr_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n)
        return sdnr_fail(SDNR_ERR_NODEV, "sdnr_create: device %d of %d", device, n);
    SDNR_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    SDNR_HIP(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return sdnr_fail(SDNR_ERR_NODEV, "sdnr_create: device %d is %s, built for gfx950",
                         device, prop.gcnArchName);
    sdnr_ctx *c = new sdnr_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_flag, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&c->h_flag), 4 * sizeof(int));
    // fine-grained (coherent) host words: a kernel's system-scope stores reach
    // the host without a copy on the stream
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void **>(&c->h_pub), 64,
                          hipHostMallocCoherent | hipHostMallocMapped);
    if (e == hipSuccess) memset(c->h_pub, 0, 64);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&c->d_err), sizeof(int));
    if (e == hipSuccess) e = hipMemset(c->d_err, 0, sizeof(int));
    if (e != hipSuccess) {
        delete c;
        return sdnr_hip_fail(e, "sdnr_create");
    }
    c->stream = c->own_stream;
    *out = c;
    return SDNR_OK;
}

int sdnr_create_multi(const int *devices, int ndev, sdnr_ctx **out)
{
    if (!out) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_create_multi: null out");
    *out = nullptr;
    if (!devices || ndev < 1)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_create_multi: %d devices", ndev);
    sdnr_ctx *c = nullptr;
    int rc = sdnr_create(devices[0], &c);
    if (rc) return rc;
    if (ndev > 1) {
        c->peers = new sdnr_ctx *[ndev - 1]();
        for (int k = 1; k < ndev; ++k) {
            if ((rc = sdnr_create(devices[k], &c->peers[k - 1]))) {
                const int keep = rc;
                char msg[512];
                snprintf(msg, sizeof msg, "%s", g_err);
                sdnr_destroy(c);
                return sdnr_fail(keep, "sdnr_create_multi: device %d: %s", devices[k], msg);
            }
            c->npeers = k;
        }
        // direct xGMI access between the primary and every other device: the
        // peers read their shard of the ids from, and copy their tables into,
        // the primary device's buffers
        for (int k = 1; k < ndev; ++k) {
            const int a = devices[0], b = devices[k];
            if (a == b) continue;
            int can = 0;
            for (int dir = 0; dir < 2; ++dir) {
                const int x = dir ? b : a, y = dir ? a : b;
                if (hipDeviceCanAccessPeer(&can, x, y) == hipSuccess && can &&
                    hipSetDevice(x) == hipSuccess &&
                    hipDeviceEnablePeerAccess(y, 0) != hipSuccess)
                    (void)hipGetLastError();     // already enabled: fine
            }
        }
        (void)hipSetDevice(devices[0]);
    }
    *out = c;
    return SDNR_OK;
}

int sdnr_destroy(sdnr_ctx *ctx)
{
    if (!ctx) return SDNR_OK;
    for (int k = 0; k < ctx->npeers; ++k) sdnr_destroy(ctx->peers[k]);
    delete[] ctx->peers;
    ctx->peers = nullptr;
    ctx->npeers = 0;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    free_graph(ctx);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->scratch2) (void)hipFree(ctx->scratch2);
    if (ctx->wq) (void)hipFree(ctx->wq);
    if (ctx->dmat) (void)hipFree(ctx->dmat);
    if (ctx->anc) (void)hipFree(ctx->anc);
    if (ctx->stage) (void)hipFree(ctx->stage);
    if (ctx->d_err) (void)hipFree(ctx->d_err);
    if (ctx->h_flag) (void)hipHostFree(ctx->h_flag);
    if (ctx->h_pub) (void)hipHostFree(ctx->h_pub);
    if (ctx->ev_flag) (void)hipEventDestroy(ctx->ev_flag);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
    if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return SDNR_OK;
}

int sdnr_set_stream(sdnr_ctx *ctx, void *hip_stream)
{
    CHECK_CTX(ctx);
    ctx->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : ctx->own_stream;
    return SDNR_OK;
}

int sdnr_synchronize(sdnr_ctx *ctx)
{
    CHECK_CTX(ctx);
    int first = SDNR_OK;
    for (int k = 0; k < ctx->npeers; ++k) {
        const int rc = sdnr_synchronize(ctx->peers[k]);
        if (rc && !first) first = rc;
    }
    SDNR_HIP(hipSetDevice(ctx->device));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    const int rc = sdnr_check_watchdog(ctx);
    return first ? first : rc;
}

int sdnr_device_list(const sdnr_ctx *ctx, int *devices, int cap, int *n)
{
    CHECK_CTX(ctx);
    if (!n) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_device_list: null n");
    *n = 1 + ctx->npeers;
    for (int k = 0; k < *n && k < cap && devices; ++k)
        devices[k] = k == 0 ? ctx->device : ctx->peers[k - 1]->device;
    return SDNR_OK;
}

static int graph_upload_one(sdnr_ctx *ctx, int32_t V, int32_t E, const int32_t *row_ptr,
                            const int32_t *col, const int32_t *port);

// Dictionary rows for the split DFS (dfs.hip, kRowDict): every sorted row as
// u + D[p(u)], D a list of distinct signed neighbour-offset tuples.  A
// regular fabric has few: a 32^3 torus 27 (3 boundary cases per dimension;
// the wrap-around links keep their place in the sorted row because the
// tuple is of the sorted ids' offsets).  The pattern ids are a second
// dictionary level: blocks of 32 consecutive switches as tuples of 32
// pattern bytes (a 32^3 torus: 9 distinct x-lines), so a switch's pattern is
// bt[bp[u >> 5]][u & 31] and the whole form -- V / 32 block bytes, the block
// tuples and D -- takes 2.2 KB of LDS for the 32^3 torus (a flat byte per
// switch, 32 KB, halved the workgroups per CU and measured slower: 99.5 vs
// 86.6 ms).  Then a DFS window reads no row from L2.  Built when V <= 65535,
// rows have <= 8 slots and both levels have <= kDictMaxP entries (else the
// split kernel keeps its ELL rows -- e.g. the Jellyfish); SDNROUTE_DFS_DICT=0
// skips it (A/B).
static int upload_dict(sdnr_ctx *ctx, int32_t V, int32_t W, const int32_t *row_ptr,
                       const int32_t *col)
{
    if (V > 65535 || W > 8) return SDNR_OK;
    if (const char *f = getenv("SDNROUTE_DFS_DICT"))
        if (!strcmp(f, "0")) return SDNR_OK;
    std::map<std::array<int32_t, 8>, int> ids;
    std::vector<std::array<int32_t, 8>> tuples;
    std::vector<uint8_t> pat(((size_t)V + 31) & ~(size_t)31, 0);
    for (int32_t u = 0; u < V; ++u) {
        std::array<int32_t, 8> t;
        t.fill(kDictPad);
        for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) t[e - row_ptr[u]] = col[e] - u;
        auto it = ids.find(t);
        if (it == ids.end()) {
            if ((int)tuples.size() >= kDictMaxP) return SDNR_OK;     // irregular: ELL rows
            it = ids.emplace(t, (int)tuples.size()).first;
            tuples.push_back(t);
        }
        pat[(size_t)u] = (uint8_t)it->second;
    }
    const size_t nblk = pat.size() / 32;
    std::map<std::array<uint8_t, 32>, int> bids;
    std::vector<std::array<uint8_t, 32>> blocks;
    const int32_t bpw = (int32_t)((nblk + 3) / 4);
    std::vector<uint32_t> bp((size_t)bpw, 0u);
    for (size_t b = 0; b < nblk; ++b) {
        std::array<uint8_t, 32> t;
        memcpy(t.data(), &pat[b * 32], 32);
        auto it = bids.find(t);
        if (it == bids.end()) {
            if ((int)blocks.size() >= kDictMaxP) return SDNR_OK;
            it = bids.emplace(t, (int)blocks.size()).first;
            blocks.push_back(t);
        }
        bp[b >> 2] |= (uint32_t)it->second << (8 * (b & 3));
    }
    std::vector<uint32_t> bt(blocks.size() * 8);
    for (size_t b = 0; b < blocks.size(); ++b) memcpy(&bt[b * 8], blocks[b].data(), 32);
    std::vector<int32_t> off(tuples.size() * 8);
    for (size_t p = 0; p < tuples.size(); ++p)
        for (int k = 0; k < 8; ++k) off[p * 8 + k] = tuples[p][k];
    int rc;
    if ((rc = upload(reinterpret_cast<int32_t **>(&ctx->dict_bp), bp.data(), bp.size() * 4, 0,
                     ctx->stream)) ||
        (rc = upload(reinterpret_cast<int32_t **>(&ctx->dict_bt), bt.data(), bt.size() * 4, 0,
                     ctx->stream)) ||
        (rc = upload(&ctx->dict_off, off.data(), off.size() * 4, 0, ctx->stream)))
        return rc;
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    ctx->dict_P = (int32_t)tuples.size();
    ctx->dict_NB = (int32_t)blocks.size();
    ctx->dict_bpw = bpw;
    return SDNR_OK;
}

int sdnr_graph_upload(sdnr_ctx *ctx, int32_t V, int32_t E, const int32_t *row_ptr,
                      const int32_t *col, const int32_t *port)
{
    CHECK_CTX(ctx);
    int rc = graph_upload_one(ctx, V, E, row_ptr, col, port);
    // every shard's device holds the whole graph (replicated CSR)
    for (int k = 0; k < ctx->npeers && !rc; ++k)
        rc = graph_upload_one(ctx->peers[k], V, E, row_ptr, col, port);
    if (rc) return rc;
    SDNR_HIP(hipSetDevice(ctx->device));
    return SDNR_OK;
}

static int graph_upload_one(sdnr_ctx *ctx, int32_t V, int32_t E, const int32_t *row_ptr,
                            const int32_t *col, const int32_t *port)
{
    if (V < 0 || E < 0) return sdnr_fail(SDNR_ERR_INVAL, "graph_upload: V=%d E=%d", V, E);
    if (!row_ptr || (E > 0 && (!col || !port)))
        return sdnr_fail(SDNR_ERR_INVAL, "graph_upload: null array");
    if (row_ptr[0] != 0 || row_ptr[V] != E)
        return sdnr_fail(SDNR_ERR_INVAL, "graph_upload: row_ptr[0]=%d row_ptr[V]=%d, E=%d",
                         row_ptr[0], row_ptr[V], E);
    int32_t maxdeg = 0;
    bool port16 = true;
    for (int32_t u = 0; u < V; ++u) {
        const int32_t a = row_ptr[u], b = row_ptr[u + 1];
        if (b < a) return sdnr_fail(SDNR_ERR_INVAL, "graph_upload: row_ptr decreases at %d", u);
        if (b - a > maxdeg) maxdeg = b - a;
        for (int32_t e = a; e < b; ++e) {
            if (port[e] < 0 || port[e] >= 0xFFFF) port16 = false;
            if (col[e] < 0 || col[e] >= V)
                return sdnr_fail(SDNR_ERR_INVAL, "graph_upload: col[%d]=%d out of range", e,
                                 col[e]);
            if (e > a && col[e] <= col[e - 1])
                return sdnr_fail(SDNR_ERR_INVAL,
                                 "graph_upload: row %d not strictly ascending at %d", u, e);
        }
    }
    SDNR_HIP(hipSetDevice(ctx->device));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    free_graph(ctx);
    int rc;
    // adjacency arrays carry kPad trailing entries so a wavefront may load a
    // whole 64-lane window past the last row unconditionally
    if ((rc = upload(&ctx->row_ptr, row_ptr, sizeof(int32_t) * ((size_t)V + 1), 0, ctx->stream)) ||
        (rc = upload(&ctx->col, col, sizeof(int32_t) * (size_t)E, kPad, ctx->stream)) ||
        (rc = upload(&ctx->port, port, sizeof(int32_t) * (size_t)E, kPad, ctx->stream))) {
        free_graph(ctx);
        return rc;
    }
    // ELL copy for the DFS chain: row u at u*W, -1 padded, when every row
    // fits one wavefront and padding at most doubles the adjacency
    int32_t W = 0;
    if (maxdeg > 0 && maxdeg <= SDNR_WAVE && (size_t)V * maxdeg <= 2 * (size_t)E + 64)
        W = maxdeg;
    if (const char *f = getenv("SDNROUTE_ELL"))   // debug/test knob: 0 = CSR only
        if (!strcmp(f, "0")) W = 0;
    if (W > 0) {
        std::vector<int32_t> ec((size_t)V * W, -1), ep((size_t)V * W, -1);
        for (int32_t u = 0; u < V; ++u)
            for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
                ec[(size_t)u * W + (e - row_ptr[u])] = col[e];
                ep[(size_t)u * W + (e - row_ptr[u])] = port[e];
            }
        if ((rc = upload(&ctx->ell_col, ec.data(), ec.size() * 4, kPad, ctx->stream)) ||
            (rc = upload(&ctx->ell_port, ep.data(), ep.size() * 4, kPad, ctx->stream))) {
            free_graph(ctx);
            return rc;
        }
        // narrow ELL ids for the large-graph DFS: u16 (V <= 65535: id 0xFFFF is
        // free for padding), or 16 low bits + a per-row mask of bit 16
        // (V <= 131071, rows <= 32 slots); padding decodes to an id >= V
        if (V <= 131071 && W <= 32) {
            std::vector<uint16_t> e16(ec.size() + kPad, (uint16_t)0xFFFF);
            std::vector<uint32_t> hi(V > 65535 ? (size_t)V + kPad : 0, 0u);
            for (size_t i = 0; i < ec.size(); ++i) {
                const int32_t x = ec[i];
                e16[i] = (uint16_t)(x < 0 ? 0xFFFF : (x & 0xFFFF));
                if (V > 65535 && (x < 0 || (x >> 16)))
                    hi[i / (size_t)W] |= 1u << (i % (size_t)W);
            }
            hipError_t he = hipMalloc(reinterpret_cast<void **>(&ctx->ell16), e16.size() * 2);
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->ell16, e16.data(), e16.size() * 2, hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess && !hi.empty()) {
                he = hipMalloc(reinterpret_cast<void **>(&ctx->ell_hi), hi.size() * 4);
                if (he == hipSuccess)
                    he = hipMemcpyAsync(ctx->ell_hi, hi.data(), hi.size() * 4,
                                        hipMemcpyHostToDevice, ctx->stream);
            }
            if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
            if (he != hipSuccess) {
                free_graph(ctx);
                return sdnr_hip_fail(he, "graph_upload(ell16)");
            }
        }
        SDNR_HIP(hipStreamSynchronize(ctx->stream));   // before ec/ep go away
        if ((rc = upload_dict(ctx, V, W, row_ptr, col))) {
            free_graph(ctx);
            return rc;
        }
    }
    // u16 rows of stride 64 (one 128-byte line) for the cooperative DFS
    // kernels: padding and the extra row V hold the sentinel vertex V; the
    // in-neighbour rows (same layout) and packed out-degrees feed the
    // counted-pop kernel
    int32_t max_indeg = 0x7FFFFFFF;             // known only with the u16 rows
    if (V < 65535 && maxdeg <= SDNR_WAVE) {
        const size_t rows = ((size_t)V + 1) * SDNR_WAVE;
        std::vector<uint16_t> a16(rows, (uint16_t)V), r16(rows, (uint16_t)V);
        std::vector<int32_t> indeg((size_t)V + 1, 0);
        std::vector<uint32_t> d32(((size_t)V + 2) & ~(size_t)1, 0u);   // even: read in pairs
        for (int32_t u = 0; u < V; ++u) {
            const int32_t d = row_ptr[u + 1] - row_ptr[u];
            d32[(size_t)u] = (uint32_t)d;
            for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
                a16[(size_t)u * SDNR_WAVE + (e - row_ptr[u])] = (uint16_t)col[e];
                indeg[col[e]]++;
            }
        }
        int32_t maxin = 0;
        for (int32_t v = 0; v < V; ++v) maxin = indeg[v] > maxin ? indeg[v] : maxin;
        max_indeg = maxin;
        bool sym = true;
        if (maxin <= SDNR_WAVE) {
            std::vector<int32_t> fill((size_t)V, 0);
            for (int32_t u = 0; u < V; ++u)       // ascending u: rows come out sorted
                for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
                    const int32_t v = col[e];
                    r16[(size_t)v * SDNR_WAVE + fill[v]++] = (uint16_t)u;
                }
            sym = a16 == r16;
        }
        hipError_t he = hipMalloc(reinterpret_cast<void **>(&ctx->adj16), rows * 2);
        if (he == hipSuccess)
            he = hipMemcpyAsync(ctx->adj16, a16.data(), rows * 2, hipMemcpyHostToDevice, ctx->stream);
        if (he == hipSuccess && maxin <= SDNR_WAVE) {
            he = hipMalloc(reinterpret_cast<void **>(&ctx->deg32), d32.size() * 4);
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->deg32, d32.data(), d32.size() * 4, hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess && sym) {
                ctx->radj16 = ctx->adj16;
            } else if (he == hipSuccess) {
                he = hipMalloc(reinterpret_cast<void **>(&ctx->radj16), rows * 2);
                ctx->radj_owned = he == hipSuccess;
                if (he == hipSuccess)
                    he = hipMemcpyAsync(ctx->radj16, r16.data(), rows * 2, hipMemcpyHostToDevice,
                                        ctx->stream);
            }
        }
        // in-rows as the async DFS workers' count indices: lds_swz(x); the
        // padding of slot l a dummy word of its own past the counts (one
        // shared dummy made every ds_sub a 16-way same-address conflict:
        // 3x slower) (dfs.hip, kFlagPreSwz)
        // (dummies right past the swizzled counts, inside the 256-word
        // padding where it has room: a +256-B LDS block per workgroup took
        // k=48 from 5 to 4 workgroups per CU)
        const size_t dummy = (((size_t)V + 1 + 31) & ~(size_t)31);
        if (he == hipSuccess && maxin <= SDNR_WAVE && dummy + SDNR_WAVE <= 0xFFFF) {
            std::vector<uint16_t> w16(r16.size());
            const std::vector<uint16_t> &src16 = sym ? a16 : r16;
            // rows of <= 32 in-neighbours: lanes 32..63 repeat lanes 0..31 (the
            // dummies stay per lane), so a worker pairs two children per load
            const bool pair = maxin <= SDNR_WAVE / 2;
            const char *pe = sdnr_tune_env("SDNROUTE_DFS_PAIR");          // 0: off (A/B)
            ctx->radj_pair = pair && !(pe && !strcmp(pe, "0"));
            auto at = [&](size_t i) {
                return ctx->radj_pair ? (i & ~(size_t)(SDNR_WAVE / 2)) : i;   // lane l -> l & 31
            };
            for (size_t i = 0; i < w16.size(); ++i) {
                const int x = src16[at(i)];
                w16[i] = (uint16_t)(x == V ? (int)(dummy + i % SDNR_WAVE) : (x ^ ((x >> 3) & 31)));
            }
            he = hipMalloc(reinterpret_cast<void **>(&ctx->radjw), w16.size() * 2);
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->radjw, w16.data(), w16.size() * 2, hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
            // the same for the compact-LDS kernel (u16 counts in pairs):
            // entry = lds_swz(x >> 1) << 1 | (x & 1), dummies dummyc + lane
            const size_t dummyc = ((((size_t)V + 2) >> 1) + 31) & ~(size_t)31;
            if (he == hipSuccess && 2 * (dummyc + SDNR_WAVE) <= 0xFFFF) {
                for (size_t i = 0; i < w16.size(); ++i) {
                    const int x = src16[at(i)];
                    const int h = x >> 1;
                    w16[i] = (uint16_t)(x == V ? (int)(2 * (dummyc + i % SDNR_WAVE))
                                               : ((h ^ ((h >> 3) & 31)) << 1) | (x & 1));
                }
                he = hipMalloc(reinterpret_cast<void **>(&ctx->radjc), w16.size() * 2);
                if (he == hipSuccess)
                    he = hipMemcpyAsync(ctx->radjc, w16.data(), w16.size() * 2,
                                        hipMemcpyHostToDevice, ctx->stream);
                if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
            }
        }
#ifdef SDNR_DIAG_VARIANTS
        // diagnostic build only (tools/diag/): the losing DFS variants' rows
        // the out-rows as arithmetic runs for the LDS-row DFS (dfs_runs.hip)
        const char *rf = getenv("SDNROUTE_RUNS");                 // 0: off (A/B)
        if (he == hipSuccess && maxin <= SDNR_WAVE && !(rf && !strcmp(rf, "0"))) {
            const int m = encode_runs(V, a16, 0, nullptr);
            const int R = m <= 2 ? 2 : (m <= 4 ? 4 : 0);
            if (R) {
                std::vector<uint32_t> w;
                encode_runs(V, a16, R, &w);
                he = hipMalloc(reinterpret_cast<void **>(&ctx->runs), w.size() * 4);
                if (he == hipSuccess)
                    he = hipMemcpyAsync(ctx->runs, w.data(), w.size() * 4, hipMemcpyHostToDevice,
                                        ctx->stream);
                if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
                ctx->runs_R = R;
            }
        }
        // bitmap rows + prefix counts + in-rows with vertex ids for the
        // register-visited DFS (dfs_bits.hip): V <= 4096 (64 lanes x 64 bits)
        const char *bf = getenv("SDNROUTE_BITS");                 // 0: off (A/B)
        if (he == hipSuccess && maxin <= SDNR_WAVE && V <= 4096 && !(bf && !strcmp(bf, "0"))) {
            std::vector<uint64_t> ab((size_t)V * SDNR_WAVE, 0ull);
            std::vector<uint8_t> ap((size_t)V * SDNR_WAVE, 0);
            for (int32_t u = 0; u < V; ++u)
                for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
                    const int32_t v = col[e];
                    ab[(size_t)u * SDNR_WAVE + (v >> 6)] |= 1ull << (v & 63);
                }
            for (int32_t u = 0; u < V; ++u) {
                int run = 0;
                for (int l = 0; l < SDNR_WAVE; ++l) {
                    ap[(size_t)u * SDNR_WAVE + l] = (uint8_t)run;
                    run += __builtin_popcountll(ab[(size_t)u * SDNR_WAVE + l]);
                }
            }
            const std::vector<uint16_t> &in16 = sym ? a16 : r16;
            const uint32_t dummyx = ((uint32_t)V + 31u) & ~31u;
            std::vector<uint32_t> rx(((size_t)V + 1) * SDNR_WAVE);
            for (size_t i = 0; i < rx.size(); ++i) {
                const int x = in16[i];
                rx[i] = x == V ? (dummyx + (uint32_t)(i % SDNR_WAVE)) | (0xFFFFu << 16)
                               : (uint32_t)(x ^ ((x >> 3) & 31)) | ((uint32_t)x << 16);
            }
            he = hipMalloc(reinterpret_cast<void **>(&ctx->adjb), ab.size() * 8);
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->adjb, ab.data(), ab.size() * 8, hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess) he = hipMalloc(reinterpret_cast<void **>(&ctx->adjp), ap.size());
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->adjp, ap.data(), ap.size(), hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess) he = hipMalloc(reinterpret_cast<void **>(&ctx->radjx), rx.size() * 4);
            if (he == hipSuccess)
                he = hipMemcpyAsync(ctx->radjx, rx.data(), rx.size() * 4, hipMemcpyHostToDevice,
                                    ctx->stream);
            if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
        }
#endif
        if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
        if (he != hipSuccess) {
            free_graph(ctx);
            return sdnr_hip_fail(he, "graph_upload(adj16)");
        }
    }
    // symmetric (every link has its reverse): in-rows equal out-rows, so a
    // BFS toward a destination may expand out-rows
    bool symmetric = true;
    for (int32_t u = 0; u < V && symmetric; ++u)
        for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
            const int32_t v = col[e];
            int32_t lo = row_ptr[v], hi = row_ptr[v + 1];
            while (lo < hi) {
                const int32_t mid = (lo + hi) >> 1;
                if (col[mid] < u) lo = mid + 1; else hi = mid;
            }
            if (lo == row_ptr[v + 1] || col[lo] != u) {
                symmetric = false;
                break;
            }
        }
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    ctx->V = V;
    ctx->E = E;
    ctx->W = W;
    ctx->plane_depth = 0;
    ctx->max_deg = maxdeg;
    ctx->max_indeg = max_indeg;
    ctx->port16 = port16;
    ctx->symmetric = symmetric;
    return SDNR_OK;
}

int sdnr_graph_info(const sdnr_ctx *ctx, int32_t *V, int32_t *E, int32_t *max_degree)
{
    CHECK_CTX(ctx);
    if (ctx->V < 0) return sdnr_fail(SDNR_ERR_STATE, "graph_info: no graph uploaded");
    if (V) *V = ctx->V;
    if (E) *E = ctx->E;
    if (max_degree) *max_degree = ctx->max_deg;
    return SDNR_OK;
}

// host <-> device staging for host-pointer calls
struct Stage {
    char *base = nullptr;
    size_t off = 0;
    void *take(size_t bytes)
    {
        void *p = base + off;
        off += (bytes + 255) & ~(size_t)255;
        return p;
    }
};

static int begin_call(sdnr_ctx *ctx, int32_t n, const void *ids, uint32_t flags,
                      const char *fn)
{
    if (!ctx) return sdnr_fail(SDNR_ERR_INVAL, "%s: null context", fn);
    if (ctx->V < 0) return sdnr_fail(SDNR_ERR_STATE, "%s: no graph uploaded", fn);
    if (n < 0) return sdnr_fail(SDNR_ERR_INVAL, "%s: negative count", fn);
    if (n > 0 && !ids) return sdnr_fail(SDNR_ERR_INVAL, "%s: null id array", fn);
    if (!(flags & SDNR_DEVICE_PTRS) && ids) {
        const int32_t *h = static_cast<const int32_t *>(ids);
        for (int32_t i = 0; i < n; ++i)
            if (h[i] < 0 || h[i] >= ctx->V)
                return sdnr_fail(SDNR_ERR_INVAL, "%s: id[%d]=%d outside [0,%d)", fn, i, h[i],
                                 ctx->V);
    }
    SDNR_HIP(hipSetDevice(ctx->device));
    ctx->timed = (flags & SDNR_TIMING) != 0;
    ctx->last_launches = 1;
    return SDNR_OK;
}

// One table call over the context and its peers (sdnr_create_multi): the ids
// are split into contiguous shards, shard k runs on context k, and up to three
// [n][V] output tables (entry sizes es[i], null outputs skipped) are assembled
// in the caller's buffers.
//  * host buffers: every context stages its shard, launches, and copies its
//    rows straight into the caller's tables; then all are waited for and
//    their watchdog words checked.
//  * device buffers (on the primary device, asynchronous on its stream): the
//    peers wait for the primary stream (fork event), pull their ids over
//    xGMI, compute into their own scratch and copy the rows into the primary
//    device's tables; the primary stream waits for every peer (join events).
typedef int (*shard_launch_fn)(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const out[3]);

// Run `fn(k)` for shards 1..n-1 on host threads of their own and for shard 0
// on the calling thread, then join: a shard launcher may block on the host
// (the shortest-table level loops poll a host word per group of levels), so
// the shards of a multi-device context must not wait for each other there.
// The first failing shard's error (rc + its thread's message) is returned.
extern "C++" template <typename Fn>
static int on_shard_threads(int n, Fn fn, bool threaded)
{
    if (n == 1) return fn(0);
    if (!threaded) {
        // launches that only enqueue (the DFS kernels) are issued in turn
        // from this thread: a thread start + join per shard costs more than
        // the launches themselves on small calls
        for (int k = 0; k < n; ++k)
            if (int rc = fn(k)) return rc;
        return SDNR_OK;
    }
    std::vector<int> rcs((size_t)n, SDNR_OK);
    std::vector<std::string> msgs((size_t)n);
    std::vector<std::thread> th;
    for (int k = 1; k < n; ++k)
        th.emplace_back([&, k] {
            rcs[(size_t)k] = fn(k);
            if (rcs[(size_t)k]) msgs[(size_t)k] = g_err;
        });
    rcs[0] = fn(0);
    if (rcs[0]) msgs[0] = g_err;
    for (auto &t : th) t.join();
    for (int k = 0; k < n; ++k)
        if (rcs[(size_t)k]) return sdnr_fail(rcs[(size_t)k], "%s", msgs[(size_t)k].c_str());
    return SDNR_OK;
}

static int shard_shortest(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3]);

static int run_sharded(sdnr_ctx *ctx, const int32_t *ids, int32_t n, void *const out[3],
                       const size_t es[3], uint32_t flags, shard_launch_fn launch)
{
    const int nctx = 1 + ctx->npeers;
    const size_t V = (size_t)ctx->V;
    const int32_t per = (n + nctx - 1) / nctx;
    auto sub = [&](int k) { return k == 0 ? ctx : ctx->peers[k - 1]; };
    auto lo_of = [&](int k) { return (int32_t)((int64_t)k * per < n ? (int64_t)k * per : n); };
    auto hi_of = [&](int k) { return lo_of(k) + per < n ? lo_of(k) + per : n; };
    const bool timed = ctx->timed;
    int rc;
    if (flags & SDNR_DEVICE_PTRS) {
        if (nctx == 1) return launch(ctx, ids, n, out);
        if (timed) SDNR_HIP(hipEventRecord(ctx->ev0, ctx->stream));
        SDNR_HIP(hipEventRecord(ctx->ev_fork, ctx->stream));
        ctx->timed = false;                        // the span is timed around fork/join
        rc = on_shard_threads(nctx, [&](int k) -> int {
            sdnr_ctx *c = sub(k);
            const int32_t lo = lo_of(k), cnt = hi_of(k) - lo;
            SDNR_HIP(hipSetDevice(c->device));
            if (k == 0) return launch(ctx, ids, hi_of(0), out);
            if (cnt <= 0) return SDNR_OK;
            SDNR_HIP(hipStreamWaitEvent(c->stream, ctx->ev_fork, 0));
            size_t need = 4 * (size_t)cnt + 256;
            for (int i = 0; i < 3; ++i)
                if (out[i]) need += (size_t)cnt * V * es[i] + 256;
            int r;
            if ((r = sdnr_reserve(&c->stage, &c->stage_bytes, need))) return r;
            Stage st{static_cast<char *>(c->stage)};
            int32_t *d_ids = static_cast<int32_t *>(st.take(4 * (size_t)cnt));
            void *d_out[3] = {nullptr, nullptr, nullptr};
            for (int i = 0; i < 3; ++i)
                if (out[i]) d_out[i] = st.take((size_t)cnt * V * es[i]);
            SDNR_HIP(hipMemcpyPeerAsync(d_ids, c->device, ids + lo, ctx->device, 4 * (size_t)cnt,
                                        c->stream));
            c->timed = false;
            if ((r = launch(c, d_ids, cnt, d_out))) return r;
            for (int i = 0; i < 3; ++i)
                if (out[i])
                    SDNR_HIP(hipMemcpyPeerAsync(static_cast<char *>(out[i]) + (size_t)lo * V * es[i],
                                                ctx->device, d_out[i], c->device,
                                                (size_t)cnt * V * es[i], c->stream));
            SDNR_HIP(hipEventRecord(c->ev_join, c->stream));
            return SDNR_OK;
        }, launch == shard_shortest);   // the plane BFS polls the host between levels
        ctx->timed = timed;
        SDNR_HIP(hipSetDevice(ctx->device));
        if (rc) return rc;
        for (int k = 1; k < nctx; ++k)
            if (hi_of(k) > lo_of(k)) SDNR_HIP(hipStreamWaitEvent(ctx->stream, sub(k)->ev_join, 0));
        if (timed) SDNR_HIP(hipEventRecord(ctx->ev1, ctx->stream));
        return SDNR_OK;
    }
    // host buffers: stage + launch everywhere (one host thread per shard),
    // copy out, then wait
    void *d_outs[64][3] = {};
    if (nctx > 64) return sdnr_fail(SDNR_ERR_INVAL, "more than 64 devices");
    rc = on_shard_threads(nctx, [&](int k) -> int {
        sdnr_ctx *c = sub(k);
        const int32_t lo = lo_of(k), cnt = hi_of(k) - lo;
        if (cnt <= 0) return SDNR_OK;
        SDNR_HIP(hipSetDevice(c->device));
        size_t need = 4 * (size_t)cnt + 256;
        for (int i = 0; i < 3; ++i)
            if (out[i]) need += (size_t)cnt * V * es[i] + 256;
        int r;
        if ((r = sdnr_reserve(&c->stage, &c->stage_bytes, need))) return r;
        Stage st{static_cast<char *>(c->stage)};
        int32_t *d_ids = static_cast<int32_t *>(st.take(4 * (size_t)cnt));
        for (int i = 0; i < 3; ++i)
            if (out[i]) d_outs[k][i] = st.take((size_t)cnt * V * es[i]);
        SDNR_HIP(hipMemcpyAsync(d_ids, ids + lo, 4 * (size_t)cnt, hipMemcpyHostToDevice, c->stream));
        c->timed = k == 0 && nctx == 1 && timed;  // multi: shard 0 alone is not the span
        if ((r = launch(c, d_ids, cnt, d_outs[k]))) return r;
        for (int i = 0; i < 3; ++i)
            if (out[i])
                SDNR_HIP(hipMemcpyAsync(static_cast<char *>(out[i]) + (size_t)lo * V * es[i],
                                        d_outs[k][i], (size_t)cnt * V * es[i],
                                        hipMemcpyDeviceToHost, c->stream));
        return SDNR_OK;
    }, true);      // pageable host copies block: one thread per shard
    int first = rc;
    for (int k = 0; k < nctx; ++k) {
        sdnr_ctx *c = sub(k);
        SDNR_HIP(hipSetDevice(c->device));
        SDNR_HIP(hipStreamSynchronize(c->stream));
        rc = sdnr_check_watchdog(c);
        if (rc && !first) first = rc;
    }
    ctx->timed = timed;
    SDNR_HIP(hipSetDevice(ctx->device));
    return first;
}

static int shard_dfs(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, static_cast<int32_t *>(o[0]), static_cast<int32_t *>(o[1]),
                           static_cast<int32_t *>(o[2]), nullptr);
}

static int shard_dfs_packed(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, nullptr, static_cast<uint32_t *>(o[0]));
}

static int shard_dfs_slots(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, nullptr, static_cast<uint32_t *>(o[0]),
                           true);
}

static int shard_shortest(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_shortest(c, ids, n, static_cast<uint16_t *>(o[0]),
                                static_cast<int32_t *>(o[1]), static_cast<int32_t *>(o[2]));
}

int sdnr_dfs_tables(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc, int32_t *parent,
                    int32_t *port, int32_t *hops, uint32_t flags)
{
    int rc = begin_call(ctx, nsrc, src, flags, "sdnr_dfs_tables");
    if (rc) return rc;
    if (nsrc > 0 && (!parent || !port))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables: null table");
    void *const out[3] = {parent, port, hops};
    const size_t es[3] = {4, 4, 4};
    return run_sharded(ctx, src, nsrc, out, es, flags, shard_dfs);
}

int sdnr_dfs_tables_packed(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc, uint32_t *tree,
                           uint32_t flags)
{
    int rc = begin_call(ctx, nsrc, src, flags, "sdnr_dfs_tables_packed");
    if (rc) return rc;
    if (nsrc > 0 && !tree) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_packed: null table");
    if (ctx->V > 0xFFFF || !ctx->port16)
        return sdnr_fail(SDNR_ERR_INVAL,
                         "sdnr_dfs_tables_packed: needs V <= 65535 and ports < 0xFFFF (V=%d)",
                         ctx->V);
    void *const out[3] = {tree, nullptr, nullptr};
    const size_t es[3] = {4, 0, 0};
    return run_sharded(ctx, src, nsrc, out, es, flags, shard_dfs_packed);
}

int sdnr_dfs_tables_slots(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc, uint32_t *tree,
                          uint32_t flags)
{
    int rc = begin_call(ctx, nsrc, src, flags, "sdnr_dfs_tables_slots");
    if (rc) return rc;
    if (nsrc > 0 && !tree) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_slots: null table");
    if (ctx->V > (1 << 26) - 1 || ctx->max_deg > 63)
        return sdnr_fail(SDNR_ERR_INVAL,
                         "sdnr_dfs_tables_slots: needs V < 2^26 and rows of <= 63 links "
                         "(V=%d, max degree %d)", ctx->V, ctx->max_deg);
    void *const out[3] = {tree, nullptr, nullptr};
    const size_t es[3] = {4, 0, 0};
    return run_sharded(ctx, src, nsrc, out, es, flags, shard_dfs_slots);
}

static int shard_tree_p16_h16(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, static_cast<int32_t *>(o[1]),
                           static_cast<uint32_t *>(o[0]), false, true);
}

static int shard_tree_p16_h32(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, static_cast<int32_t *>(o[1]),
                           static_cast<uint32_t *>(o[0]), false, false);
}

static int shard_tree_slot_h16(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, static_cast<int32_t *>(o[1]),
                           static_cast<uint32_t *>(o[0]), true, true);
}

static int shard_tree_slot_h32(sdnr_ctx *c, const int32_t *ids, int32_t n, void *const o[3])
{
    return sdnr_launch_dfs(c, ids, n, nullptr, nullptr, static_cast<int32_t *>(o[1]),
                           static_cast<uint32_t *>(o[0]), true, false);
}

int sdnr_dfs_tables_tree(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc, uint32_t *tree,
                         void *depth, int32_t layout, int32_t depth_bytes, uint32_t flags)
{
    int rc = begin_call(ctx, nsrc, src, flags, "sdnr_dfs_tables_tree");
    if (rc) return rc;
    if (nsrc > 0 && !tree) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: null table");
    if (layout == SDNR_TREE_PORT16) {
        if (ctx->V > 0xFFFF || !ctx->port16)
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: port16 needs V <= 65535 and "
                             "ports < 0xFFFF (V=%d)", ctx->V);
    } else if (layout == SDNR_TREE_SLOT) {
        if (ctx->V > (1 << 26) - 1 || ctx->max_deg > 63)
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: slots need V < 2^26 and rows "
                             "of <= 63 links (V=%d, max degree %d)", ctx->V, ctx->max_deg);
    } else {
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: layout %d", layout);
    }
    if (depth && depth_bytes != 2 && depth_bytes != 4)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: depth_bytes %d", depth_bytes);
    if (depth && depth_bytes == 2 && ctx->V > 0xFFFF)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_tables_tree: u16 depths need V <= 65535");
    void *const out[3] = {tree, depth, nullptr};
    const size_t es[3] = {4, depth ? (size_t)depth_bytes : 0, 0};
    const bool h16 = depth && depth_bytes == 2;
    shard_launch_fn fn = layout == SDNR_TREE_SLOT ? (h16 ? shard_tree_slot_h16 : shard_tree_slot_h32)
                                                  : (h16 ? shard_tree_p16_h16 : shard_tree_p16_h32);
    return run_sharded(ctx, src, nsrc, out, es, flags, fn);
}

int sdnr_tree_pack(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port, int64_t n,
                   uint32_t *tree, int32_t layout, uint32_t flags)
{
    CHECK_CTX(ctx);
    if (ctx->V < 0) return sdnr_fail(SDNR_ERR_STATE, "sdnr_tree_pack: no graph uploaded");
    if (!(flags & SDNR_DEVICE_PTRS))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_tree_pack: device pointers only");
    if (n < 0 || (n > 0 && (!parent || !tree || (layout == SDNR_TREE_PORT16 && !port))))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_tree_pack: null table");
    if (layout == SDNR_TREE_PORT16 && (ctx->V > 0xFFFF || !ctx->port16))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_tree_pack: port16 needs V <= 65535 and ports "
                         "< 0xFFFF (V=%d)", ctx->V);
    if (layout == SDNR_TREE_SLOT && (ctx->V > (1 << 26) - 1 || ctx->max_deg > 63))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_tree_pack: slots need V < 2^26 and rows of "
                         "<= 63 links (V=%d)", ctx->V);
    if (layout != SDNR_TREE_PORT16 && layout != SDNR_TREE_SLOT)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_tree_pack: layout %d", layout);
    if (n == 0 || ctx->V == 0) return SDNR_OK;
    SDNR_HIP(hipSetDevice(ctx->device));
    return sdnr_launch_tree_pack(ctx, parent, port, (size_t)n, tree, layout == SDNR_TREE_SLOT);
}

int sdnr_dfs_rows_affected(sdnr_ctx *ctx, const uint32_t *tree, const void *depth, int32_t layout,
                           int32_t depth_bytes, int32_t nrows, const int32_t *row_src,
                           const int32_t *links, int32_t nremoved, int32_t nadded,
                           uint8_t *affected, uint32_t flags)
{
    CHECK_CTX(ctx);
    if (ctx->V < 0) return sdnr_fail(SDNR_ERR_STATE, "sdnr_dfs_rows_affected: no graph uploaded");
    if (!(flags & SDNR_DEVICE_PTRS))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: device pointers only");
    if (nrows < 0 || nremoved < 0 || nadded < 0)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: negative count");
    if (layout != SDNR_TREE_INT32 && layout != SDNR_TREE_PORT16 && layout != SDNR_TREE_SLOT)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: layout %d", layout);
    if (depth_bytes != 2 && depth_bytes != 4)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: depth_bytes %d", depth_bytes);
    if (depth_bytes == 2 && ctx->V > 0xFFFF)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: u16 depths need V <= 65535");
    if (nrows > 0 && (!tree || !depth || !row_src || !affected))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: null table");
    if (nremoved + nadded > 0 && !links)
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_dfs_rows_affected: null links");
    if (nrows == 0) return SDNR_OK;
    SDNR_HIP(hipSetDevice(ctx->device));
    ctx->timed = (flags & SDNR_TIMING) != 0;
    return sdnr_launch_dfs_rows_affected(ctx, tree, depth, layout, depth_bytes, nrows, row_src,
                                         links, nremoved, nadded, affected);
}

int sdnr_shortest_tables(sdnr_ctx *ctx, const int32_t *dst, int32_t ndst, uint16_t *dist,
                         int32_t *nh, int32_t *nh_port, uint32_t flags)
{
    int rc = begin_call(ctx, ndst, dst, flags, "sdnr_shortest_tables");
    if (rc) return rc;
    if (ndst > 0 && !dist) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_shortest_tables: null dist");
    if ((nh == nullptr) != (nh_port == nullptr))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_shortest_tables: nh and nh_port go together");
    void *const out[3] = {dist, nh, nh_port};
    const size_t es[3] = {2, 4, 4};
    return run_sharded(ctx, dst, ndst, out, es, flags, shard_shortest);
}

int sdnr_apsp(sdnr_ctx *ctx, uint16_t *dist, uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_apsp");
    if (rc) return rc;
    if (!dist) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_apsp: null dist");
    if (flags & SDNR_DEVICE_PTRS) return sdnr_launch_apsp(ctx, dist);
    const size_t bytes = (size_t)ctx->V * ctx->V * 2;
    if ((rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes, bytes))) return rc;
    uint16_t *d = static_cast<uint16_t *>(ctx->stage);
    if ((rc = sdnr_launch_apsp(ctx, d))) return rc;
    SDNR_HIP(hipMemcpyAsync(dist, d, bytes, hipMemcpyDeviceToHost, ctx->stream));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

static int check_pairs(const sdnr_ctx *ctx, int32_t nrows, const int32_t *rows,
                       const int32_t *dsts, int32_t npairs, const char *fn)
{
    for (int32_t i = 0; i < npairs; ++i) {
        if (rows[i] < 0 || rows[i] >= nrows)
            return sdnr_fail(SDNR_ERR_INVAL, "%s: row[%d]=%d outside [0,%d)", fn, i, rows[i], nrows);
        if (dsts[i] < 0 || dsts[i] >= ctx->V)
            return sdnr_fail(SDNR_ERR_INVAL, "%s: dst[%d]=%d outside [0,%d)", fn, i, dsts[i], ctx->V);
    }
    return SDNR_OK;
}

int sdnr_route_offsets(sdnr_ctx *ctx, const int32_t *hops, int32_t nrows, const int32_t *rows,
                       const int32_t *dsts, int32_t npairs, int64_t *offsets, uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_route_offsets");
    if (rc) return rc;
    if (npairs < 0 || nrows < 0 || !offsets || (npairs > 0 && (!hops || !rows || !dsts)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_offsets: bad arguments");
    if (flags & SDNR_DEVICE_PTRS)
        return sdnr_launch_route_offsets(ctx, hops, rows, dsts, npairs, offsets);
    if ((rc = check_pairs(ctx, nrows, rows, dsts, npairs, "sdnr_route_offsets"))) return rc;
    const size_t tab = (size_t)nrows * ctx->V * 4, pr = (size_t)npairs * 4;
    if ((rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes,
                           tab + 2 * pr + ((size_t)npairs + 1) * 8 + 1024)))
        return rc;
    Stage st{static_cast<char *>(ctx->stage)};
    int32_t *d_h = static_cast<int32_t *>(st.take(tab));
    int32_t *d_r = static_cast<int32_t *>(st.take(pr));
    int32_t *d_d = static_cast<int32_t *>(st.take(pr));
    int64_t *d_o = static_cast<int64_t *>(st.take(((size_t)npairs + 1) * 8));
    SDNR_HIP(hipMemcpyAsync(d_h, hops, tab, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_r, rows, pr, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_d, dsts, pr, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = sdnr_launch_route_offsets(ctx, d_h, d_r, d_d, npairs, d_o))) return rc;
    SDNR_HIP(hipMemcpyAsync(offsets, d_o, ((size_t)npairs + 1) * 8, hipMemcpyDeviceToHost,
                            ctx->stream));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

int sdnr_route_expand_packed(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port,
                             int32_t nrows, const int32_t *rows, const int32_t *dsts,
                             const int32_t *last_port, int32_t npairs, const int64_t *offsets,
                             uint32_t *entries, uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_route_expand_packed");
    if (rc) return rc;
    if (!(flags & SDNR_DEVICE_PTRS))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand_packed: device pointers only");
    if (npairs < 0 || nrows < 0 || !offsets ||
        (npairs > 0 && (!parent || !port || !rows || !dsts || !last_port || !entries)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand_packed: bad arguments");
    return sdnr_launch_route_expand(ctx, parent, port, nrows, rows, dsts, last_port, npairs,
                                    offsets, nullptr, nullptr, entries,
                                    (flags & SDNR_SAME_TABLES) != 0);
}

int sdnr_route_expand(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port, int32_t nrows,
                      const int32_t *rows, const int32_t *dsts, const int32_t *last_port,
                      int32_t npairs, const int64_t *offsets, int32_t *hop_switch,
                      int32_t *hop_port, uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_route_expand");
    if (rc) return rc;
    if (npairs < 0 || nrows < 0 || !offsets ||
        (npairs > 0 && (!parent || !port || !rows || !dsts || !last_port)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand: bad arguments");
    if (flags & SDNR_DEVICE_PTRS)
        return sdnr_launch_route_expand(ctx, parent, port, nrows, rows, dsts, last_port, npairs,
                                        offsets, hop_switch, hop_port, nullptr,
                                        (flags & SDNR_SAME_TABLES) != 0);
    if ((rc = check_pairs(ctx, nrows, rows, dsts, npairs, "sdnr_route_expand"))) return rc;
    const int64_t total = offsets[npairs];
    if (total > 0 && (!hop_switch || !hop_port))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand: null output");
    for (int32_t i = 0; i < npairs; ++i)
        if (offsets[i + 1] < offsets[i] || offsets[i] < 0)
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_route_expand: offsets not ascending at %d", i);
    const size_t tab = (size_t)nrows * ctx->V * 4, pr = (size_t)npairs * 4;
    const size_t ent = (size_t)total * 4;
    if ((rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes,
                           2 * tab + 3 * pr + ((size_t)npairs + 1) * 8 + 2 * ent + 2048)))
        return rc;
    Stage st{static_cast<char *>(ctx->stage)};
    int32_t *d_p = static_cast<int32_t *>(st.take(tab));
    int32_t *d_t = static_cast<int32_t *>(st.take(tab));
    int32_t *d_r = static_cast<int32_t *>(st.take(pr));
    int32_t *d_d = static_cast<int32_t *>(st.take(pr));
    int32_t *d_l = static_cast<int32_t *>(st.take(pr));
    int64_t *d_o = static_cast<int64_t *>(st.take(((size_t)npairs + 1) * 8));
    int32_t *d_s = static_cast<int32_t *>(st.take(ent));
    int32_t *d_q = static_cast<int32_t *>(st.take(ent));
    SDNR_HIP(hipMemcpyAsync(d_p, parent, tab, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_t, port, tab, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_r, rows, pr, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_d, dsts, pr, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_l, last_port, pr, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_o, offsets, ((size_t)npairs + 1) * 8, hipMemcpyHostToDevice,
                            ctx->stream));
    if ((rc = sdnr_launch_route_expand(ctx, d_p, d_t, nrows, d_r, d_d, d_l, npairs, d_o, d_s, d_q)))
        return rc;
    if (ent) {
        SDNR_HIP(hipMemcpyAsync(hop_switch, d_s, ent, hipMemcpyDeviceToHost, ctx->stream));
        SDNR_HIP(hipMemcpyAsync(hop_port, d_q, ent, hipMemcpyDeviceToHost, ctx->stream));
    }
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

int sdnr_ecmp_counts(sdnr_ctx *ctx, const uint16_t *dist, int32_t ndst, uint64_t *paths,
                     uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_ecmp_counts");
    if (rc) return rc;
    if (ndst < 0 || (ndst > 0 && (!dist || !paths)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_ecmp_counts: bad arguments");
    if (flags & SDNR_DEVICE_PTRS) return sdnr_launch_ecmp_counts(ctx, dist, ndst, paths);
    const size_t n = (size_t)ndst * ctx->V;
    if ((rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes, n * 10 + 512))) return rc;
    Stage st{static_cast<char *>(ctx->stage)};
    uint16_t *d_d = static_cast<uint16_t *>(st.take(n * 2));
    uint64_t *d_p = static_cast<uint64_t *>(st.take(n * 8));
    SDNR_HIP(hipMemcpyAsync(d_d, dist, n * 2, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = sdnr_launch_ecmp_counts(ctx, d_d, ndst, d_p))) return rc;
    SDNR_HIP(hipMemcpyAsync(paths, d_p, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

int sdnr_ecmp_routes(sdnr_ctx *ctx, const uint16_t *dist, const uint64_t *paths, int32_t ndst,
                     const int32_t *rows, const int32_t *srcs, const uint64_t *ranks,
                     int32_t nroutes, int32_t max_len, int32_t *route_vertices, uint32_t flags)
{
    int rc = begin_call(ctx, 0, nullptr, flags, "sdnr_ecmp_routes");
    if (rc) return rc;
    if (ndst < 0 || nroutes < 0 || max_len < 1 ||
        (nroutes > 0 && (!dist || !paths || !rows || !srcs || !ranks || !route_vertices)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_ecmp_routes: bad arguments");
    if (flags & SDNR_DEVICE_PTRS)
        return sdnr_launch_ecmp_unrank(ctx, dist, paths, rows, srcs, ranks, nroutes, max_len,
                                       route_vertices);
    if ((rc = check_pairs(ctx, ndst, rows, srcs, nroutes, "sdnr_ecmp_routes"))) return rc;
    const size_t n = (size_t)ndst * ctx->V, r = (size_t)nroutes;
    const size_t outb = r * (size_t)max_len * 4;
    if ((rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes, n * 10 + r * 16 + outb + 2048)))
        return rc;
    Stage st{static_cast<char *>(ctx->stage)};
    uint16_t *d_d = static_cast<uint16_t *>(st.take(n * 2));
    uint64_t *d_p = static_cast<uint64_t *>(st.take(n * 8));
    int32_t *d_r = static_cast<int32_t *>(st.take(r * 4));
    int32_t *d_s = static_cast<int32_t *>(st.take(r * 4));
    uint64_t *d_k = static_cast<uint64_t *>(st.take(r * 8));
    int32_t *d_o = static_cast<int32_t *>(st.take(outb));
    SDNR_HIP(hipMemcpyAsync(d_d, dist, n * 2, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_p, paths, n * 8, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_r, rows, r * 4, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_s, srcs, r * 4, hipMemcpyHostToDevice, ctx->stream));
    SDNR_HIP(hipMemcpyAsync(d_k, ranks, r * 8, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = sdnr_launch_ecmp_unrank(ctx, d_d, d_p, d_r, d_s, d_k, nroutes, max_len, d_o)))
        return rc;
    SDNR_HIP(hipMemcpyAsync(route_vertices, d_o, outb, hipMemcpyDeviceToHost, ctx->stream));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

int sdnr_edge_ports(sdnr_ctx *ctx, const uint64_t *ends, int32_t nends, const uint64_t *ports,
                    int32_t nports, uint8_t *is_edge, uint32_t flags)
{
    CHECK_CTX(ctx);
    if (nends < 0 || nports < 0 || (nends > 0 && !ends) || (nports > 0 && (!ports || !is_edge)))
        return sdnr_fail(SDNR_ERR_INVAL, "sdnr_edge_ports: bad arguments");
    SDNR_HIP(hipSetDevice(ctx->device));
    ctx->timed = (flags & SDNR_TIMING) != 0;
    ctx->last_launches = 1;
    if (flags & SDNR_DEVICE_PTRS)
        return sdnr_launch_edge_ports(ctx, ends, nends, ports, nports, is_edge);
    for (int32_t i = 1; i < nends; ++i)
        if (ends[i] < ends[i - 1])
            return sdnr_fail(SDNR_ERR_INVAL, "sdnr_edge_ports: ends not sorted at %d", i);
    const size_t eb = (size_t)nends * 8, pb = (size_t)nports * 8;
    int rc = sdnr_reserve(&ctx->stage, &ctx->stage_bytes, eb + pb + (size_t)nports + 1024);
    if (rc) return rc;
    Stage st{static_cast<char *>(ctx->stage)};
    uint64_t *d_e = static_cast<uint64_t *>(st.take(eb));
    uint64_t *d_p = static_cast<uint64_t *>(st.take(pb));
    uint8_t *d_o = static_cast<uint8_t *>(st.take((size_t)nports));
    if (eb) SDNR_HIP(hipMemcpyAsync(d_e, ends, eb, hipMemcpyHostToDevice, ctx->stream));
    if (pb) SDNR_HIP(hipMemcpyAsync(d_p, ports, pb, hipMemcpyHostToDevice, ctx->stream));
    if ((rc = sdnr_launch_edge_ports(ctx, d_e, nends, d_p, nports, d_o))) return rc;
    if (nports) SDNR_HIP(hipMemcpyAsync(is_edge, d_o, (size_t)nports, hipMemcpyDeviceToHost,
                                        ctx->stream));
    SDNR_HIP(hipStreamSynchronize(ctx->stream));
    return SDNR_OK;
}

const char *sdnr_last_kernel(const sdnr_ctx *ctx) { return ctx ? ctx->last_kernel : ""; }

int sdnr_last_sweeps(const sdnr_ctx *ctx, int32_t *sweeps)
{
    CHECK_CTX(ctx);
    if (!sweeps) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_last_sweeps: null out");
    *sweeps = ctx->last_sweeps;
    return SDNR_OK;
}

int sdnr_last_launches(const sdnr_ctx *ctx, int32_t *launches)
{
    CHECK_CTX(ctx);
    if (!launches) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_last_launches: null out");
    *launches = ctx->last_launches;
    return SDNR_OK;
}

int sdnr_last_kernel_ms(sdnr_ctx *ctx, float *ms)
{
    CHECK_CTX(ctx);
    if (!ms) return sdnr_fail(SDNR_ERR_INVAL, "sdnr_last_kernel_ms: null ms");
    if (!ctx->timed) return sdnr_fail(SDNR_ERR_STATE, "sdnr_last_kernel_ms: last call untimed");
    SDNR_HIP(hipSetDevice(ctx->device));
    SDNR_HIP(hipEventSynchronize(ctx->ev1));
    SDNR_HIP(hipEventElapsedTime(ms, ctx->ev0, ctx->ev1));
    return SDNR_OK;
}

}  // extern "C"
