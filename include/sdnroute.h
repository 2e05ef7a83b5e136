/*
 * sdnroute.h -- C ABI of the MI355X route engine (libsdnroute.so).
 *
 * Drop-in boundary for the route hot path of keichi/sdn-mpi-router:
 * the Python TopologyDB (reference sdnmpi/util/topology_db.py:8) keeps its
 * API and dict state; its route computation is replaced by per-source /
 * per-destination tables computed by the HIP kernels behind these entry
 * points.  The reference has no FFI of its own (it is pure Python); these
 * are the entry points a ctypes binding of that class binds (INTEGRATION.md
 * shows the binding, sdn-mpi-router_amd/sdnmpi_amd/_native.py is ours).
 *
 * Conventions
 *  - Every call returns SDNR_OK (0) or a negative errno-style code; the
 *    message of the last failure on the calling thread is sdnr_last_error().
 *  - Graph = dense CSR, vertex i = i-th smallest dpid, each row sorted
 *    strictly ascending (== sorted(self.links[dpid].keys()),
 *    topology_db.py:76), port[e] = links[u][v].src.port_no (:130).
 *  - Tables are row-major [n_rows][V] int32 (dist: uint16); the caller owns
 *    every buffer.  Without SDNR_DEVICE_PTRS they are host buffers and the
 *    call is synchronous; with it they are device buffers on the context's
 *    device and the call is asynchronous on the context's stream.
 *  - Unreachable entries are SDNR_UNREACHED (-1) / SDNR_DIST_INF (0xFFFF).
 *  - A context is not re-entrant (the reference calls TopologyDB from
 *    Ryu's single OS thread); distinct contexts are independent.
 */
#ifndef SDNROUTE_H
#define SDNROUTE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDNR_ABI_VERSION 1

#define SDNR_OK          0
#define SDNR_ERR_INVAL (-22)  /* EINVAL: bad argument / malformed CSR      */
#define SDNR_ERR_NOMEM (-12)  /* ENOMEM: device or host allocation failed  */
#define SDNR_ERR_NODEV (-19)  /* ENODEV: no such HIP device                */
#define SDNR_ERR_STATE (-77)  /* EBADFD: no graph uploaded to the context  */
#define SDNR_ERR_HIP   (-5)   /* EIO:    HIP runtime error                 */

#define SDNR_DEVICE_PTRS 0x1u /* table/source pointers are device pointers */
#define SDNR_TIMING      0x2u /* time the main kernel (sdnr_last_kernel_ms) */
#define SDNR_SAME_TABLES 0x4u /* route expansion: the parent / port tables are the
                                 ones (same pointers, same contents) of the
                                 previous expansion on this context -- its
                                 derived walk tables are reused */

#define SDNR_UNREACHED (-1)
#define SDNR_DIST_INF  0xFFFFu
#define SDNR_TREE_NONE 0xFFFFFFFFu

typedef struct sdnr_ctx sdnr_ctx;

/* ABI version of the loaded library (== SDNR_ABI_VERSION it was built with) */
int sdnr_abi_version(void);

/* Build identity: the SHA-256 (64 hex digits) of the sources, headers and
 * compile flags the library was built from ("unversioned" for a build made
 * without it).  The Python loader refuses a library whose id is not the
 * tree's (sdn-mpi-router_amd/sdnmpi_amd/_buildinfo.py). */
const char *sdnr_build_id(void);

/* Message of the last failing call on this thread ("" if none). */
const char *sdnr_last_error(void);

/* Number of visible HIP devices. */
int sdnr_device_count(int *count);

/* Create / destroy a context bound to HIP device `device`.  The context owns
 * the uploaded graph, scratch memory and a HIP stream.
 * Replaces the state of TopologyDB.__init__ (topology_db.py:9-18). */
int sdnr_create(int device, sdnr_ctx **out);
int sdnr_destroy(sdnr_ctx *ctx);

/* A context over several devices of one node (the controller's single
 * TopologyDB, reference sdnmpi/topology.py:67, driving all of them; SURVEY.md
 * 8(e)).  devices[0] is the primary: device-pointer buffers live there and
 * asynchronous work is ordered on its stream.  Every device holds a copy of
 * the uploaded graph; sdnr_dfs_tables, sdnr_dfs_tables_packed and
 * sdnr_shortest_tables split their ids into ndev contiguous shards, one per
 * device (each with its own stream), and assemble the rows in the caller's
 * tables -- host buffers by one device-to-host copy per shard, primary-device
 * buffers by peer copies over xGMI (fork/join events on the primary stream).
 * The other entry points run on the primary device.  A device may be listed
 * more than once (several shards on one device).  Destroy with sdnr_destroy. */
int sdnr_create_multi(const int *devices, int ndev, sdnr_ctx **out);

/* Devices of a context in shard order: *n = their number; the first
 * min(*n, cap) are written to devices (may be NULL). */
int sdnr_device_list(const sdnr_ctx *ctx, int *devices, int cap, int *n);

/* Run subsequent asynchronous work on `hip_stream` (a hipStream_t of the
 * context's device, e.g. torch.cuda.current_stream().cuda_stream); NULL
 * restores the context's own stream. */
int sdnr_set_stream(sdnr_ctx *ctx, void *hip_stream);

/* Wait for all work queued on the context's stream.  Also reports (as
 * SDNR_ERR_HIP) a kernel whose bounded internal wait ran out -- the
 * kernels never spin unboundedly; that only happens on a bug. */
int sdnr_synchronize(sdnr_ctx *ctx);

/* Upload the switch graph (host buffers).  Replaces the graph state that
 * add_switch/add_link/delete_* maintain (topology_db.py:14-42); the Python
 * side re-exports and re-uploads whenever that state changes.  Validates
 * the CSR (monotone row_ptr, rows strictly ascending, 0 <= col < V). */
int sdnr_graph_upload(sdnr_ctx *ctx, int32_t V, int32_t E,
                      const int32_t *row_ptr, const int32_t *col,
                      const int32_t *port);

/* V, E and maximum out-degree of the uploaded graph (NULL fields skipped). */
int sdnr_graph_info(const sdnr_ctx *ctx, int32_t *V, int32_t *E,
                    int32_t *max_degree);

/* Default route, find_route(src, dst) (multiple=False) -> _find_route_dfs
 * (topology_db.py:59-84, called from :181-188), batched over all
 * destinations: for every source src[i] the tree of first pushes of one full
 * LIFO traversal.  Row i of each table (V entries):
 *   parent[i*V+v]  vertex whose pop first pushed v (src[i] for v == src[i]),
 *   port[i*V+v]    links[parent][v].src.port_no (-1 for the root),
 *   hops[i*V+v]    tree depth (0 for the root); hops may be NULL.
 * The route src -> d is the tree path; it equals the reference's route for
 * every d, bit for bit (ports included). */
int sdnr_dfs_tables(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc,
                    int32_t *parent, int32_t *port, int32_t *hops,
                    uint32_t flags);

/* The same default-route trees in the packed layout (4 bytes per entry
 * instead of 8, half the HBM writes, device-to-host copy and all-gather
 * volume):
 *   tree[i*V+v] = parent | port << 16   (parent, port as in sdnr_dfs_tables;
 *                                         port 0xFFFF for the root),
 *   tree[i*V+v] = 0xFFFFFFFF            v unreachable (SDNR_TREE_NONE).
 * Needs V <= 65535 and every port in [0, 0xFFFE] -- OpenFlow 1.0 port
 * numbers are 16-bit (ofp_phy_port.port_no) -- else SDNR_ERR_INVAL. */
int sdnr_dfs_tables_packed(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc,
                           uint32_t *tree, uint32_t flags);

/* The same default-route trees for any fabric size (4 bytes per entry; the
 * packed layout above needs V <= 65535):
 *   tree[i*V+v] = parent | slot << 26   slot: position of v in parent's
 *                                         ascending neighbour list (links[
 *                                         parent] sorted by dpid, the CSR row);
 *                                         the port is that link's src.port_no;
 *                                         slot 63 for the root,
 *   tree[i*V+v] = 0xFFFFFFFF            v unreachable (SDNR_TREE_NONE).
 * The table pass stores one word per vertex and looks no port up.  Needs
 * V < 2^26 and every switch with <= 63 links, else SDNR_ERR_INVAL. */
int sdnr_dfs_tables_slots(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc,
                          uint32_t *tree, uint32_t flags);

/* Pack n entries of int32 default-route tables (sdnr_dfs_tables' parent /
 * port) into the 4-byte layouts above: layout SDNR_TREE_PORT16 = parent |
 * port << 16 (sdnr_dfs_tables_packed), SDNR_TREE_SLOT = parent | slot << 26
 * (sdnr_dfs_tables_slots; the slot is found in the uploaded CSR).  Device
 * pointers only (flags must hold SDNR_DEVICE_PTRS); asynchronous on the
 * context stream.  The route cache of the Python TopologyDB keeps its rows
 * in these layouts (a third of the int32 tables' bytes). */
#define SDNR_TREE_INT32  0   /* int32 parents (sdnr_dfs_rows_affected only) */
#define SDNR_TREE_PORT16 1
#define SDNR_TREE_SLOT   2
int sdnr_tree_pack(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port,
                   int64_t n, uint32_t *tree, int32_t layout, uint32_t flags);

/* Default-route trees straight in a 4-byte layout (SDNR_TREE_PORT16 as
 * sdnr_dfs_tables_packed, SDNR_TREE_SLOT as sdnr_dfs_tables_slots) plus the
 * tree depth -- the rows the Python TopologyDB's route cache keeps (the
 * route lengths of _route_to_fdb, topology_db.py:127-138, and the
 * incremental row tests need the depth):
 *   depth[i*V+v]  hops src[i] -> v; depth_bytes 2: u16, 0xFFFF unreachable
 *                 (needs V <= 65535), 4: int32, -1 unreachable; NULL: none.
 * The same kernels as the benched packed / slot tables, with no int32
 * intermediate. */
int sdnr_dfs_tables_tree(sdnr_ctx *ctx, const int32_t *src, int32_t nsrc,
                         uint32_t *tree, void *depth, int32_t layout,
                         int32_t depth_bytes, uint32_t flags);

/* Incremental recompute on link events: EventLinkAdd /
 * EventLinkDelete -> TopologyDB.add_link / delete_link (reference
 * sdnmpi/topology.py:192-198, sdnmpi/util/topology_db.py:30-42).  Which
 * cached default-route rows a set of link changes alters, decided from the
 * rows themselves: the tree words (layout SDNR_TREE_PORT16 / SDNR_TREE_SLOT
 * as sdnr_dfs_tables_tree writes them, or SDNR_TREE_INT32: int32 parents)
 * and depths (depth_bytes 2: u16, 0xFFFF unreached; 4: int32, -1) of
 * [nrows][V] rows; row_src[r] = the source of row r (-1: a free row, never
 * flagged).  links = (u, v) dense-id pairs: the first nremoved removed or
 * re-ported links, then nadded added links (ids against the CURRENT graph's
 * vertex set, which must equal the rows').  affected[r] = 1 iff the row
 * changes (exact for one link change, a superset for several):
 *   removed / re-ported (u, v): parent[v] == u;
 *   added (u, v): u reached and v unreached, or v pushed in a pop after u's
 *   (preorder, children in descending id order: the two root paths decide).
 * Device pointers only (flags must hold SDNR_DEVICE_PTRS); asynchronous on
 * the context stream; a row that is not a tree is reported by
 * sdnr_synchronize as SDNR_ERR_INVAL. */
int sdnr_dfs_rows_affected(sdnr_ctx *ctx, const uint32_t *tree, const void *depth,
                           int32_t layout, int32_t depth_bytes, int32_t nrows,
                           const int32_t *row_src, const int32_t *links,
                           int32_t nremoved, int32_t nadded, uint8_t *affected,
                           uint32_t flags);

/* Shortest routes, find_route(src, dst, multiple=True) -> _find_routes_bfs
 * (topology_db.py:86-122, called from :168-180), as per-destination tables:
 * for every destination dst[i] and every vertex x
 *   dist[i*V+x]     hop distance x -> dst[i] (SDNR_DIST_INF if none),
 *   nh[i*V+x]       smallest out-neighbour n with dist(n) == dist(x) - 1
 *                   (-1 for x == dst[i] or unreachable),
 *   nh_port[i*V+x]  links[x][nh].src.port_no.
 * Following nh from x gives routes[0] (the lexicographically smallest
 * shortest path); the shortest-path DAG in dist gives the whole ECMP set in
 * the reference's order.  nh / nh_port may be NULL (distances only). */
int sdnr_shortest_tables(sdnr_ctx *ctx, const int32_t *dst, int32_t ndst,
                         uint16_t *dist, int32_t *nh, int32_t *nh_port,
                         uint32_t flags);

/* All-pairs hop distances by min-plus squaring (D <- min(D, D (x) D) until
 * stable) for small dense graphs: dist[i*V+j] = hops i -> j (SDNR_DIST_INF
 * if none).
 * V <= 16384. */
int sdnr_apsp(sdnr_ctx *ctx, uint16_t *dist, uint32_t flags);

/* ECMP sets of find_route(src, dst, multiple=True) (_find_routes_bfs,
 * topology_db.py:86-122: every shortest route, lexicographic dpid order),
 * counted and unranked instead of enumerated.  dist = sdnr_shortest_tables
 * rows ([ndst][V], hops toward each destination).
 * sdnr_ecmp_counts: paths[i*V+x] = number of shortest x -> dst_i routes
 *   (saturating at UINT64_MAX; 1 at the destination, 0 if unreachable).
 * sdnr_ecmp_routes: route k = the ranks[k]-th (0-based, lexicographic) shortest
 *   route from srcs[k] to the destination of row rows[k], as dense vertex ids
 *   src..dst in route_vertices[k*max_len ...], padded with -1; a row of -1
 *   if the rank is out of range or the route is longer than max_len. */
int sdnr_ecmp_counts(sdnr_ctx *ctx, const uint16_t *dist, int32_t ndst,
                     uint64_t *paths, uint32_t flags);
int sdnr_ecmp_routes(sdnr_ctx *ctx, const uint16_t *dist, const uint64_t *paths,
                     int32_t ndst, const int32_t *rows, const int32_t *srcs,
                     const uint64_t *ranks, int32_t nroutes, int32_t max_len,
                     int32_t *route_vertices, uint32_t flags);

/* Flow entries of many host pairs from default-route tables (the OFPFlowMods
 * Router._add_flows_for_path installs, reference sdnmpi/router.py:83-104,
 * for the fdb _route_to_fdb builds, sdnmpi/util/topology_db.py:127-138).
 * Tables: row-major [nrows][V] as returned by sdnr_dfs_tables (hops needed
 * for the sizes).  Pair i is (row rows[i] = its source's tree, destination
 * switch dsts[i], last_port[i] = the destination host's port or OFPP_LOCAL).
 *
 * sdnr_route_offsets: offsets[0..npairs] (int64), offsets[i+1]-offsets[i] =
 *   entries of pair i = hops + 1 (0 if unreachable); offsets[npairs] = total.
 * sdnr_route_expand: for pair i, entries offsets[i]..offsets[i+1]-1 in path
 *   order: hop_switch[j] = dense switch id, hop_port[j] = its out port; the
 *   last entry is (dsts[i], last_port[i]).  Bit-identical to find_route's
 *   fdb with switch ids mapped to dpids.
 * nrows is required in both modes (the expansion builds ancestor
 * tables of the nrows trees).  Host buffers: the tables are staged per call
 * (nrows * V entries each). */
int sdnr_route_offsets(sdnr_ctx *ctx, const int32_t *hops, int32_t nrows,
                       const int32_t *rows, const int32_t *dsts, int32_t npairs,
                       int64_t *offsets, uint32_t flags);
int sdnr_route_expand(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port,
                      int32_t nrows, const int32_t *rows, const int32_t *dsts,
                      const int32_t *last_port, int32_t npairs,
                      const int64_t *offsets, int32_t *hop_switch,
                      int32_t *hop_port, uint32_t flags);

/* Replaces, like sdnr_route_expand, _route_to_fdb for many pairs
 * (sdnmpi/util/topology_db.py:127-138; the entries Router._add_flows_for_path
 * installs, sdnmpi/router.py:83-104).
 * The same entries as ONE u32 word each, switch | out_port << 16 (the
 * packed tree word's layout: a dense switch id and a 16-bit OpenFlow 1.0
 * port, OFPP_LOCAL = 0xfffe included) -- half the bytes of the two int32
 * arrays.  Needs V <= 65535 and 16-bit link ports (else SDNR_ERR_INVAL);
 * a last (host) port above 0xffff keeps only its low 16 bits, so callers
 * with such ports use sdnr_route_expand (the drop-in does).  Device
 * pointers only (flags must hold SDNR_DEVICE_PTRS). */
int sdnr_route_expand_packed(sdnr_ctx *ctx, const int32_t *parent, const int32_t *port,
                             int32_t nrows, const int32_t *rows, const int32_t *dsts,
                             const int32_t *last_port, int32_t npairs, const int64_t *offsets,
                             uint32_t *entries, uint32_t flags);

/* Flood ports (TopologyManager._is_edge_port / _do_broadcast, reference
 * sdnmpi/topology.py:150-177): is_edge[i] = 1 iff ports[i] is neither end of
 * any link.  Keys are (dense switch id << 32) | port_no; ends (both ends of
 * every link, the reference's link.src and link.dst) must be sorted
 * ascending (duplicates allowed).  Needs no uploaded graph. */
int sdnr_edge_ports(sdnr_ctx *ctx, const uint64_t *ends, int32_t nends,
                    const uint64_t *ports, int32_t nports, uint8_t *is_edge,
                    uint32_t flags);

/* Device time in milliseconds of the main kernel(s) of the last table call
 * made with SDNR_TIMING (waits for that call to finish). */
int sdnr_last_kernel_ms(sdnr_ctx *ctx, float *ms);

/* Number of launches of the main kernel in the last table call: the
 * min-plus squaring passes of sdnr_apsp, the BFS levels of the level-by-level
 * shortest kernel, 1 for single-launch kernels (0 before the first call). */
int sdnr_last_launches(const sdnr_ctx *ctx, int32_t *launches);

/* Bellman-Ford sweeps of the last sdnr_apsp call (the most any 8-row block
 * ran, summed over its relaxation launches; 0 with SDNROUTE_APSP_RELAX=0). */
int sdnr_last_sweeps(const sdnr_ctx *ctx, int32_t *sweeps);

/* Name of the kernel variant the last table call launched on this context
 * (e.g. "dfs_count_kernel<4>"; "" before the first call). */
const char *sdnr_last_kernel(const sdnr_ctx *ctx);

#ifdef __cplusplus
}
#endif

#endif /* SDNROUTE_H */
