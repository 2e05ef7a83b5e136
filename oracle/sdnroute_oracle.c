/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference route computation
 * (keichi/sdn-mpi-router, sdnmpi/util/topology_db.py) used as the parity
 * checker for the HIP path and as bench.py's cpu_baseline leg.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load this library;
 * the product (sdn-mpi-router_amd/) never links or calls it.
 *
 * Parity pinned: tests/test_oracle_golden.py checks every function here
 * against fixtures produced by running the reference TopologyDB itself
 * (tests/golden/make_golden.py) on the mock square, fat-tree k=4/k=8, small
 * torus/dragonfly/random directed graphs, and sampled pairs of the five
 * BASELINE configs.
 *
 * Graph input: dense CSR, vertices in ascending dpid order, each row sorted
 * ascending (= sorted(self.links[dpid].keys()), topology_db.py:76/:106),
 * port[e] = links[u][v].src.port_no (topology_db.py:130).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_UNREACHED (-1)

/*
 * Default route, find_route(multiple=False) -> _find_route_dfs
 * (topology_db.py:59-84): LIFO stack of paths, a vertex is marked visited
 * when it is pushed (:78-82), neighbours pushed in ascending order (:76), the
 * search returns when the destination is popped (:70-71).
 *
 * A vertex's predecessor on its path is fixed at the push that first marks
 * it, and the early return at :70-71 only stops the traversal after the
 * destination's push, so the path returned for (s, d) is the path from s to d
 * in the tree of first pushes of ONE full traversal from s.  This function
 * runs that full traversal and records, for every vertex v:
 *   parent[v]  dense id of the vertex whose pop pushed v (s for v == s),
 *   port[v]    links[parent][v].src.port_no (-1 for v == s),
 *   hops[v]    tree depth (0 for v == s);
 * -1 in all three when v is unreachable (:84 returns []).
 * stack must hold V ints.
 */
void oracle_dfs_tree(int32_t V, const int32_t *row_ptr, const int32_t *col,
                     const int32_t *port, int32_t s, int32_t *parent,
                     int32_t *port_out, int32_t *hops, int32_t *stack)
{
    for (int32_t v = 0; v < V; ++v) {
        parent[v] = ORACLE_UNREACHED;
        port_out[v] = ORACLE_UNREACHED;
        if (hops) hops[v] = ORACLE_UNREACHED;
    }
    int32_t sp = 0;
    parent[s] = s;
    if (hops) hops[s] = 0;
    stack[sp++] = s;
    while (sp > 0) {
        int32_t u = stack[--sp];
        int32_t du = hops ? hops[u] : 0;
        for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
            int32_t v = col[e];
            if (parent[v] != ORACLE_UNREACHED) continue;  /* visited */
            parent[v] = u;
            port_out[v] = port[e];
            if (hops) hops[v] = du + 1;
            stack[sp++] = v;
        }
    }
}

/*
 * find_route(multiple=True) -> _find_routes_bfs (topology_db.py:86-122)
 * returns every shortest simple path, in FIFO order, which is lexicographic
 * order of the dpid sequence (children appended in ascending order, :106-111;
 * stable sort by length, :118-122).  routes[0] is the lexicographically
 * smallest shortest path, which is the greedy destination rule: from x take
 * the smallest neighbour n with dist(n, d) == dist(x, d) - 1.
 *
 * oracle_dest_tables computes, for ONE destination d, over every vertex x:
 *   dist[x]     hop distance x -> d (0xFFFF if d unreachable from x),
 *   nh[x]       smallest out-neighbour one hop closer to d (-1 for x == d or
 *               unreachable), and nh_port[x] its links[x][nh].src.port_no.
 * It needs the reverse CSR (rrow, rcol) for the BFS from d and scratch of V
 * ints.
 */
void oracle_dest_tables(int32_t V, const int32_t *row_ptr, const int32_t *col,
                        const int32_t *port, const int32_t *rrow,
                        const int32_t *rcol, int32_t d, uint16_t *dist,
                        int32_t *nh, int32_t *nh_port, int32_t *queue)
{
    for (int32_t v = 0; v < V; ++v) {
        dist[v] = 0xFFFF;
        nh[v] = -1;
        nh_port[v] = -1;
    }
    int32_t qh = 0, qt = 0;
    dist[d] = 0;
    queue[qt++] = d;
    while (qh < qt) {
        int32_t y = queue[qh++];
        for (int32_t e = rrow[y]; e < rrow[y + 1]; ++e) {
            int32_t x = rcol[e];                 /* x -> y is a link */
            if (dist[x] != 0xFFFF) continue;
            dist[x] = (uint16_t)(dist[y] + 1);
            queue[qt++] = x;
        }
    }
    for (int32_t x = 0; x < V; ++x) {
        if (x == d || dist[x] == 0xFFFF) continue;
        for (int32_t e = row_ptr[x]; e < row_ptr[x + 1]; ++e) {
            int32_t n = col[e];                  /* ascending: first is min */
            if (dist[n] != 0xFFFF && dist[n] + 1 == dist[x]) {
                nh[x] = n;
                nh_port[x] = port[e];
                break;
            }
        }
    }
}

/*
 * Per-source tree of the lexicographically smallest shortest paths (FIFO BFS
 * with ascending neighbour order): parent[v] is the first dequeued vertex
 * that reaches v.  Equals routes[0] of _find_routes_bfs for every (s, v).
 */
void oracle_bfs_tree(int32_t V, const int32_t *row_ptr, const int32_t *col,
                     const int32_t *port, int32_t s, int32_t *parent,
                     int32_t *port_out, int32_t *hops, int32_t *queue)
{
    for (int32_t v = 0; v < V; ++v) {
        parent[v] = ORACLE_UNREACHED;
        port_out[v] = ORACLE_UNREACHED;
        hops[v] = ORACLE_UNREACHED;
    }
    int32_t qh = 0, qt = 0;
    parent[s] = s;
    hops[s] = 0;
    queue[qt++] = s;
    while (qh < qt) {
        int32_t u = queue[qh++];
        for (int32_t e = row_ptr[u]; e < row_ptr[u + 1]; ++e) {
            int32_t v = col[e];
            if (parent[v] != ORACLE_UNREACHED) continue;
            parent[v] = u;
            port_out[v] = port[e];
            hops[v] = hops[u] + 1;
            queue[qt++] = v;
        }
    }
}

/* Floyd-Warshall over hop counts (0xFFFF = infinity); dist is V*V row-major,
 * dist[i*V+j] = hops i -> j.  Reference for the min-plus APSP kernel. */
void oracle_apsp(int32_t V, const int32_t *row_ptr, const int32_t *col,
                 uint16_t *dist)
{
    for (int64_t i = 0; i < (int64_t)V * V; ++i) dist[i] = 0xFFFF;
    for (int32_t i = 0; i < V; ++i) {
        dist[(int64_t)i * V + i] = 0;
        for (int32_t e = row_ptr[i]; e < row_ptr[i + 1]; ++e)
            if (col[e] != i) dist[(int64_t)i * V + col[e]] = 1;
    }
    for (int32_t k = 0; k < V; ++k)
        for (int32_t i = 0; i < V; ++i) {
            uint32_t dik = dist[(int64_t)i * V + k];
            if (dik == 0xFFFF) continue;
            for (int32_t j = 0; j < V; ++j) {
                uint32_t c = dik + dist[(int64_t)k * V + j];
                if (c < dist[(int64_t)i * V + j]) dist[(int64_t)i * V + j] = (uint16_t)c;
            }
        }
}

/* ---------------- batched drivers (pthreads over sources) ---------------- */

typedef struct {
    int kind; /* 0 dfs, 1 bfs tree, 2 dest tables */
    int32_t V;
    const int32_t *row_ptr, *col, *port, *rrow, *rcol, *srcs;
    int32_t nsrc;
    int32_t *a, *b, *c;
    uint16_t *dist;
    int32_t next;
    pthread_mutex_t mu;
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    int32_t *scratch = (int32_t *)malloc(sizeof(int32_t) * (size_t)(j->V > 0 ? j->V : 1));
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int32_t i = j->next;
        j->next += 16;
        pthread_mutex_unlock(&j->mu);
        if (i >= j->nsrc) break;
        int32_t hi = i + 16 < j->nsrc ? i + 16 : j->nsrc;
        for (; i < hi; ++i) {
            size_t off = (size_t)i * (size_t)j->V;
            if (j->kind == 0)
                oracle_dfs_tree(j->V, j->row_ptr, j->col, j->port, j->srcs[i],
                                j->a + off, j->b + off, j->c ? j->c + off : NULL,
                                scratch);
            else if (j->kind == 1)
                oracle_bfs_tree(j->V, j->row_ptr, j->col, j->port, j->srcs[i],
                                j->a + off, j->b + off, j->c + off, scratch);
            else
                oracle_dest_tables(j->V, j->row_ptr, j->col, j->port, j->rrow,
                                   j->rcol, j->srcs[i], j->dist + off,
                                   j->a + off, j->b + off, scratch);
        }
    }
    free(scratch);
    return NULL;
}

static void run_job(job_t *j, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    j->next = 0;
    pthread_mutex_init(&j->mu, NULL);
    for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, j);
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
    pthread_mutex_destroy(&j->mu);
}

/* tables[i*V + v] for source srcs[i]; hops may be NULL */
void oracle_dfs_tables(int32_t V, const int32_t *row_ptr, const int32_t *col,
                       const int32_t *port, const int32_t *srcs, int32_t nsrc,
                       int32_t *parent, int32_t *port_out, int32_t *hops,
                       int nthreads)
{
    job_t j;
    memset(&j, 0, sizeof j);
    j.kind = 0; j.V = V; j.row_ptr = row_ptr; j.col = col; j.port = port;
    j.srcs = srcs; j.nsrc = nsrc; j.a = parent; j.b = port_out; j.c = hops;
    run_job(&j, nthreads);
}

void oracle_bfs_tables(int32_t V, const int32_t *row_ptr, const int32_t *col,
                       const int32_t *port, const int32_t *srcs, int32_t nsrc,
                       int32_t *parent, int32_t *port_out, int32_t *hops,
                       int nthreads)
{
    job_t j;
    memset(&j, 0, sizeof j);
    j.kind = 1; j.V = V; j.row_ptr = row_ptr; j.col = col; j.port = port;
    j.srcs = srcs; j.nsrc = nsrc; j.a = parent; j.b = port_out; j.c = hops;
    run_job(&j, nthreads);
}

/* dist/nh/nh_port[i*V + x] for destination dsts[i] */
void oracle_dest_tables_batch(int32_t V, const int32_t *row_ptr,
                              const int32_t *col, const int32_t *port,
                              const int32_t *rrow, const int32_t *rcol,
                              const int32_t *dsts, int32_t ndst, uint16_t *dist,
                              int32_t *nh, int32_t *nh_port, int nthreads)
{
    job_t j;
    memset(&j, 0, sizeof j);
    j.kind = 2; j.V = V; j.row_ptr = row_ptr; j.col = col; j.port = port;
    j.rrow = rrow; j.rcol = rcol; j.srcs = dsts; j.nsrc = ndst;
    j.dist = dist; j.a = nh; j.b = nh_port;
    run_job(&j, nthreads);
}
