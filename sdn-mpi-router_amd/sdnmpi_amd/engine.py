"""Route tables on the GPU and their expansion into fdb lists.

``RouteEngine`` owns one native context (``_native.Context``) and the graph
uploaded to it.  ``TableCache`` keeps, per uploaded graph, the per-source DFS
tables (default route, reference ``_find_route_dfs``,
``sdnmpi/util/topology_db.py:59-84``) and the per-destination shortest
tables (``_find_routes_bfs``, :86-122) that have been computed, and extends
them on demand.  Expansion follows the reference's ``_route_to_fdb``
(:127-138): one ``(dpid, out_port)`` per switch on the path, the last one
being the destination switch's host port or ``OFPP_LOCAL``.
"""

import numpy as np

from . import _native
from .graph import empty_csr

__all__ = ["RouteEngine", "TableCache", "tree_path", "expand_tree_paths",
           "shortest_paths_lex"]


class RouteEngine(object):
    """The GPU route engine of one TopologyDB (one HIP device)."""

    def __init__(self, device=0):
        self.ctx = _native.Context(device)
        self._loaded = None

    def load(self, export):
        if self._loaded is not export:
            self.ctx.upload(export.csr if export.csr.V else empty_csr())
            self._loaded = export

    def dfs_tables(self, export, srcs, with_hops=True):
        self.load(export)
        return self.ctx.dfs_tables(srcs, with_hops=with_hops)

    def shortest_tables(self, export, dsts):
        self.load(export)
        return self.ctx.shortest_tables(dsts, with_nexthop=True)

    def ecmp(self, export, dist, rows, srcs):
        """Every shortest route of each (rows[i], srcs[i]) pair, lexicographic
        order (ecmp.hip): list of int32 [n_i, len_i] vertex arrays."""
        self.load(export)
        paths = self.ctx.ecmp_counts(dist)
        rows = np.asarray(rows, np.int64)
        srcs = np.asarray(srcs, np.int64)
        cnt = paths[rows, srcs].astype(np.int64)
        if (paths[rows, srcs] > np.uint64(1 << 40)).any():
            raise MemoryError("ECMP set too large to enumerate")
        lens = dist[rows, srcs].astype(np.int64) + 1
        rr = np.repeat(rows, cnt)
        ss = np.repeat(srcs, cnt)
        starts = np.cumsum(cnt) - cnt
        ranks = np.arange(int(cnt.sum()), dtype=np.int64) - np.repeat(starts, cnt)
        max_len = int(lens[cnt > 0].max()) if (cnt > 0).any() else 1
        verts = self.ctx.ecmp_routes(dist, paths, rr, ss, ranks.astype(np.uint64), max_len)
        out, k = [], 0
        for i in range(rows.shape[0]):
            out.append(verts[k:k + cnt[i], :lens[i]] if cnt[i] else verts[0:0, :0])
            k += int(cnt[i])
        return out

    def expand(self, export, tables, rows, dsts, last_port):
        """Flow entries of many pairs (routes.hip): (offsets, switch ids, ports)."""
        self.load(export)
        parent, port, hops = tables
        return self.ctx.expand_routes(parent, port, hops, rows, dsts, last_port)

    def close(self):
        self.ctx.close()


class TableCache(object):
    """Per-graph cache of computed table rows, keyed by dense vertex id."""

    def __init__(self, export):
        self.export = export
        self.dfs_row = {}          # source vertex -> row
        self.dfs = None            # (parent, port, hops)
        self.sp_row = {}           # destination vertex -> row
        self.sp = None             # (dist, nh, nh_port)
        self.rows_computed = 0     # rows sent to the GPU (both modes)
        self.rows_inherited = 0    # rows kept across a graph change

    def inherit(self, old, diff):
        """Keep the rows of ``old`` (a cache of the previous graph over the
        same vertex set) that the link changes in ``diff`` cannot alter
        (:mod:`sdnmpi_amd.incremental`); the rest are recomputed on demand."""
        from .incremental import dfs_rows_affected, sp_rows_affected
        if old.dfs is not None and old.dfs[2] is not None:
            srcs = np.empty(len(old.dfs_row), np.int64)
            for v, r in old.dfs_row.items():
                srcs[r] = v
            keep = ~dfs_rows_affected(old.dfs[0], old.dfs[2], srcs, diff)
            if keep.any():
                self.dfs = tuple(a[keep] for a in old.dfs)
                self.dfs_row = {int(v): i for i, v in enumerate(srcs[keep].tolist())}
                self.rows_inherited += int(keep.sum())
        if old.sp is not None and old.sp[1] is not None:
            dsts = np.empty(len(old.sp_row), np.int64)
            for v, r in old.sp_row.items():
                dsts[r] = v
            keep = ~sp_rows_affected(old.sp[0], old.sp[1], diff)
            if keep.any():
                self.sp = tuple(a[keep] for a in old.sp)
                self.sp_row = {int(v): i for i, v in enumerate(dsts[keep].tolist())}
                self.rows_inherited += int(keep.sum())

    @staticmethod
    def _append(old, new):
        if old is None:
            return new
        return tuple(np.concatenate([a, b]) if a is not None else None
                     for a, b in zip(old, new))

    def dfs_rows(self, engine, wanted, batch=()):
        missing = [v for v in dict.fromkeys(list(wanted) + list(batch))
                   if v not in self.dfs_row]
        if missing:
            tabs = engine.dfs_tables(self.export, np.asarray(missing, np.int32))
            self.rows_computed += len(missing)
            base = 0 if self.dfs is None else self.dfs[0].shape[0]
            self.dfs = self._append(self.dfs, tabs)
            for i, v in enumerate(missing):
                self.dfs_row[v] = base + i
        return self.dfs

    def sp_rows(self, engine, wanted, batch=()):
        missing = [v for v in dict.fromkeys(list(wanted) + list(batch))
                   if v not in self.sp_row]
        if missing:
            tabs = engine.shortest_tables(self.export, np.asarray(missing, np.int32))
            self.rows_computed += len(missing)
            base = 0 if self.sp is None else self.sp[0].shape[0]
            self.sp = self._append(self.sp, tabs)
            for i, v in enumerate(missing):
                self.sp_row[v] = base + i
        return self.sp


def tree_path(parent_row, s, d):
    """Dense vertex sequence s..d along a per-source tree row ([] if d is
    unreachable)."""
    if parent_row[d] < 0:
        return []
    seq = [int(d)]
    x = int(d)
    limit = parent_row.shape[0]
    while x != s:
        x = int(parent_row[x])
        seq.append(x)
        if len(seq) > limit:
            raise RuntimeError("route table corrupt: cycle at vertex %d" % x)
    seq.reverse()
    return seq


def shortest_paths_lex(row_ptr, col, dist_row, s, d):
    """Every shortest s->d vertex sequence in lexicographic dpid order (the
    order _find_routes_bfs returns them, topology_db.py:95-122): walk the
    shortest-path DAG (dist_row = hops to d) taking successors ascending."""
    INF = _native.DIST_INF
    if int(dist_row[s]) == INF:
        return []
    out = []
    acc = [int(s)]

    def walk(x):
        if x == d:
            out.append(list(acc))
            return
        want = int(dist_row[x]) - 1
        for e in range(int(row_ptr[x]), int(row_ptr[x + 1])):
            n = int(col[e])
            if int(dist_row[n]) == want:
                acc.append(n)
                walk(n)
                acc.pop()

    walk(int(s))
    return out


def expand_tree_paths(parent, port, rows, dsts, max_len=None):
    """Vectorised tree walks for many (row, dst) pairs.

    Returns ``(off, verts, ports)``: pair i's vertex sequence is
    ``verts[off[i]:off[i+1]]`` (source first) and ``ports[j]`` is the port on
    ``verts[j]`` toward ``verts[j+1]`` (undefined for the last vertex).
    Unreachable pairs get an empty range.
    """
    rows = np.asarray(rows, np.int64)
    dsts = np.asarray(dsts, np.int64)
    n = rows.shape[0]
    reach = parent[rows, dsts] >= 0
    # walk upward from the destinations collecting (vertex, in-port)
    chain_v, chain_p = [dsts.copy()], [np.full(n, -1, np.int64)]
    cur = dsts.copy()
    active = reach.copy()
    limit = parent.shape[1] if max_len is None else max_len
    for _ in range(limit):
        par = parent[rows, cur]
        done = par == cur                          # reached the root
        active &= ~done
        if not active.any():
            break
        prt = port[rows, cur]
        cur = np.where(active, par, cur)
        chain_v.append(np.where(active, cur, -1))
        chain_p.append(np.where(active, prt, -1))
    V = np.stack(chain_v, 1)      # [n, L] dst first
    P = np.stack(chain_p, 1)      # in-port of chain_v[k-1] from chain_v[k]
    lens = np.where(reach, (V >= 0).sum(1), 0)
    off = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    verts = np.empty(off[-1], np.int64)
    ports = np.full(off[-1], -1, np.int64)
    for i in np.nonzero(reach)[0]:
        L = lens[i]
        verts[off[i]:off[i + 1]] = V[i, :L][::-1]
        # chain slot k holds V[k] and P[k] = port on V[k] toward V[k-1];
        # source-first position j is V[L-1-j], its out-port P[L-1-j]
        ports[off[i]:off[i + 1] - 1] = P[i, 1:L][::-1]
    return off, verts, ports
