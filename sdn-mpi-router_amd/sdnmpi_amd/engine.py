"""Route tables on the GPU and their expansion into fdb lists.

``RouteEngine`` owns one native context (``_native.Context``: one HIP device,
or several of one node, sharded by source) and the graph uploaded to it.
Tables stay in HBM: the engine returns them as torch tensors on the primary
device (torch is only the device-memory plumbing here) and ``TableCache``
keeps, per uploaded graph, the per-source DFS tables (default route,
reference ``_find_route_dfs``, ``sdnmpi/util/topology_db.py:59-84``) and the
per-destination shortest tables (``_find_routes_bfs``, :86-122) computed so
far, within a byte budget.  A single ``find_route`` copies back one table row
(V entries, kept in a small host cache), a batch is expanded on the device.
Expansion follows the reference's ``_route_to_fdb`` (:127-138): one
``(dpid, out_port)`` per switch on the path, the last one being the
destination switch's host port or ``OFPP_LOCAL``.

The cache is storage-agnostic: an engine may hand back numpy arrays instead
(the CPU tests' oracle-backed double), and every array operation below
dispatches on the array type.
"""

import collections
import os

import numpy as np

from . import _native
from .graph import empty_csr

__all__ = ["RouteEngine", "TableCache", "tree_path", "expand_tree_paths",
           "shortest_paths_lex", "DEFAULT_TABLE_BUDGET"]

# bytes of device tables one TableCache keeps per route mode before it
# evicts rows (SDNROUTE_TABLE_BUDGET overrides); the torus 32^3 default-route
# tables of every source are 12.9 GB, Jellyfish 100k's would be 120 GB
DEFAULT_TABLE_BUDGET = int(os.environ.get("SDNROUTE_TABLE_BUDGET", str(24 << 30)))
HOST_ROW_CACHE = 256            # table rows kept on the host for find_route


# ------------------------------------------------------- array dispatch --

def _is_np(a):
    return isinstance(a, np.ndarray)


def _take(a, idx):
    """Rows ``idx`` (int64 numpy) of a table."""
    if a is None:
        return None
    if _is_np(a):
        return a[idx]
    import torch
    return a.index_select(0, torch.as_tensor(idx, dtype=torch.int64, device=a.device))


def _cat(blocks):
    if blocks[0] is None:
        return None
    if _is_np(blocks[0]):
        return np.concatenate(blocks)
    import torch
    return torch.cat(blocks)


def _host(a):
    if a is None or _is_np(a):
        return a
    return a.cpu().numpy()


def _nbytes(a):
    if a is None:
        return 0
    return a.nbytes if _is_np(a) else a.element_size() * a.numel()


class RouteEngine(object):
    """The GPU route engine of one TopologyDB: HIP device ``device`` (int),
    or the devices of a list (single-process multi-GPU, sources sharded over
    them; tables assembled on the first)."""

    def __init__(self, device=0):
        import torch
        self._torch = torch
        self.ctx = _native.Context(device)
        self.devices = self.ctx.devices
        self.dev = torch.device("cuda", self.devices[0])
        self._loaded = None

    # -- plumbing -------------------------------------------------------
    def _ready(self):
        # the library runs on its own stream: torch work that produced its
        # inputs (or last used the memory of its outputs) must be done
        self._torch.cuda.current_stream(self.dev).synchronize()

    def _ids(self, ids):
        return self._torch.from_numpy(np.ascontiguousarray(ids, np.int32)).to(self.dev)

    def _empty(self, n, V, dtype):
        return self._torch.empty((n, V), dtype=dtype, device=self.dev)

    def load(self, export):
        if self._loaded is not export:
            self.ctx.upload(export.csr if export.csr.V else empty_csr())
            self._loaded = export

    # -- tables (device-resident) ---------------------------------------
    def dfs_tables(self, export, srcs, with_hops=True):
        """(parent, port, hops) int32 [S, V] tensors on the primary device."""
        self.load(export)
        t = self._torch
        S, V = len(srcs), export.csr.V
        par = self._empty(S, V, t.int32)
        prt = self._empty(S, V, t.int32)
        hop = self._empty(S, V, t.int32) if with_hops else None
        if S and V:
            ts = self._ids(srcs)
            self._ready()
            self.ctx.dfs_tables_device(ts.data_ptr(), S, par.data_ptr(), prt.data_ptr(),
                                       hop.data_ptr() if hop is not None else 0)
            self.ctx.synchronize()          # also raises on a tripped kernel watchdog
        return par, prt, hop

    def shortest_tables(self, export, dsts):
        """(dist int16 [D, V] holding u16, nh, nh_port int32) on the device."""
        self.load(export)
        t = self._torch
        D, V = len(dsts), export.csr.V
        dist = self._empty(D, V, t.int16)
        nh = self._empty(D, V, t.int32)
        nhp = self._empty(D, V, t.int32)
        if D and V:
            td = self._ids(dsts)
            self._ready()
            self.ctx.shortest_tables_device(td.data_ptr(), D, dist.data_ptr(), nh.data_ptr(),
                                            nhp.data_ptr())
            self.ctx.synchronize()
        return dist, nh, nhp

    def ecmp(self, export, dist, rows, srcs):
        """Every shortest route of each (rows[i], srcs[i]) pair, lexicographic
        order (ecmp.hip): list of int32 [n_i, len_i] vertex arrays.  ``dist``
        holds the destination rows the pairs use (device tensor)."""
        self.load(export)
        t = self._torch
        rows = np.asarray(rows, np.int64)
        srcs = np.asarray(srcs, np.int64)
        if rows.size == 0:
            return []
        dist = dist.contiguous()
        R, V = int(dist.shape[0]), export.csr.V
        paths = self._empty(R, V, t.int64)
        self._ready()
        self.ctx.ecmp_counts_device(dist.data_ptr(), R, paths.data_ptr())
        self.ctx.synchronize()
        flat = t.as_tensor(rows * V + srcs, dtype=t.int64, device=self.dev)
        cnt_u = paths.view(-1).index_select(0, flat).cpu().numpy().view(np.uint64)
        if (cnt_u > np.uint64(1 << 40)).any():
            raise MemoryError("ECMP set too large to enumerate")
        cnt = cnt_u.astype(np.int64)
        dsel = dist.view(-1).index_select(0, flat).cpu().numpy().view(np.uint16)
        lens = dsel.astype(np.int64) + 1
        total = int(cnt.sum())
        out = []
        if total == 0:
            return [np.zeros((0, 0), np.int32) for _ in range(rows.shape[0])]
        rr = np.repeat(rows, cnt).astype(np.int32)
        ss = np.repeat(srcs, cnt).astype(np.int32)
        starts = np.cumsum(cnt) - cnt
        ranks = (np.arange(total, dtype=np.int64) - np.repeat(starts, cnt)).astype(np.uint64)
        max_len = int(lens[cnt > 0].max())
        d_rr, d_ss = self._ids(rr), self._ids(ss)
        d_rk = t.from_numpy(ranks.view(np.int64)).to(self.dev)
        verts = t.empty((total, max_len), dtype=t.int32, device=self.dev)
        self._ready()
        self.ctx.ecmp_routes_device(dist.data_ptr(), paths.data_ptr(), R, d_rr.data_ptr(),
                                    d_ss.data_ptr(), d_rk.data_ptr(), total, max_len,
                                    verts.data_ptr())
        self.ctx.synchronize()
        verts = verts.cpu().numpy()
        k = 0
        for i in range(rows.shape[0]):
            out.append(verts[k:k + cnt[i], :lens[i]] if cnt[i] else verts[0:0, :0])
            k += int(cnt[i])
        return out

    def expand(self, export, tables, rows, dsts, last_port):
        """Flow entries of many pairs (routes.hip) from device tables:
        (offsets int64 [n+1], switch ids int32, ports int32) on the host.
        Only the table rows the pairs use go through the expansion."""
        self.load(export)
        t = self._torch
        parent, port, hops = tables
        rows = np.asarray(rows, np.int64)
        n = rows.shape[0]
        off = np.zeros(n + 1, np.int64)
        if n == 0:
            return off, np.zeros(0, np.int32), np.zeros(0, np.int32)
        urows, inv = np.unique(rows, return_inverse=True)
        sel = t.as_tensor(urows, dtype=t.int64, device=self.dev)
        par = parent.index_select(0, sel)
        prt = port.index_select(0, sel)
        hop = hops.index_select(0, sel)
        d_rows = self._ids(inv)
        d_dsts = self._ids(dsts)
        d_last = self._ids(last_port)
        d_off = t.empty(n + 1, dtype=t.int64, device=self.dev)
        self._ready()
        self.ctx.route_offsets_device(hop.data_ptr(), d_rows.data_ptr(), d_dsts.data_ptr(), n,
                                      d_off.data_ptr(), nrows=len(urows))
        self.ctx.synchronize()
        off = d_off.cpu().numpy()
        total = int(off[-1])
        sw = t.empty(max(total, 1), dtype=t.int32, device=self.dev)
        hp = t.empty(max(total, 1), dtype=t.int32, device=self.dev)
        self.ctx.expand_routes_device(par.data_ptr(), prt.data_ptr(), len(urows),
                                      d_rows.data_ptr(), d_dsts.data_ptr(), d_last.data_ptr(), n,
                                      d_off.data_ptr(), sw.data_ptr(), hp.data_ptr())
        self.ctx.synchronize()
        return off, sw[:total].cpu().numpy(), hp[:total].cpu().numpy()

    def edge_ports(self, ends, ports):
        """Flood-port mask (sdnr_edge_ports, reference topology.py:150-155):
        bool [n] -- ``ports`` keys that are no link end (``ends`` sorted)."""
        return self.ctx.edge_ports(ends, ports)

    def close(self):
        self.ctx.close()


class _Rows(object):
    """Table rows of one route mode (tuple of [n, V] arrays, one row per
    vertex), appended in blocks, merged on use, bounded by a byte budget with
    oldest-first eviction."""

    def __init__(self, budget):
        self.budget = budget
        self.blocks = []           # list of tuples, merged lazily
        self.order = []            # vertex of every row, row order
        self.row = {}              # vertex -> row
        self.row_bytes = 0
        self.host = collections.OrderedDict()   # vertex -> host row tuple (LRU)

    def __contains__(self, v):
        return v in self.row

    def __len__(self):
        return len(self.order)

    def cap(self):
        """Rows the budget holds (at least one)."""
        return max(1, self.budget // self.row_bytes) if self.row_bytes else 1 << 62

    def tables(self):
        if len(self.blocks) > 1:
            self.blocks = [tuple(_cat([b[i] for b in self.blocks])
                                 for i in range(len(self.blocks[0])))]
        return self.blocks[0] if self.blocks else None

    def add(self, verts, tabs):
        if not verts:
            return
        if not self.row_bytes:
            self.row_bytes = sum(_nbytes(a) for a in tabs) // len(verts)
        base = len(self.order)
        self.blocks.append(tabs)
        for i, v in enumerate(verts):
            self.row[v] = base + i
        self.order.extend(verts)

    def keep(self, mask):
        """Keep the rows where ``mask`` (bool numpy [n]) is set."""
        idx = np.nonzero(np.asarray(mask, bool))[0]
        if idx.size == len(self.order):
            return
        tabs = self.tables()
        self.blocks = [tuple(_take(a, idx) for a in tabs)] if idx.size else []
        self.order = [self.order[i] for i in idx.tolist()]
        self.row = {v: i for i, v in enumerate(self.order)}
        self.host.clear()

    def make_room(self, n, protect):
        """Evict the oldest rows not in ``protect`` until n more fit."""
        over = len(self.order) + n - self.cap()
        if over <= 0:
            return
        mask = np.ones(len(self.order), bool)
        for i, v in enumerate(self.order):
            if over <= 0:
                break
            if v not in protect:
                mask[i] = False
                over -= 1
        self.keep(mask)

    def host_row(self, v):
        """One row of every table, on the host (small LRU)."""
        hit = self.host.get(v)
        if hit is not None:
            self.host.move_to_end(v)
            return hit
        r = self.row[v]
        tabs = self.tables()
        rows = tuple(_host(a[r:r + 1])[0] if a is not None else None for a in tabs)
        self.host[v] = rows
        if len(self.host) > HOST_ROW_CACHE:
            self.host.popitem(last=False)
        return rows


class TableCache(object):
    """Per-graph cache of computed table rows, keyed by dense vertex id."""

    def __init__(self, export, budget=None):
        self.export = export
        b = DEFAULT_TABLE_BUDGET if budget is None else int(budget)
        V = export.csr.V
        self.dfs = _Rows(b)        # (parent, port, hops) per source
        self.sp = _Rows(b)         # (dist, nh, nh_port) per destination
        self.dfs.row_bytes = 12 * V    # int32 parent + port + hops
        self.sp.row_bytes = 10 * V     # u16 dist + int32 nh + nh_port
        self.rows_computed = 0     # rows sent to the GPU (both modes)
        self.rows_inherited = 0    # rows kept across a graph change

    # back-compat views used by callers/tests
    @property
    def dfs_row(self):
        return self.dfs.row

    @property
    def sp_row(self):
        return self.sp.row

    def inherit(self, old, diff):
        """Keep the rows of ``old`` (a cache of the previous graph over the
        same vertex set) that the link changes in ``diff`` cannot alter
        (:mod:`sdnmpi_amd.incremental`); the rest are recomputed on demand.
        The tests run where the tables live (device tensors stay on the
        device)."""
        from .incremental import dfs_rows_affected, sp_rows_affected
        self.dfs.budget, self.sp.budget = old.dfs.budget, old.sp.budget
        for mine, theirs, test in (
                (self.dfs, old.dfs, lambda t, vs: dfs_rows_affected(t[0], t[2], vs, diff)),
                (self.sp, old.sp, lambda t, vs: sp_rows_affected(t[0], t[1], diff))):
            tabs = theirs.tables()
            if tabs is None or tabs[1] is None or (mine is self.dfs and tabs[2] is None):
                continue
            verts = np.asarray(theirs.order, np.int64)
            keep = ~np.asarray(test(tabs, verts), bool)
            if keep.any():
                idx = np.nonzero(keep)[0]
                mine.add(verts[idx].tolist(), tuple(_take(a, idx) for a in tabs))
                mine.row_bytes = theirs.row_bytes
                self.rows_inherited += int(idx.size)

    def _rows(self, store, compute, wanted, batch):
        """Ensure the rows of ``wanted`` (and as many of ``batch`` as the budget
        allows) exist; return the merged tables."""
        wanted = list(dict.fromkeys(int(v) for v in wanted))
        missing = [v for v in wanted if v not in store]
        miss = set(missing)
        extra = [int(v) for v in batch if int(v) not in store and int(v) not in miss] \
            if batch else []
        if missing or extra:
            cap = store.cap()
            room = cap - len(store) - len(missing)
            extra = extra[:max(0, room)]
            todo = missing + extra
            store.make_room(len(todo), set(wanted))
            tabs = compute(np.asarray(todo, np.int32))
            self.rows_computed += len(todo)
            store.add(todo, tabs)
        return store.tables()

    def dfs_rows(self, engine, wanted, batch=()):
        return self._rows(self.dfs, lambda s: engine.dfs_tables(self.export, s),
                          wanted, batch)

    def sp_rows(self, engine, wanted, batch=()):
        return self._rows(self.sp, lambda d: engine.shortest_tables(self.export, d),
                          wanted, batch)


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
    dist_row = np.asarray(dist_row).view(np.uint16) if np.asarray(dist_row).dtype == np.int16 \
        else dist_row
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
