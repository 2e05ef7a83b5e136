"""Route tables on the GPU and their expansion into fdb lists.

``RouteEngine`` owns one native context (``_native.Context``: one HIP device,
or several of one node, sharded by source) and the graph uploaded to it.
Tables stay in HBM: the engine returns them as torch tensors on the primary
device (torch is only the device-memory plumbing here) and ``TableCache``
keeps, per uploaded graph, the per-source DFS tables (default route,
reference ``_find_route_dfs``, ``sdnmpi/util/topology_db.py:59-84``) and the
per-destination shortest tables (``_find_routes_bfs``, :86-122) computed so
far, within a byte budget, in a fixed-capacity pool of compact rows:

* default route: one 4-byte tree word per vertex -- ``parent | port << 16``
  (V <= 65535, 16-bit ports: sdnr_dfs_tables_packed's layout) or ``parent |
  slot << 26`` (sdnr_dfs_tables_slots') -- plus the tree depth (u16 for
  V <= 65535, else int32): 6 bytes per entry where the int32 parent / port /
  hops tables take 12 (8 on fabrics above 65,535 switches);
* shortest route: u16 distance plus the next hop (u16 for V <= 65535): 4
  bytes per entry; the next hop's port is looked up in the CSR on demand.

Slots are taken from a free list and given back on eviction or when a graph
change invalidates the row; the pool is allocated once (min(budget rows, V)
rows) and no operation copies it, free slots hold all-unreached rows.  A single
``find_route`` copies back one table row (V entries, kept in a small host
cache), a batch is expanded on the device.  Expansion follows the
reference's ``_route_to_fdb`` (:127-138): one ``(dpid, out_port)`` per switch
on the path, the last one being the destination switch's host port or
``OFPP_LOCAL``.

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
           "shortest_paths_lex", "count_shortest_paths", "ECMP_LIMIT", "DEFAULT_TABLE_BUDGET", "tree_layout", "dfs_row_bytes",
           "sp_row_bytes"]

# bytes of device tables one TableCache keeps per route mode before it
# evicts rows (SDNROUTE_TABLE_BUDGET overrides); the torus 32^3 default-route
# tables of every source take 6.4 GB in the pool, Jellyfish 100k's 80 GB
# Largest ECMP set either find_route(..., multiple=True) path builds; above
# it both raise MemoryError (the reference's enumeration runs out of memory
# long before).
ECMP_LIMIT = 1 << 40
DEFAULT_TABLE_BUDGET = int(os.environ.get("SDNROUTE_TABLE_BUDGET", str(24 << 30)))
HOST_ROW_CACHE = 256            # table rows kept on the host for find_route
COMPUTE_ROWS = 4096             # rows per engine call when filling the pool

PORT16, SLOT, INT32 = "port16", "slot", "int32"


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


def _host(a):
    if a is None or _is_np(a):
        return a
    return a.cpu().numpy()


def _nbytes(a):
    if a is None:
        return 0
    return a.nbytes if _is_np(a) else a.element_size() * a.numel()


def _i64(a):
    return a.astype(np.int64) if _is_np(a) else a.to(dtype=_torch().int64)


def _torch():
    import torch
    return torch


# ------------------------------------------------------- compact layouts --

def tree_layout(csr):
    """4-byte tree layout the cache keeps default-route rows in."""
    V = csr.V
    port = np.asarray(csr.port)
    if V <= 0xFFFF and (port.size == 0 or (port.min() >= 0 and port.max() < 0xFFFF)):
        return PORT16
    if V < (1 << 26) and csr.max_degree() <= 63:
        return SLOT
    return INT32


def _hops_dtype(V):
    return "int16" if V <= 0xFFFF else "int32"


def _nh_dtype(V):
    return "int16" if V <= 0xFFFF else "int32"


def dfs_row_bytes(csr):
    """Bytes of one default-route row in the cache."""
    lay = tree_layout(csr)
    hb = 2 if csr.V <= 0xFFFF else 4
    return (4 + hb if lay != INT32 else 12) * csr.V


def sp_row_bytes(csr):
    return (2 + (2 if csr.V <= 0xFFFF else 4)) * csr.V


def _u16(a):
    """u16 values stored in int16 (0xFFFF: -1) as int64."""
    x = _i64(a) & 0xFFFF
    return (x - ((x == 0xFFFF) * 0x10000)) if _is_np(x) else x.masked_fill(x == 0xFFFF, -1)


class Wide(object):
    """Read view of a compact table: indexing returns int64 values (u16
    planes widened, 0xFFFF -> -1; tree words decoded to parents)."""

    def __init__(self, arr, kind):
        self.arr = arr
        self.kind = kind               # "u16" | "u16raw" | "int" | PORT16 | SLOT
        self.shape = arr.shape

    def __getitem__(self, idx):
        w = self.arr[idx]
        if self.kind == "u16":
            return _u16(w)
        if self.kind == "u16raw":                  # distances: 0xFFFF stays INF
            return _i64(w) & 0xFFFF
        if self.kind == "int":
            return _i64(w)
        return tree_parent(w, self.kind)


def tree_parent(w, layout):
    """Parents (int64, -1 unreached) of tree words (int32 storage)."""
    x = _i64(w) & 0xFFFFFFFF
    if layout == PORT16:
        p = x & 0xFFFF
        bad = p == 0xFFFF
    else:
        p = x & 0x3FFFFFF
        bad = x == 0xFFFFFFFF
    if _is_np(p):
        p[bad] = -1
        return p
    return p.masked_fill(bad, -1)


def tree_port(w, layout, row_ptr, port, parent=None):
    """Ports (int64, -1 for the root / unreached) of tree words.  Slot trees
    look the port up in the CSR (row_ptr / port arrays of the tree's type)."""
    x = _i64(w) & 0xFFFFFFFF
    if layout == PORT16:
        t = x >> 16
        return _where(t == 0xFFFF, -1, t)
    slot = x >> 26
    par = tree_parent(w, layout) if parent is None else parent
    none = (par < 0) | (slot == 63)
    if _is_np(x):
        pz = np.where(none, 0, par)
        idx = np.where(none, 0, row_ptr[pz] + slot)
        return np.where(none, -1, np.asarray(port, np.int64)[idx])
    pz = par.masked_fill(none, 0)
    idx = (row_ptr[pz] + slot).masked_fill(none, 0)
    return port[idx].to(x.dtype).masked_fill(none, -1)


def _empty_rows(a, n):
    """Uninitialised [n] + a.shape[1:] array of a's type (and device)."""
    if _is_np(a):
        return np.empty((n,) + tuple(a.shape[1:]), a.dtype)
    return _torch().empty((n,) + tuple(a.shape[1:]), dtype=a.dtype, device=a.device)


def _where(c, a, b):
    if _is_np(b):
        return np.where(c, a, b)
    return b.masked_fill(c, a)


def _edge_keys_host(csr):
    """(keys int64 ascending = x * V + col of every CSR entry, port int32)."""
    rp = np.asarray(csr.row_ptr, np.int64)
    keys = np.repeat(np.arange(csr.V, dtype=np.int64), np.diff(rp)) * csr.V + \
        np.asarray(csr.col, np.int64)
    return keys, np.asarray(csr.port, np.int32)


def _next_hop_port(nh, keys, port, V):
    """CSR port of edge (x, nh[r, x]) for every entry of an int64 next-hop
    block (-1 where nh < 0); numpy or device tensors."""
    if keys.shape[0] == 0:
        return nh * 0 - 1
    n = nh.shape[-1]
    if _is_np(nh):
        x = np.broadcast_to(np.arange(n, dtype=np.int64), nh.shape)
        ok = nh >= 0
        e = np.minimum(np.searchsorted(keys, np.where(ok, x * V + nh, 0)), keys.shape[0] - 1)
        return np.where(ok, port[e].astype(np.int64), -1)
    t = _torch()
    x = t.arange(n, dtype=t.int64, device=nh.device).expand_as(nh)
    ok = nh >= 0
    k = (x * V + nh).masked_fill(~ok, 0)
    e = t.searchsorted(keys, k).clamp_(max=keys.shape[0] - 1)
    return port[e].to(t.int64).masked_fill(~ok, -1)


def pack_host_tree(parent, port, csr, layout):
    """Host (numpy) tables -> tree words (int32 storage): the test double's
    counterpart of sdnr_tree_pack."""
    p = np.asarray(parent, np.int64)
    if layout == PORT16:
        t = (p & 0xFFFF) | ((np.asarray(port, np.int64) & 0xFFFF) << 16)
    else:
        V = csr.V
        rp = np.asarray(csr.row_ptr, np.int64)
        src = np.repeat(np.arange(V, dtype=np.int64), np.diff(rp))
        keys = src * V + np.asarray(csr.col, np.int64)
        v = np.broadcast_to(np.arange(V, dtype=np.int64), p.shape)
        ok = p >= 0
        e = np.searchsorted(keys, np.where(ok, p, 0) * V + v)
        slot = np.where(ok, e - rp[np.where(ok, p, 0)], 0)
        slot = np.where(p == v, 63, slot)
        t = np.where(ok, p | (slot << 26), 0xFFFFFFFF)
    return (t & 0xFFFFFFFF).astype(np.uint32).view(np.int32)


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
        self._csr_dev = None        # (export, row_ptr int64, port int32) on the device
        self._keys_dev = None       # (export, edge keys int64, port int32) on the device

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

    def csr_device(self, export):
        """(row_ptr int64, port int32) of the export on the device (slot trees
        look their ports up here)."""
        if self._csr_dev is None or self._csr_dev[0] is not export:
            t = self._torch
            c = export.csr
            self._csr_dev = (export, t.from_numpy(np.asarray(c.row_ptr, np.int64)).to(self.dev),
                             t.from_numpy(np.asarray(c.port, np.int32)).to(self.dev))
        return self._csr_dev[1], self._csr_dev[2]

    def edge_keys_device(self, export):
        """(keys int64 = x * V + col per CSR entry, ascending; port int32) on
        the device: the next-hop port lookups of the shortest tables."""
        if self._keys_dev is None or self._keys_dev[0] is not export:
            keys, port = _edge_keys_host(export.csr)
            t = self._torch
            self._keys_dev = (export, t.from_numpy(keys).to(self.dev),
                              t.from_numpy(port).to(self.dev))
        return self._keys_dev[1], self._keys_dev[2]

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

    def empty_rows(self, n, V, dtypes):
        """Uninitialised [n, V] device tensors of the named dtypes."""
        return tuple(self._empty(n, V, getattr(self._torch, d)) for d in dtypes)

    def dfs_tree_tables(self, export, srcs, layout, out=None):
        """Default-route trees as 4-byte words of ``layout`` (PORT16 / SLOT)
        plus depths (int16 holding u16 for V <= 65535, else int32), from the
        DFS kernels directly (sdnr_dfs_tables_tree) -- into ``out`` (two
        [S, V] tensors, e.g. pool rows) or new tensors."""
        self.load(export)
        t = self._torch
        S, V = len(srcs), export.csr.V
        if out is None:
            out = self.empty_rows(S, V, ("int32", _hops_dtype(V)))
        tree, dep = out
        if S and V:
            ts = self._ids(srcs)
            self._ready()
            self.ctx.dfs_tables_tree_device(
                ts.data_ptr(), S, tree.data_ptr(), dep.data_ptr(),
                _native.TREE_PORT16 if layout == PORT16 else _native.TREE_SLOT,
                dep.element_size())
            self.ctx.synchronize()          # also raises on a tripped kernel watchdog
        return tree, dep

    def pack_trees(self, export, parent, port, layout):
        """int32 tables -> tree words (int32 tensor), sdnr_tree_pack."""
        self.load(export)
        tree = self._torch.empty_like(parent)
        n = parent.numel()
        if n:
            self._ready()
            self.ctx.tree_pack_device(parent.data_ptr(), port.data_ptr(), n, tree.data_ptr(),
                                      _native.TREE_PORT16 if layout == PORT16
                                      else _native.TREE_SLOT)
            self.ctx.synchronize()
        return tree

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
        if (cnt_u > np.uint64(ECMP_LIMIT)).any():
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
        ``tables`` = (parent, port, hops) [k, V] of the rows the pairs use
        (int32, or any integer view the cache decodes to)."""
        self.load(export)
        t = self._torch
        par, prt, hop = (a.to(t.int32).contiguous() for a in tables)
        rows = np.asarray(rows, np.int64)
        n = rows.shape[0]
        off = np.zeros(n + 1, np.int64)
        if n == 0:
            return off, np.zeros(0, np.int32), np.zeros(0, np.int32)
        nrows = int(par.shape[0])
        d_rows = self._ids(rows)
        d_dsts = self._ids(dsts)
        d_last = self._ids(last_port)
        d_off = t.empty(n + 1, dtype=t.int64, device=self.dev)
        self._ready()
        self.ctx.route_offsets_device(hop.data_ptr(), d_rows.data_ptr(), d_dsts.data_ptr(), n,
                                      d_off.data_ptr(), nrows=nrows)
        self.ctx.synchronize()
        off = d_off.cpu().numpy()
        total = int(off[-1])
        lp = np.asarray(last_port)
        env = os.environ.get
        if tree_layout(export.csr) == PORT16 and (lp.size == 0 or
                                                  (lp.min() >= 0 and lp.max() <= 0xFFFF)) \
                and env("SDNROUTE_ROUTE_OUT", "") != "int32" \
                and env("SDNROUTE_ROUTE_WALK", "") != "serial" and env("SDNROUTE_ROUTE_SEG", "") != "0" \
                and env("SDNROUTE_ROUTE_PACKED", "") != "0":
            # one u32 per entry (switch | port << 16): half the bytes written
            # and copied back; split on the host
            ent = t.empty(max(total, 1), dtype=t.int32, device=self.dev)
            self.ctx.expand_routes_packed_device(par.data_ptr(), prt.data_ptr(), nrows,
                                                 d_rows.data_ptr(), d_dsts.data_ptr(),
                                                 d_last.data_ptr(), n, d_off.data_ptr(),
                                                 ent.data_ptr())
            self.ctx.synchronize()
            e = ent[:total].cpu().numpy().view(np.uint32)
            return off, (e & 0xFFFF).astype(np.int32), (e >> 16).astype(np.int32)
        sw = t.empty(max(total, 1), dtype=t.int32, device=self.dev)
        hp = t.empty(max(total, 1), dtype=t.int32, device=self.dev)
        self.ctx.expand_routes_device(par.data_ptr(), prt.data_ptr(), nrows,
                                      d_rows.data_ptr(), d_dsts.data_ptr(), d_last.data_ptr(), n,
                                      d_off.data_ptr(), sw.data_ptr(), hp.data_ptr())
        self.ctx.synchronize()
        return off, sw[:total].cpu().numpy(), hp[:total].cpu().numpy()

    def dfs_rows_affected(self, export, tree, depth, layout, row_src, diff):
        """bool numpy [rows]: the pool rows (device tree words / int32
        parents ``tree`` and depths ``depth``, [rows, V]; ``row_src`` the
        source of each row, -1 for a free one) that the link changes of
        ``diff`` alter -- one device pass (sdnr_dfs_rows_affected), only
        the verdicts come back."""
        self.load(export)
        t = self._torch
        n = int(tree.shape[0])
        rm = [np.concatenate([diff.removed[0], diff.ported[0]]),
              np.concatenate([diff.removed[1], diff.ported[1]])]
        links = np.concatenate([np.stack(rm, 1).reshape(-1),
                                np.stack([diff.added[0], diff.added[1]], 1).reshape(-1)])
        nrm, nadd = int(rm[0].size), int(diff.added[0].size)
        if n == 0 or nrm + nadd == 0:
            return np.zeros(n, bool)
        tl = self._torch.from_numpy(links.astype(np.int32)).to(self.dev)
        ts = self._ids(row_src)
        out = t.empty(n, dtype=t.uint8, device=self.dev)
        lay = {PORT16: _native.TREE_PORT16, SLOT: _native.TREE_SLOT,
               INT32: _native.TREE_INT32}[layout]
        self._ready()
        self.ctx.dfs_rows_affected_device(tree.data_ptr(), depth.data_ptr(), lay,
                                          depth.element_size(), n, ts.data_ptr(),
                                          tl.data_ptr(), nrm, nadd, out.data_ptr())
        self.ctx.synchronize()              # raises if a row was not a tree
        return out.cpu().numpy().astype(bool)

    def edge_ports(self, ends, ports):
        """Flood-port mask (sdnr_edge_ports, reference topology.py:150-155):
        bool [n] -- ``ports`` keys that are no link end (``ends`` sorted)."""
        return self.ctx.edge_ports(ends, ports)

    def close(self):
        self.ctx.close()


class _Pool(object):
    """Table rows of one route mode in a fixed-capacity store.

    ``arrays`` is a tuple of [capacity, V] tables (device tensors or numpy);
    a row lives in a slot, ``row`` maps vertex -> slot, ``lru`` orders the
    vertices oldest first.  Adding takes slots from the free list (evicting
    the oldest unprotected rows when the budget is full), dropping gives
    them back and refills them with the ``blank`` row (all unreached), so a
    test over the whole store never sees garbage.  The store is allocated
    once, min(cap, V) rows, on first use; it is never grown, concatenated,
    re-indexed or copied."""

    def __init__(self, budget, row_bytes, blanks):
        self.budget = budget
        self.row_bytes = row_bytes
        self.blanks = blanks                   # fill value per table
        self.arrays = None
        self.size = 0                          # allocated slots
        self.row = {}
        self.lru = collections.OrderedDict()
        self.free = []
        self.host = collections.OrderedDict()  # vertex -> host row tuple (LRU)

    def __contains__(self, v):
        return v in self.row

    def __len__(self):
        return len(self.row)

    def cap(self):
        """Rows the budget holds (at least one)."""
        return max(1, self.budget // self.row_bytes) if self.row_bytes else 1 << 62

    def tables(self):
        return self.arrays

    def slot_vertices(self):
        """int64 numpy [size]: vertex of every slot, -1 for free ones."""
        s = np.full(self.size, -1, np.int64)
        if self.row:
            s[np.fromiter(self.row.values(), np.int64, len(self.row))] = \
                np.fromiter(self.row.keys(), np.int64, len(self.row))
        return s

    def _grow(self, need, like):
        """Make at least ``need`` slots exist.  The first call allocates the
        whole store -- min(cap, V) rows: a graph has at most V distinct rows
        -- so it never grows again (and never holds more than the budget)."""
        if need <= self.size:
            return
        V = int(like[0].shape[1]) if like[0].ndim > 1 else 1
        new = max(need, min(self.cap(), V))
        fresh = []
        for a, b in zip(like, self.blanks):
            shape = (new,) + tuple(a.shape[1:])
            if _is_np(a):
                z = np.full(shape, b, a.dtype)
            else:
                z = _torch().full(shape, b, dtype=a.dtype, device=a.device)
            fresh.append(z)
        if self.arrays is not None:
            for z, a in zip(fresh, self.arrays):
                z[:self.size] = a
        self.free.extend(range(new - 1, self.size - 1, -1))   # lowest slot popped first
        self.arrays = tuple(fresh)
        self.size = new

    def make_room(self, n, protect):
        """Evict the oldest rows not in ``protect`` until n more fit."""
        over = len(self.row) + n - self.cap()
        if over <= 0:
            return
        out = []
        for v in self.lru:
            if over <= 0:
                break
            if v not in protect:
                out.append(v)
                over -= 1
        self.drop(out)

    def drop(self, verts):
        """Give the slots of ``verts`` back (blank rows)."""
        slots = [self.row.pop(v) for v in verts if v in self.row]
        for v in verts:
            self.lru.pop(v, None)
            self.host.pop(v, None)
        if not slots:
            return
        self._blank(np.asarray(slots, np.int64))
        self.free.extend(slots)

    def _blank(self, idx):
        """Rows ``idx`` back to all-unreached (every free slot is blank)."""
        for a, b in zip(self.arrays, self.blanks):
            if _is_np(a):
                a[idx] = b
            else:
                a[_torch().as_tensor(idx, device=a.device)] = b

    def add(self, verts, tabs=None, fill=None, like=None):
        """Store rows for ``verts`` (room was made): either ``tabs`` ([n, V]
        each, already computed) or ``fill(out)``, which computes them into
        ``out`` -- views of the store itself when the slots taken are
        contiguous (the kernels write their rows in place: no copy), else
        fresh [n, V] arrays copied in afterwards.  ``like``: [0, V] arrays of
        the tables' types (the first call allocates the store from them)."""
        if not verts:
            return
        self._grow(len(self.row) + len(verts), tabs if tabs is not None else like)
        slots = [self.free.pop() for _ in verts]
        idx = np.asarray(slots, np.int64)
        contiguous = bool(np.all(np.diff(idx) == 1))
        n = len(slots)
        if tabs is None:
            try:
                if contiguous:
                    fill(tuple(a[slots[0]:slots[0] + n] for a in self.arrays))
                else:
                    tabs = tuple(_empty_rows(a, n) for a in self.arrays)
                    fill(tabs)
            except BaseException:
                # the kernels may have written part of the rows in place:
                # blank the slots before they go back
                self._blank(idx)
                self.free.extend(slots)
                raise
        if tabs is not None:
            for a, t in zip(self.arrays, tabs):
                if contiguous:
                    a[slots[0]:slots[0] + n] = t
                elif _is_np(a):
                    a[idx] = t
                else:
                    a.index_copy_(0, _torch().as_tensor(idx, device=a.device), t)
        for v, s in zip(verts, slots):
            self.row[v] = s
            self.lru[v] = None

    def host_row(self, v):
        """One row of every table, on the host (small LRU)."""
        hit = self.host.get(v)
        if hit is not None:
            self.host.move_to_end(v)
            return hit
        r = self.row[v]
        rows = tuple(_host(a[r:r + 1])[0] for a in self.arrays)
        self.host[v] = rows
        if len(self.host) > HOST_ROW_CACHE:
            self.host.popitem(last=False)
        return rows


class TableCache(object):
    """Per-graph cache of computed table rows, keyed by dense vertex id, in
    compact pools (module docstring).  ``retarget`` follows a graph change
    over the same vertex set in place: the rows the change can alter are
    dropped (:mod:`sdnmpi_amd.incremental`), the rest stay in their slots."""

    def __init__(self, export, budget=None):
        self.export = export
        b = DEFAULT_TABLE_BUDGET if budget is None else int(budget)
        csr = export.csr
        self.layout = tree_layout(csr)
        self.V = csr.V
        dfs_blank = (-1, -1, -1) if self.layout == INT32 else (-1, -1)
        self.dfs = _Pool(b, dfs_row_bytes(csr), dfs_blank)
        self.sp = _Pool(b, sp_row_bytes(csr), (-1, -1))
        self.rows_computed = 0     # rows sent to the GPU (both modes)
        self.rows_inherited = 0    # rows kept across a graph change

    # vertex -> row (slot) maps
    @property
    def dfs_row(self):
        return self.dfs.row

    @property
    def sp_row(self):
        return self.sp.row

    # -- decoded views ---------------------------------------------------
    def dfs_parent_hops(self):
        """(parent, hops) read views over the whole DFS pool (Wide)."""
        a = self.dfs.tables()
        if a is None:
            return None, None
        if self.layout == INT32:
            return Wide(a[0], "int"), Wide(a[2], "int")
        return Wide(a[0], self.layout), Wide(a[1], "u16" if self.V <= 0xFFFF else "int")

    def dfs_int32(self, slots, engine=None):
        """(parent, port, hops) int32-valued int64 tables of pool slots
        ``slots`` (array type of the pool)."""
        a = self.dfs.tables()
        sel = [_take(x, slots) for x in a]
        if self.layout == INT32:
            return tuple(_i64(x) for x in sel)
        par = tree_parent(sel[0], self.layout)
        if self.layout == PORT16:
            prt = tree_port(sel[0], PORT16, None, None)
        elif _is_np(sel[0]):
            c = self.export.csr
            prt = tree_port(sel[0], SLOT, np.asarray(c.row_ptr, np.int64), c.port, par)
        else:
            rp, pt = engine.csr_device(self.export)
            prt = tree_port(sel[0], SLOT, rp, pt, par)
        hop = _u16(sel[1]) if self.V <= 0xFFFF else _i64(sel[1])
        return par, prt, hop

    def dfs_host_row(self, v):
        """(parent, port) int64 numpy rows of source v (host LRU)."""
        row = self.dfs.host_row(v)
        if self.layout == INT32:
            return row[0], row[1]
        c = self.export.csr
        par = tree_parent(row[0], self.layout)
        return par, tree_port(row[0], self.layout, np.asarray(c.row_ptr, np.int64), c.port, par)

    def sp_dist_host_row(self, d):
        """u16 distances to destination d (host LRU)."""
        return np.asarray(self.sp.host_row(d)[0]).view(np.uint16)

    def sp_views(self):
        """(dist, nh) read views over the whole shortest pool (Wide)."""
        a = self.sp.tables()
        if a is None:
            return None, None
        return Wide(a[0], "u16raw"), Wide(a[1], "u16" if self.V <= 0xFFFF else "int")

    def sp_decoded(self, slots, engine=None):
        """(dist u16, nh int32, nh_port int32) numpy rows of pool slots.  The
        next hop's port -- ``links[x][nh].src.port_no``, the CSR port of edge
        (x, nh) -- is looked up where the rows live (on the device for a
        device pool), so only the three output planes cross to the host."""
        a = self.sp.tables()
        d = _take(a[0], slots)
        nh = _take(a[1], slots)
        nh = _u16(nh) if self.V <= 0xFFFF else _i64(nh)
        if _is_np(nh):
            keys, port = _edge_keys_host(self.export.csr)
        else:
            keys, port = engine.edge_keys_device(self.export)
        nhp = _next_hop_port(nh, keys, port, self.V)
        return (_host(d).view(np.uint16), _host(nh).astype(np.int32),
                _host(nhp).astype(np.int32))

    # -- graph changes ---------------------------------------------------
    def retarget(self, export, diff, engine=None):
        """Follow a link change over the same vertex set: drop the rows
        ``diff`` can alter (tests run where the tables live), keep the rest.
        Returns False when the compact layout no longer fits the new graph
        (the caller starts a new cache)."""
        from .incremental import dfs_rows_affected, sp_rows_affected
        if tree_layout(export.csr) != self.layout:
            return False
        self.export = export
        if self.dfs.row:
            verts = self.dfs.slot_vertices()
            a = self.dfs.tables()
            if engine is not None and not _is_np(a[0]):
                # the device pool: one kernel climbs the trees (incremental.hip)
                hit = engine.dfs_rows_affected(export, a[0], a[-1], self.layout, verts, diff)
            else:
                par, hop = self.dfs_parent_hops()
                hit = np.asarray(dfs_rows_affected(par, hop, verts, diff), bool)
            hit &= verts >= 0
            self.dfs.drop(verts[hit].tolist())
            if self.layout == SLOT:
                self._reslot(diff)
            self.rows_inherited += len(self.dfs.row)
        if self.sp.row:
            dist, nh = self.sp_views()
            verts = self.sp.slot_vertices()
            hit = np.asarray(sp_rows_affected(dist, nh, diff), bool) & (verts >= 0)
            self.sp.drop(verts[hit].tolist())
            self.rows_inherited += len(self.sp.row)
        self.dfs.host.clear()
        self.sp.host.clear()
        return True

    RESLOT_ROWS = 256             # pool rows per re-slot pass (bounded temporaries)

    def _reslot(self, diff):
        """Slot trees name a position in the parent's CSR row, and a link
        added to or removed from row u moves the later positions of row u.
        The rows kept across the change are still the right trees (the row
        tests above are about the tree, not the encoding), so every kept
        entry whose parent's row changed gets its slot re-derived from the
        new CSR: the position of (parent, v) in the new row of the parent.
        The edge exists: a kept tree's edges are unaffected by the change."""
        rows_changed = np.unique(np.concatenate([diff.removed[0], diff.added[0]]))
        a = self.dfs.tables()
        if a is None or rows_changed.size == 0 or not self.dfs.row:
            return
        csr = self.export.csr
        V = csr.V
        rp = np.asarray(csr.row_ptr, np.int64)
        # keys (p * V + v) -> global edge index, for the changed rows only
        lo, hi = rp[rows_changed], rp[rows_changed + 1]
        eidx = np.concatenate([np.arange(s, e, dtype=np.int64) for s, e in zip(lo, hi)]) \
            if rows_changed.size else np.zeros(0, np.int64)
        src = np.repeat(rows_changed.astype(np.int64), hi - lo)
        keys = src * V + np.asarray(csr.col, np.int64)[eidx]     # ascending: rows sorted
        changed = np.zeros(V, bool)
        changed[rows_changed] = True
        tree = a[0]
        used = np.sort(np.fromiter(self.dfs.row.values(), np.int64, len(self.dfs.row)))
        if _is_np(tree):
            xp_keys, xp_e, xp_rp, xp_ch = keys, eidx, rp, changed
        else:
            t = _torch()
            dv = tree.device
            xp_keys = t.from_numpy(keys).to(dv)
            xp_e = t.from_numpy(eidx).to(dv)
            xp_rp = t.from_numpy(rp).to(dv)
            xp_ch = t.from_numpy(changed).to(dv)
        for i in range(0, used.size, self.RESLOT_ROWS):
            sl = used[i:i + self.RESLOT_ROWS]
            w = _take(tree, sl)
            x = _i64(w) & 0xFFFFFFFF
            par = x & 0x3FFFFFF
            slot = x >> 26
            need = (x != 0xFFFFFFFF) & (slot != 63)
            if _is_np(x):
                need &= xp_ch[np.where(need, par, 0)]
                if not need.any():
                    continue
                r, v = np.nonzero(need)
                p = par[r, v]
                e = np.searchsorted(xp_keys, p * V + v)
                assert np.all(xp_keys[e] == p * V + v), "kept tree edge missing"
                x[r, v] = p | ((xp_e[e] - xp_rp[p]) << 26)
                tree[sl] = (x & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
            else:
                need &= xp_ch[par.masked_fill(~need, 0)]
                if not bool(need.any()):
                    continue
                r, v = t.nonzero(need, as_tuple=True)
                p = par[r, v]
                k = p * V + v
                e = t.searchsorted(xp_keys, k).clamp_(max=xp_keys.shape[0] - 1)
                if not bool((xp_keys[e] == k).all()):     # the kept tree edge must exist
                    raise AssertionError("kept tree edge missing")
                x[r, v] = p | ((xp_e[e] - xp_rp[p]) << 26)
                x = t.where(x >= (1 << 31), x - (1 << 32), x).to(t.int32)
                tree.index_copy_(0, t.as_tensor(sl, device=dv), x)

    # -- filling ---------------------------------------------------------
    def _rows(self, store, compute, wanted, batch):
        """Ensure the rows of ``wanted`` (and as many of ``batch`` as the
        budget allows) exist; return the pool tables."""
        wanted = list(dict.fromkeys(int(v) for v in wanted))
        missing = [v for v in wanted if v not in store]
        miss = set(missing)
        extra = [int(v) for v in batch if int(v) not in store and int(v) not in miss] \
            if batch else []
        for v in wanted:                       # recently used
            if v in store.lru:
                store.lru.move_to_end(v)
        if missing or extra:
            cap = store.cap()
            room = cap - len(store) - len(missing)
            extra = extra[:max(0, room)]
            todo = missing + extra
            store.make_room(len(todo), set(wanted))
            for i in range(0, len(todo), COMPUTE_ROWS):
                part = todo[i:i + COMPUTE_ROWS]
                compute(store, part)
            self.rows_computed += len(todo)
        return store.tables()

    def _dfs_compute(self, engine, store, part):
        """Default-route rows of sources ``part`` into the pool.  Compact
        layouts: the tree words and depths come straight from the DFS
        kernels the bench times (sdnr_dfs_tables_tree), written into the
        pool's own rows when the free slots are contiguous."""
        srcs = np.asarray(part, np.int32)
        if self.layout == INT32:
            store.add(part, engine.dfs_tables(self.export, srcs))
            return
        like = engine.empty_rows(0, self.V, ("int32", _hops_dtype(self.V)))
        store.add(part, fill=lambda out: engine.dfs_tree_tables(self.export, srcs, self.layout,
                                                                out),
                  like=like)

    def _sp_compute(self, engine, store, part):
        dist, nh, _ = engine.shortest_tables(self.export, np.asarray(part, np.int32))
        dt = _nh_dtype(self.V)
        if _is_np(dist):
            store.add(part, (dist.view(np.int16), nh.astype(dt)))
        else:
            store.add(part, (dist, nh.to(getattr(_torch(), dt))))

    def dfs_rows(self, engine, wanted, batch=()):
        return self._rows(self.dfs, lambda st, p: self._dfs_compute(engine, st, p), wanted, batch)

    def sp_rows(self, engine, wanted, batch=()):
        return self._rows(self.sp, lambda st, p: self._sp_compute(engine, st, p), wanted, batch)


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


def count_shortest_paths(row_ptr, col, dist_row, s, d, limit=None):
    """Number of shortest s->d routes: a DP over the part of the
    shortest-path DAG reachable from s, deepest level first (the host twin of
    ecmp.hip's per-row count).  Stops counting once ``limit`` is passed and
    returns limit + 1."""
    dist_row = np.asarray(dist_row)
    want = int(dist_row[s])
    levels = [[int(s)]]
    seen = {int(s)}
    for _ in range(want):             # BFS down the DAG, one level at a time
        nxt = []
        for x in levels[-1]:
            dn = int(dist_row[x]) - 1
            for e in range(int(row_ptr[x]), int(row_ptr[x + 1])):
                n = int(col[e])
                if int(dist_row[n]) == dn and n not in seen:
                    seen.add(n)
                    nxt.append(n)
        levels.append(nxt)
    cnt = {int(d): 1}
    cap = None if limit is None else int(limit) + 1
    for lv in reversed(levels[:-1]):
        for x in lv:
            dn, c = int(dist_row[x]) - 1, 0
            for e in range(int(row_ptr[x]), int(row_ptr[x + 1])):
                n = int(col[e])
                if int(dist_row[n]) == dn:
                    c += cnt.get(n, 0)
            cnt[x] = c if cap is None else min(c, cap)
    return cnt.get(int(s), 0)


def shortest_paths_lex(row_ptr, col, dist_row, s, d):
    """Every shortest s->d vertex sequence in lexicographic dpid order (the
    order _find_routes_bfs returns them, topology_db.py:95-122): walk the
    shortest-path DAG (dist_row = hops to d) taking successors ascending.
    Sets above ECMP_LIMIT routes raise MemoryError before any is built, as
    the batched device path (RouteEngine.ecmp) does."""
    INF = _native.DIST_INF
    dist_row = np.asarray(dist_row)
    if dist_row.dtype == np.int16:
        dist_row = dist_row.view(np.uint16)
    dist_row = np.where(dist_row < 0, INF, dist_row)
    if int(dist_row[s]) == INF:
        return []
    if count_shortest_paths(row_ptr, col, dist_row, s, d, ECMP_LIMIT) > ECMP_LIMIT:
        raise MemoryError("ECMP set too large to enumerate")
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
