"""Exact incremental maintenance of the route tables on link events.

SURVEY.md 8(f) 2: a link that Ryu reports added or removed
(``EventLinkAdd`` / ``EventLinkDelete`` -> ``TopologyDB.add_link`` /
``delete_link``, reference ``sdnmpi/topology.py:192-198``,
``sdnmpi/util/topology_db.py:30-42``) changes only the table rows whose result
depends on that link.  The tests below decide that per row from the tables
already computed, so only those rows go back to the GPU.  Every criterion is
exact for a single event (a row is flagged iff it changes) and sound for a
batch of events (the union may flag a row that ends up unchanged).

Default route (``_find_route_dfs``, topology_db.py:59-84), per source s with
tree ``parent_s`` (the tree of first pushes):

* removed link (u, v), or a new port on it: the search looks at (u, v) only
  when it pops u, and pushes v only if v is unvisited then -- which is exactly
  ``parent_s[v] == u``.  Any other row is unchanged.
* added link (u, v): it matters iff u is reached and v is still unvisited
  when u is popped: v unreached, or v pushed (by ``parent_s[v]``) in a pop
  that comes after u's.  Pops follow the tree's preorder with children taken
  in DESCENDING id order (LIFO over ascending pushes), so "after" is decided
  from the two tree paths: an ancestor pops first; otherwise, below their
  lowest common ancestor, the branch of the larger child pops first.

Shortest routes (``_find_routes_bfs``, :86-122), per destination d with hop
distances ``dist`` and lexicographic next hops ``nh``:

* removed link (x, n), or a new port on it: the row changes iff
  ``nh[x] == n``.  Otherwise either the link is not tight (on no shortest
  path) or x keeps its next hop ``nh[x]``, one hop closer, so ``dist[x]`` and
  with it every distance and next hop stay as they are.
* added link (x, n): with ``dist[n] + 1 >= dist[x]`` for every added link the
  old distances still satisfy every edge constraint, so they are unchanged;
  ``nh[x]`` changes iff ``dist[n] + 1 == dist[x]`` and ``n < nh[x]``.
"""

import numpy as np

__all__ = ["EdgeDiff", "edge_diff", "dfs_rows_affected", "sp_rows_affected"]

_INF = 0xFFFF


class EdgeDiff(object):
    """Directed-link differences between two CSRs over the same vertex set
    (dense ids): removed, added and re-ported links as (u, v) id arrays."""

    __slots__ = ("removed", "added", "ported")

    def __init__(self, removed, added, ported):
        self.removed = removed
        self.added = added
        self.ported = ported

    def empty(self):
        return not (self.removed[0].size or self.added[0].size or self.ported[0].size)


def _edge_keys(csr):
    V = np.int64(csr.V)
    src = np.repeat(np.arange(csr.V, dtype=np.int64), np.diff(csr.row_ptr.astype(np.int64)))
    return src * V + csr.col.astype(np.int64)


def edge_diff(old, new):
    """EdgeDiff of two CSRs, or None when the vertex sets differ (dense ids
    would not line up; the caller recomputes everything)."""
    if old.V != new.V or not np.array_equal(old.dpids, new.dpids):
        return None
    V = np.int64(old.V)
    ko, kn = _edge_keys(old), _edge_keys(new)       # both ascending (rows sorted)
    common, io, inn = np.intersect1d(ko, kn, assume_unique=True, return_indices=True)
    rem = np.setdiff1d(ko, kn, assume_unique=True)
    add = np.setdiff1d(kn, ko, assume_unique=True)
    prt = common[old.port[io] != new.port[inn]]

    def split(k):
        return (k // V).astype(np.int64), (k % V).astype(np.int64)
    return EdgeDiff(split(rem), split(add), split(prt))


class _NumpyNS(object):
    """Array ops of the row tests on host (numpy) tables."""

    @staticmethod
    def zeros_bool(n):
        return np.zeros(n, bool)

    @staticmethod
    def i64(a):
        return np.asarray(a).astype(np.int64)

    @staticmethod
    def full_i64(n, v):
        return np.full(n, v, np.int64)

    @staticmethod
    def nonzero(m):
        return np.nonzero(m)[0]

    @staticmethod
    def host(a):
        return a


class _TorchNS(object):
    """The same ops on device (torch) tables: the tests run where the tables
    live, only the per-row verdict comes back to the host."""

    def __init__(self, device):
        import torch
        self.t = torch
        self.device = device

    def zeros_bool(self, n):
        return self.t.zeros(n, dtype=self.t.bool, device=self.device)

    def i64(self, a):
        if isinstance(a, np.ndarray):
            return self.t.as_tensor(a.astype(np.int64), device=self.device)
        return a.to(self.t.int64, copy=True)

    def full_i64(self, n, v):
        return self.t.full((n,), int(v), dtype=self.t.int64, device=self.device)

    def nonzero(self, m):
        return self.t.nonzero(m).flatten()

    @staticmethod
    def host(a):
        return a.cpu().numpy()


def _ns(a):
    a = getattr(a, "arr", a)           # engine.Wide: a decoding view of a compact table
    return _NumpyNS() if isinstance(a, np.ndarray) else _TorchNS(a.device)


def _u16(xp, a):
    """u16 distances as int64 (device tables hold them in int16)."""
    d = xp.i64(a)
    return d & 0xFFFF if str(a.dtype).endswith("int16") and "u" not in str(a.dtype) else d


def _popped_before(parent, hops, rows, a, b):
    """bool[n]: in row ``rows[i]``'s tree, vertex a[i] is popped before b[i]
    (a != b, both reached) -- preorder, children in descending id order."""
    xp = _ns(parent)
    n = rows.shape[0]
    res = xp.zeros_bool(n)
    if n == 0:
        return res
    x, y = xp.i64(a), xp.i64(b)          # copies: climbed in place below
    hx, hy = xp.i64(hops[rows, x]), xp.i64(hops[rows, y])
    a_deeper, b_deeper = hx > hy, hy > hx
    # lift the deeper vertex to the other's depth
    while True:
        sel = hx > hy
        if not bool(sel.any()):
            break
        x[sel] = xp.i64(parent[rows[sel], x[sel]])
        hx[sel] -= 1
    while True:
        sel = hy > hx
        if not bool(sel.any()):
            break
        y[sel] = xp.i64(parent[rows[sel], y[sel]])
        hy[sel] -= 1
    done = x == y                    # one is the other's ancestor
    res[done & b_deeper] = True      # a is b's ancestor: a pops first
    res[done & a_deeper] = False     # b is a's ancestor
    # climb together until the parents meet: x, y are then the LCA's children
    while not bool(done.all()):
        act = ~done
        px = xp.i64(parent[rows[act], x[act]])
        py = xp.i64(parent[rows[act], y[act]])
        meet = px == py
        idx = xp.nonzero(act)
        hit = idx[meet]
        res[hit] = x[hit] > y[hit]   # larger child's branch pops first
        done[hit] = True
        go = idx[~meet]
        x[go] = px[~meet]
        y[go] = py[~meet]
    return res


def dfs_rows_affected(parent, hops, srcs, diff):
    """bool[S] (numpy): rows of the per-source default-route tables (parent,
    hops [S, V], sources ``srcs``; numpy or device tensors) that the link
    changes in ``diff`` alter."""
    xp = _ns(parent)
    S = parent.shape[0]
    out = xp.zeros_bool(S)
    # removed or re-ported link (u, v): only when it is the tree edge into v
    for u, v in (diff.removed, diff.ported):
        for uu, vv in zip(u.tolist(), v.tolist()):
            out |= parent[:, vv] == uu
    # added link (u, v)
    rows_all = xp.i64(np.arange(S, dtype=np.int64))
    srcs = xp.i64(np.asarray(srcs, np.int64))
    for uu, vv in zip(diff.added[0].tolist(), diff.added[1].tolist()):
        if uu == vv:
            continue                                  # u is visited when popped
        reach_u = parent[:, uu] >= 0
        pv = parent[:, vv]
        cand = reach_u & (srcs != vv) & ~out
        unreached_v = cand & (pv < 0)
        out |= unreached_v
        chk = cand & (pv >= 0)
        if bool(chk.any()):
            r = rows_all[chk]
            before = _popped_before(parent, hops, r, xp.i64(pv[chk]),
                                    xp.full_i64(r.shape[0], uu))
            out[r[~before]] = True
    return xp.host(out)


def sp_rows_affected(dist, nh, diff):
    """bool[D] (numpy): rows of the per-destination shortest tables (dist
    u16 with 0xFFFF = unreachable, nh [D, V]; numpy or device tensors) that
    the link changes alter."""
    xp = _ns(dist)
    D = dist.shape[0]
    out = xp.zeros_bool(D)
    for u, v in (diff.removed, diff.ported):
        for xx, nn in zip(u.tolist(), v.tolist()):
            out |= nh[:, xx] == nn
    for xx, nn in zip(diff.added[0].tolist(), diff.added[1].tolist()):
        dx, dn = _u16(xp, dist[:, xx]), _u16(xp, dist[:, nn])
        ok = dn != _INF
        nhx = xp.i64(nh[:, xx])
        out |= ok & ((dn + 1 < dx) | ((dn + 1 == dx) & ((nhx < 0) | (nn < nhx))))
    return xp.host(out)
