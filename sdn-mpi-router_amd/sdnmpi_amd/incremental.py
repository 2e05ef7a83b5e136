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


def _popped_before(parent, hops, rows, a, b):
    """bool[n]: in row ``rows[i]``'s tree, vertex a[i] is popped before b[i]
    (a != b, both reached) -- preorder, children in descending id order."""
    n = rows.shape[0]
    res = np.zeros(n, bool)
    if n == 0:
        return res
    x, y = a.astype(np.int64).copy(), b.astype(np.int64).copy()
    hx, hy = hops[rows, x].astype(np.int64), hops[rows, y].astype(np.int64)
    a_deeper, b_deeper = hx > hy, hy > hx
    # lift the deeper vertex to the other's depth
    while True:
        sel = hx > hy
        if not sel.any():
            break
        x[sel] = parent[rows[sel], x[sel]]
        hx[sel] -= 1
    while True:
        sel = hy > hx
        if not sel.any():
            break
        y[sel] = parent[rows[sel], y[sel]]
        hy[sel] -= 1
    done = x == y                    # one is the other's ancestor
    res[done & b_deeper] = True      # a is b's ancestor: a pops first
    res[done & a_deeper] = False     # b is a's ancestor
    # climb together until the parents meet: x, y are then the LCA's children
    while not done.all():
        act = ~done
        px = parent[rows[act], x[act]]
        py = parent[rows[act], y[act]]
        meet = px == py
        idx = np.nonzero(act)[0]
        hit = idx[meet]
        res[hit] = x[hit] > y[hit]   # larger child's branch pops first
        done[hit] = True
        go = idx[~meet]
        x[go] = px[~meet]
        y[go] = py[~meet]
    return res


def dfs_rows_affected(parent, hops, srcs, diff):
    """bool[S]: rows of the per-source default-route tables (parent, hops
    [S, V], sources ``srcs``) that the link changes in ``diff`` alter."""
    S = parent.shape[0]
    out = np.zeros(S, bool)
    # removed or re-ported link (u, v): only when it is the tree edge into v
    for u, v in (diff.removed, diff.ported):
        for uu, vv in zip(u.tolist(), v.tolist()):
            out |= parent[:, vv] == uu
    # added link (u, v)
    rows_all = np.arange(S, dtype=np.int64)
    srcs = np.asarray(srcs, np.int64)
    for uu, vv in zip(diff.added[0].tolist(), diff.added[1].tolist()):
        if uu == vv:
            continue                                  # u is visited when popped
        reach_u = parent[:, uu] >= 0
        pv = parent[:, vv]
        cand = reach_u & (srcs != vv) & ~out
        unreached_v = cand & (pv < 0)
        out |= unreached_v
        chk = cand & (pv >= 0)
        if chk.any():
            r = rows_all[chk]
            before = _popped_before(parent, hops, r, pv[chk].astype(np.int64),
                                    np.full(r.shape[0], uu, np.int64))
            out[r[~before]] = True
    return out


def sp_rows_affected(dist, nh, diff):
    """bool[D]: rows of the per-destination shortest tables (dist u16 with
    0xFFFF = unreachable, nh [D, V]) that the link changes alter."""
    D = dist.shape[0]
    out = np.zeros(D, bool)
    d32 = dist.astype(np.int64)
    for u, v in (diff.removed, diff.ported):
        for xx, nn in zip(u.tolist(), v.tolist()):
            out |= nh[:, xx] == nn
    for xx, nn in zip(diff.added[0].tolist(), diff.added[1].tolist()):
        dx, dn = d32[:, xx], d32[:, nn]
        ok = dn != _INF
        nhx = nh[:, xx].astype(np.int64)
        out |= ok & ((dn + 1 < dx) | ((dn + 1 == dx) & ((nhx < 0) | (nn < nhx))))
    return out
