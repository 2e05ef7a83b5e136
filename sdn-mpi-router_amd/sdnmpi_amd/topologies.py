"""Canonical synthetic fabrics (fat-tree, 3-D torus, dragonfly, Jellyfish).

The reference's default route (``_find_route_dfs``, reference
``sdnmpi/util/topology_db.py:59-84``) depends on dpid numbering, because every
neighbour scan is ``sorted(self.links[dpid].keys())`` (:76).  The numbering and
port conventions below are therefore part of the benchmark contract (SURVEY.md
section 8(d)); the golden fixtures under ``tests/golden/`` were produced by
feeding these exact fabrics to the reference ``TopologyDB``.

A :class:`Fabric` is a plain record of what Ryu would have reported:

* directed links in creation order (Ryu raises one ``EventLinkAdd`` per
  direction, reference ``sdnmpi/topology.py:192-194``), so parallel links
  collapse last-write-wins exactly as ``links[src][dst] = link`` does
  (``topology_db.py:30-35``);
* hosts (``EventHostAdd`` -> ``add_host``, ``topology_db.py:20-21``);
* switches (``EventSwitchEnter`` -> ``add_switch``, ``topology_db.py:23-24``).

``Fabric.populate(db)`` replays those events into any object with the
``TopologyDB`` mutator API; ``Fabric.csr()`` builds the same CSR the drop-in
exports from its dicts (``sdnmpi_amd.graph``), without materialising objects,
for benchmarks at 10^5..10^6 links.
"""

import hashlib

import numpy as np

from .objects import Host, Link, Port, Switch

__all__ = [
    "Fabric", "fat_tree", "torus3d", "dragonfly", "jellyfish", "mock_square",
    "mac_str", "HOST_MAC_BASE", "by_name",
]

HOST_MAC_BASE = 0x10000000


def mac_str(x):
    """48-bit int -> ``xx:xx:xx:xx:xx:xx`` (the inverse of the reference's
    ``_mac_to_int``, ``topology_db.py:124-125``)."""
    x = int(x)
    return ":".join("%02x" % ((x >> (8 * (5 - i))) & 0xFF) for i in range(6))


class _Builder(object):
    """Accumulates bidirectional links with per-switch port counters."""

    def __init__(self):
        self.next_port = {}
        self.src, self.sport, self.dst, self.dport = [], [], [], []

    def port(self, dpid):
        p = self.next_port.get(dpid, 1)
        self.next_port[dpid] = p + 1
        return p

    def link(self, u, pu, v, pv):
        # one EventLinkAdd per direction, u->v first
        self.src += [u, v]
        self.sport += [pu, pv]
        self.dst += [v, u]
        self.dport += [pv, pu]

    def auto_link(self, u, v):
        self.link(u, self.port(u), v, self.port(v))


class CSR(object):
    """Dense, dpid-sorted CSR of the switch graph.

    ``dpids[i]`` is the dpid of dense vertex ``i`` (ascending, so row order of
    ``col`` equals ``sorted(links[u].keys())``); ``col``/``port`` give the
    destination vertex and ``links[u][v].src.port_no`` of every directed link.
    Datapath ids are unsigned 64-bit in OpenFlow (ofp_switch_features.
    datapath_id), so ``dpids`` is uint64 and the whole range sorts as the
    reference's Python ints do.
    """

    __slots__ = ("dpids", "row_ptr", "col", "port")

    def __init__(self, dpids, row_ptr, col, port):
        self.dpids = np.ascontiguousarray(dpids, dtype=np.uint64)
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int32)
        self.col = np.ascontiguousarray(col, dtype=np.int32)
        self.port = np.ascontiguousarray(port, dtype=np.int32)

    @property
    def V(self):
        return int(self.dpids.shape[0])

    @property
    def E(self):
        return int(self.col.shape[0])

    def index_of(self, dpids):
        d = np.asarray(dpids, dtype=np.uint64)
        i = np.searchsorted(self.dpids, d)
        i = np.minimum(i, self.V - 1)
        ok = self.dpids[i] == d
        return np.where(ok, i, -1).astype(np.int32)

    def digest(self):
        h = hashlib.sha256()
        for a in (self.dpids, self.row_ptr, self.col, self.port):
            h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()

    def max_degree(self):
        if self.V == 0:
            return 0
        return int(np.diff(self.row_ptr).max())


def _dpid_array(x):
    """dpids (Python ints up to 2**64 - 1, or an integer array) as uint64."""
    if isinstance(x, np.ndarray):
        if x.dtype.kind == "i" and x.size and int(x.min()) < 0:
            raise ValueError("datapath ids are unsigned")
        return x.astype(np.uint64)
    return np.asarray(x, dtype=np.uint64)


def build_csr(link_src, link_dst, link_sport, extra_vertices=()):
    """CSR from directed links in creation order (last duplicate wins)."""
    src = _dpid_array(link_src)
    dst = _dpid_array(link_dst)
    sport = np.asarray(link_sport, dtype=np.int64)
    parts = [src, dst, _dpid_array(list(extra_vertices))]
    dpids = np.unique(np.concatenate(parts)) if sum(p.size for p in parts) else \
        np.zeros(0, np.uint64)
    V = dpids.shape[0]
    if src.size:
        si = np.searchsorted(dpids, src)
        di = np.searchsorted(dpids, dst)
        key = si * np.int64(V) + di
        # last occurrence of every (src, dst): unique over the reversed array
        rev = key[::-1]
        _, first_rev = np.unique(rev, return_index=True)
        keep = (key.size - 1 - first_rev)            # positions of last writes
        keep.sort()
        k2 = key[keep]
        order = np.argsort(k2, kind="stable")
        sel = keep[order]
        si, di, sp = si[sel], di[sel], sport[sel]
    else:
        si = di = sp = np.zeros(0, np.int64)
    counts = np.bincount(si, minlength=V) if V else np.zeros(0, np.int64)
    row_ptr = np.zeros(V + 1, np.int64)
    np.cumsum(counts, out=row_ptr[1:])
    if sp.size and (sp.max() > 0x7FFFFFFF or sp.min() < -0x80000000):
        raise ValueError("port numbers must fit in int32")
    return CSR(dpids, row_ptr, di, sp)


class Fabric(object):
    """A synthetic fabric: links (creation order), hosts, switches."""

    def __init__(self, name, link_src, link_sport, link_dst, link_dport,
                 host_mac, host_dpid, host_port, switches, params=None):
        self.name = name
        self.link_src = np.asarray(link_src, dtype=np.int64)
        self.link_sport = np.asarray(link_sport, dtype=np.int64)
        self.link_dst = np.asarray(link_dst, dtype=np.int64)
        self.link_dport = np.asarray(link_dport, dtype=np.int64)
        self.host_mac = np.asarray(host_mac, dtype=np.int64)      # 48-bit ints
        self.host_dpid = np.asarray(host_dpid, dtype=np.int64)
        self.host_port = np.asarray(host_port, dtype=np.int64)
        self.switches = np.asarray(sorted(switches), dtype=np.int64)
        self.params = dict(params or {})
        self._csr = None

    # -- sizes ---------------------------------------------------------
    @property
    def n_switches(self):
        return int(self.switches.shape[0])

    @property
    def n_hosts(self):
        return int(self.host_mac.shape[0])

    @property
    def n_links(self):
        return int(self.link_src.shape[0])

    def host_macs(self):
        return [mac_str(m) for m in self.host_mac]

    # -- exports -------------------------------------------------------
    def csr(self):
        if self._csr is None:
            extra = np.concatenate([self.host_dpid, self.switches])
            self._csr = build_csr(self.link_src, self.link_dst, self.link_sport,
                                  extra_vertices=extra)
        return self._csr

    def host_table(self):
        """(host_vertex int32[H], host_port int32[H]) in host order."""
        c = self.csr()
        return c.index_of(self.host_dpid), self.host_port.astype(np.int32)

    def populate(self, db, switch_cls=Switch, port_cls=Port, link_cls=Link,
                 host_cls=Host):
        """Replay the Ryu events into ``db`` (a reference-API TopologyDB)."""
        ports = {}
        for d in self.switches.tolist():
            db.add_switch(switch_cls(d))
        s, sp, t, tp = (self.link_src.tolist(), self.link_sport.tolist(),
                        self.link_dst.tolist(), self.link_dport.tolist())
        for i in range(len(s)):
            a = ports.get((s[i], sp[i]))
            if a is None:
                a = ports[(s[i], sp[i])] = port_cls(s[i], sp[i])
            b = ports.get((t[i], tp[i]))
            if b is None:
                b = ports[(t[i], tp[i])] = port_cls(t[i], tp[i])
            db.add_link(link_cls(a, b))
        for m, d, p in zip(self.host_mac.tolist(), self.host_dpid.tolist(),
                           self.host_port.tolist()):
            db.add_host(host_cls(mac_str(m), port_cls(d, p)))
        return db


# ----------------------------------------------------------------------
# generators
# ----------------------------------------------------------------------

def mock_square():
    """The reference test fixture (``tests/test_topologydb.py:14-61``):
    square 1-2-4-3-1, host ``02:00:00:00:00:0N`` on port 1 of switch N."""
    spec = [(1, 2, 2, 2), (1, 3, 3, 3), (2, 3, 4, 2), (3, 2, 4, 3)]
    b = _Builder()
    for u, pu, v, pv in spec:
        b.link(u, pu, v, pv)
    macs = [0x020000000000 + n for n in (1, 2, 3, 4)]
    return Fabric("mock", b.src, b.sport, b.dst, b.dport, macs, [1, 2, 3, 4],
                  [1, 1, 1, 1], [1, 2, 3, 4], {})


def fat_tree(k):
    """k-ary fat-tree (k even), h = k/2; SURVEY.md section 8(d):

    core c -> 1+c; agg(p,a) -> 1+h^2+p*h+a; edge(p,e) -> 1+h^2+k*h+p*h+e.
    edge ports 1..h = hosts, h+1+a = uplink to agg a; agg ports 1+e = edge e,
    h+1+j = core a*h+j; core port 1+p = pod p.  Host n = (p*h+e)*h+j has MAC
    0x10000000+n on edge(p,e) port 1+j.
    """
    if k < 2 or k % 2:
        raise ValueError("fat-tree arity k must be even and >= 2")
    h = k // 2

    def core(c):
        return 1 + c

    def agg(p, a):
        return 1 + h * h + p * h + a

    def edge(p, e):
        return 1 + h * h + k * h + p * h + e

    b = _Builder()
    for p in range(k):
        for e in range(h):
            for a in range(h):
                b.link(edge(p, e), h + 1 + a, agg(p, a), 1 + e)
    for p in range(k):
        for a in range(h):
            for j in range(h):
                b.link(agg(p, a), h + 1 + j, core(a * h + j), 1 + p)
    macs, hd, hp = [], [], []
    for p in range(k):
        for e in range(h):
            for j in range(h):
                macs.append(HOST_MAC_BASE + (p * h + e) * h + j)
                hd.append(edge(p, e))
                hp.append(1 + j)
    switches = list(range(1, 1 + h * h + 2 * k * h))
    return Fabric("fat_tree_k%d" % k, b.src, b.sport, b.dst, b.dport, macs, hd,
                  hp, switches, {"k": k})


def torus3d(X, Y, Z):
    """X*Y*Z torus: dpid 1+x+X*(y+Y*z); links created in (z,y,x) order with
    +x, +y, +z wraparound (no self-loops for a size-1 dimension); ports per
    switch in creation order; then one host per switch on the next port,
    host n = dpid-1, MAC 0x10000000+n."""
    def dp(x, y, z):
        return 1 + x + X * (y + Y * z)

    b = _Builder()
    for z in range(Z):
        for y in range(Y):
            for x in range(X):
                u = dp(x, y, z)
                for v in (dp((x + 1) % X, y, z), dp(x, (y + 1) % Y, z),
                          dp(x, y, (z + 1) % Z)):
                    if v != u:
                        b.auto_link(u, v)
    n = X * Y * Z
    switches = list(range(1, n + 1))
    hd = switches
    hp = [b.port(d) for d in hd]
    macs = [HOST_MAC_BASE + d - 1 for d in hd]
    return Fabric("torus_%dx%dx%d" % (X, Y, Z), b.src, b.sport, b.dst, b.dport,
                  macs, hd, hp, switches, {"X": X, "Y": Y, "Z": Z})


def dragonfly(a, h, p):
    """Balanced dragonfly: g = a*h+1 groups of a routers, router (G,i) ->
    dpid 1+G*a+i.  All intra-group full meshes first (i<j order), then global
    links for G<H: router (G,(H-1)//h) <-> (H, G//h).  Ports per router in
    creation order; then p hosts per router (router dpid order)."""
    g = a * h + 1

    def r(G, i):
        return 1 + G * a + i

    b = _Builder()
    for G in range(g):
        for i in range(a):
            for j in range(i + 1, a):
                b.auto_link(r(G, i), r(G, j))
    for G in range(g):
        for H in range(G + 1, g):
            b.auto_link(r(G, (H - 1) // h), r(H, G // h))
    switches = list(range(1, g * a + 1))
    macs, hd, hp = [], [], []
    n = 0
    for d in switches:
        for _ in range(p):
            macs.append(HOST_MAC_BASE + n)
            hd.append(d)
            hp.append(b.port(d))
            n += 1
    return Fabric("dragonfly_a%d_h%d_p%d" % (a, h, p), b.src, b.sport, b.dst,
                  b.dport, macs, hd, hp, switches, {"a": a, "h": h, "p": p})


def _random_regular_edges(n, r, seed):
    """Simple r-regular graph on n vertices: seeded configuration-model
    pairing; rejected stubs (self-loops, duplicates) are re-paired for a few
    rounds and the rest placed by degree-preserving edge switches.
    Deterministic for a given (n, r, seed) and numpy version."""
    if (n * r) % 2:
        raise ValueError("n*r must be even")
    if r >= n:
        raise ValueError("degree must be < n")
    rng = np.random.Generator(np.random.PCG64(seed))
    adj = [set() for _ in range(n)]
    edges = set()
    pool = np.repeat(np.arange(n, dtype=np.int64), r)
    for _round in range(64):
        if pool.size == 0:
            break
        rng.shuffle(pool)
        left = []
        for u, v in zip(pool[0::2].tolist(), pool[1::2].tolist()):
            if u == v or v in adj[u]:
                left += [u, v]
                continue
            adj[u].add(v)
            adj[v].add(u)
            edges.add((u, v) if u < v else (v, u))
        pool = np.asarray(left, dtype=np.int64)
    # repair the remainder: stub pair (u, v) with u == v or u~v.  Pick an
    # existing edge (x, y) with x, y new to u resp. v, replace by u-x, v-y.
    left = pool.tolist()
    edge_list = None
    while left:
        u, v = left.pop(), left.pop()
        if u != v and v not in adj[u]:
            adj[u].add(v)
            adj[v].add(u)
            edges.add((u, v) if u < v else (v, u))
            continue
        if edge_list is None:
            edge_list = sorted(edges)
        for _try in range(1 << 20):
            x, y = edge_list[int(rng.integers(len(edge_list)))]
            if (x, y) not in edges:
                continue
            if rng.integers(2):
                x, y = y, x
            if x in (u, v) or y in (u, v) or x in adj[u] or y in adj[v]:
                continue
            edges.discard((x, y) if x < y else (y, x))
            adj[x].discard(y)
            adj[y].discard(x)
            for a_, b_ in ((u, x), (v, y)):
                adj[a_].add(b_)
                adj[b_].add(a_)
                e = (a_, b_) if a_ < b_ else (b_, a_)
                edges.add(e)
                edge_list.append(e)
            break
        else:
            raise RuntimeError("jellyfish repair failed")
    return sorted(edges)


def jellyfish(n, r, seed=1):
    """Jellyfish: random r-regular switch graph (``_random_regular_edges``),
    switch i -> dpid 1+i; edges in sorted (u<v) order get the next free port
    on each end; one host per switch on port r+1, MAC 0x10000000+i."""
    b = _Builder()
    for u, v in _random_regular_edges(n, r, seed):
        b.auto_link(u + 1, v + 1)
    switches = list(range(1, n + 1))
    hp = [b.port(d) for d in switches]
    macs = [HOST_MAC_BASE + d - 1 for d in switches]
    return Fabric("jellyfish_n%d_r%d_s%d" % (n, r, seed), b.src, b.sport,
                  b.dst, b.dport, macs, switches, hp, switches,
                  {"n": n, "r": r, "seed": seed})


def by_name(name):
    """Parse names like ``fat_tree:48``, ``torus:32,32,32``,
    ``dragonfly:16,8,8``, ``jellyfish:100000,16,1`` or ``mock``."""
    kind, _, arg = name.partition(":")
    args = [int(x) for x in arg.split(",") if x]
    if kind == "mock":
        return mock_square()
    if kind == "fat_tree":
        return fat_tree(*args)
    if kind == "torus":
        return torus3d(*args)
    if kind == "dragonfly":
        return dragonfly(*args)
    if kind == "jellyfish":
        return jellyfish(*args)
    raise ValueError("unknown fabric %r" % name)
