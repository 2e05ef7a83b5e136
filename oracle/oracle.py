"""ORACLE -- TEST INFRASTRUCTURE ONLY.

Python side of the parity oracle for the route hot path of
keichi/sdn-mpi-router (``sdnmpi/util/topology_db.py``).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product package never does.

Two restatements live here:

* ctypes bindings of ``liboracle.so`` (``sdnroute_oracle.c``): whole per-source
  tables over a CSR, multi-threaded, used to check the HIP tables and as the
  strong CPU baseline;
* :func:`find_route_pair` / :func:`find_routes_all_shortest`: per-pair
  restatements of ``TopologyDB.find_route`` over the reference's own dict
  state (``links``/``hosts``/``switches``), used for the per-pair CPU
  baseline and for small end-to-end checks.

Pinning: ``tests/test_oracle_golden.py`` checks both against the fixtures
``tests/golden/make_golden.py`` produced by running the reference itself.
"""

import ctypes
import os
import subprocess
from collections import deque

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

OFPP_LOCAL = 0xFFFE   # ryu.ofproto.ofproto_v1_0.OFPP_LOCAL (topology_db.py:134)

_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")


def build():
    """Compile liboracle.so with the committed Makefile (gcc)."""
    subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        i32, c_int = ctypes.c_int32, ctypes.c_int
        L.oracle_dfs_tables.argtypes = [i32, _i32p, _i32p, _i32p, _i32p, i32,
                                        _i32p, _i32p, ctypes.c_void_p, c_int]
        L.oracle_bfs_tables.argtypes = [i32, _i32p, _i32p, _i32p, _i32p, i32,
                                        _i32p, _i32p, _i32p, c_int]
        L.oracle_dest_tables_batch.argtypes = [i32, _i32p, _i32p, _i32p, _i32p,
                                               _i32p, _i32p, i32, _u16p, _i32p,
                                               _i32p, c_int]
        L.oracle_apsp.argtypes = [i32, _i32p, _i32p, _u16p]
        for f in (L.oracle_dfs_tables, L.oracle_bfs_tables,
                  L.oracle_dest_tables_batch, L.oracle_apsp):
            f.restype = None
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _threads(n):
    return int(n) if n else (os.cpu_count() or 1)


def dfs_tables(csr, srcs, with_hops=True, nthreads=None):
    """Reference-exact default-route trees: (parent, port, hops) [S, V]."""
    srcs = _i32(srcs)
    S, V = srcs.shape[0], csr.V
    parent = np.empty((S, V), np.int32)
    port = np.empty((S, V), np.int32)
    hops = np.empty((S, V), np.int32) if with_hops else None
    lib().oracle_dfs_tables(V, _i32(csr.row_ptr), _i32(csr.col),
                            _i32(csr.port), srcs, S, parent, port,
                            hops.ctypes.data if hops is not None else None,
                            _threads(nthreads))
    return parent, port, hops


def bfs_tables(csr, srcs, nthreads=None):
    """Per-source lexicographically-smallest shortest-path trees."""
    srcs = _i32(srcs)
    S, V = srcs.shape[0], csr.V
    parent = np.empty((S, V), np.int32)
    port = np.empty((S, V), np.int32)
    hops = np.empty((S, V), np.int32)
    lib().oracle_bfs_tables(V, _i32(csr.row_ptr), _i32(csr.col),
                            _i32(csr.port), srcs, S, parent, port, hops,
                            _threads(nthreads))
    return parent, port, hops


def reverse_csr(csr):
    """In-neighbour CSR (rrow, rcol): rcol lists x for every link x -> y."""
    V = csr.V
    src = np.repeat(np.arange(V, dtype=np.int64), np.diff(csr.row_ptr))
    order = np.lexsort((src, csr.col))
    rcol = src[order].astype(np.int32)
    counts = np.bincount(csr.col, minlength=V)
    rrow = np.zeros(V + 1, np.int64)
    np.cumsum(counts, out=rrow[1:])
    return rrow.astype(np.int32), rcol


def dest_tables(csr, dsts, nthreads=None):
    """Shortest-mode per-destination tables (dist u16, nh, nh_port) [D, V]."""
    dsts = _i32(dsts)
    D, V = dsts.shape[0], csr.V
    rrow, rcol = reverse_csr(csr)
    dist = np.empty((D, V), np.uint16)
    nh = np.empty((D, V), np.int32)
    nh_port = np.empty((D, V), np.int32)
    lib().oracle_dest_tables_batch(V, _i32(csr.row_ptr), _i32(csr.col),
                                   _i32(csr.port), rrow, rcol, dsts, D, dist,
                                   nh, nh_port, _threads(nthreads))
    return dist, nh, nh_port


def apsp(csr):
    V = csr.V
    dist = np.empty((V, V), np.uint16)
    lib().oracle_apsp(V, _i32(csr.row_ptr), _i32(csr.col), dist)
    return dist


# ---------------------------------------------------------------------------
# Per-pair restatement of TopologyDB.find_route over the reference dict state.
# ---------------------------------------------------------------------------

def _mac_int(mac):
    # topology_db.py:124-125
    return int(mac.replace(":", ""), 16)


def _endpoints(db, src_mac, dst_mac):
    """topology_db.py:143-166 -> (src_dpid, dst_dpid, dst_is_local) or None."""
    s_local = _mac_int(src_mac) in db.switches
    d_local = _mac_int(dst_mac) in db.switches
    if not s_local and src_mac not in db.hosts:
        return None
    if not d_local and dst_mac not in db.hosts:
        return None
    s = _mac_int(src_mac) if s_local else db.hosts[src_mac].port.dpid
    d = _mac_int(dst_mac) if d_local else db.hosts[dst_mac].port.dpid
    return s, d, d_local


def _to_fdb(db, seq, d, d_local, dst_mac):
    # topology_db.py:127-138
    out = [(a, db.links[a][b].src.port_no) for a, b in zip(seq, seq[1:])]
    out.append((d, OFPP_LOCAL if d_local else db.hosts[dst_mac].port.port_no))
    return out


def _dfs_path(links, s, d):
    """Stack search of topology_db.py:59-84 with predecessor links instead of
    path copies; stops when d is popped."""
    pred = {s: None}
    stack = [s]
    while stack:
        u = stack.pop()
        if u == d:
            seq = []
            while u is not None:
                seq.append(u)
                u = pred[u]
            return seq[::-1]
        nbrs = links.get(u)
        if not nbrs:
            continue
        for v in sorted(nbrs):
            if v not in pred:
                pred[v] = u
                stack.append(v)
    return []


def _dfs_path_copying(links, s, d):
    """The stack search of topology_db.py:59-84 in the reference's own shape:
    a visited set (:63), a stack of whole paths (:65), and a fresh copy of the
    popped path for every pushed neighbour (:79-82) -- the per-pair cost the
    controller pays per packet-in.  Same result as _dfs_path."""
    visited = set([s])
    paths = [[s]]
    while paths:
        current = paths.pop()
        u = current[-1]
        if u == d:
            return current
        if u not in links:
            continue
        for v in sorted(links[u].keys()):
            if v not in visited:
                nxt = list(current)
                nxt.append(v)
                visited.add(v)
                paths.append(nxt)
    return []


def find_route_pair(db, src_mac, dst_mac, copying=False):
    """find_route(src_mac, dst_mac) (multiple=False), reference semantics.
    ``copying``: search with the reference's path copies (_dfs_path_copying,
    the reference's cost) instead of predecessor links (_dfs_path)."""
    ep = _endpoints(db, src_mac, dst_mac)
    if ep is None:
        return []
    s, d, d_local = ep
    seq = (_dfs_path_copying if copying else _dfs_path)(db.links, s, d)
    if not seq:
        return []
    return _to_fdb(db, seq, d, d_local, dst_mac)


def _shortest_paths_lex(links, s, d):
    """All shortest s->d dpid sequences in lexicographic order (= the order
    _find_routes_bfs returns them, topology_db.py:86-122), by BFS distances
    to d and a lexicographic walk of the shortest-path DAG."""
    # BFS from d over reversed links
    rev = {}
    for u, nb in links.items():
        for v in nb:
            rev.setdefault(v, []).append(u)
    dist = {d: 0}
    q = deque([d])
    while q:
        y = q.popleft()
        for x in rev.get(y, ()):
            if x not in dist:
                dist[x] = dist[y] + 1
                q.append(x)
    if s not in dist:
        return []
    out = []

    def walk(x, acc):
        if x == d:
            out.append(list(acc))
            return
        for n in sorted(links.get(x, ())):
            if dist.get(n, -1) == dist[x] - 1:
                acc.append(n)
                walk(n, acc)
                acc.pop()
    walk(s, [s])
    return out


def ecmp_counts(csr, dist_row):
    """Number of routes find_route(src, dst, multiple=True) returns from every
    vertex toward one destination (topology_db.py:86-122 enumerates every
    shortest simple path; their number is the count of shortest-path DAG
    walks): a level DP over dist_row (hops x -> dst, 0xFFFF unreachable, from
    dest_tables), in Python integers, saturated at 2**64-1 as the device's
    u64 counts are.  Pinned by tests/test_oracle_golden.py against the sizes
    of the reference's own multiple=True outputs."""
    V = csr.V
    order = sorted((int(dist_row[x]), x) for x in range(V) if dist_row[x] != 0xFFFF)
    cnt = [0] * V
    for dx, x in order:
        if dx == 0:
            cnt[x] = 1
            continue
        c = 0
        for e in range(int(csr.row_ptr[x]), int(csr.row_ptr[x + 1])):
            n = int(csr.col[e])
            if dist_row[n] != 0xFFFF and int(dist_row[n]) + 1 == dx:
                c += cnt[n]
        cnt[x] = c
    return np.array([min(c, 2**64 - 1) for c in cnt], dtype=np.uint64)


def find_routes_all_shortest(db, src_mac, dst_mac):
    """find_route(src_mac, dst_mac, multiple=True), reference semantics."""
    ep = _endpoints(db, src_mac, dst_mac)
    if ep is None:
        return []
    s, d, d_local = ep
    seqs = _shortest_paths_lex(db.links, s, d)
    return [_to_fdb(db, q, d, d_local, dst_mac) for q in seqs]


# ---------------------------------------------------------------------------
# Table -> fdb expansion (shared by tests)
# ---------------------------------------------------------------------------

def tree_path(parent_row, s, d):
    """Dense vertex sequence s..d in a per-source tree row, [] if unreached."""
    if parent_row[d] < 0:
        return []
    seq = [int(d)]
    x = int(d)
    while x != s:
        x = int(parent_row[x])
        seq.append(x)
        if len(seq) > parent_row.shape[0] + 1:
            raise RuntimeError("cycle in parent table")
    return seq[::-1]


def tree_fdb(csr, parent_row, port_row, s, d, last_port):
    seq = tree_path(parent_row, s, d)
    if not seq:
        return []
    out = [(int(csr.dpids[a]), int(port_row[b])) for a, b in zip(seq, seq[1:])]
    out.append((int(csr.dpids[d]), int(last_port)))
    return out
