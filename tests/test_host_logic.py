"""Host-side logic on CPU: canonical generators (sizes and the survey's
self-check histograms), dict -> CSR export == the generators' direct CSR,
CSR conventions (ascending dpid order, sorted rows, last-write-wins parallel
links), and fdb expansion helpers."""
import collections
import os

import numpy as np
import pytest

from oracle import oracle as O
from sdnmpi_amd import topologies as T
from sdnmpi_amd.engine import (ECMP_LIMIT, count_shortest_paths, expand_tree_paths,
                               shortest_paths_lex, tree_path)
from sdnmpi_amd.graph import export_graph
from sdnmpi_amd.util.topology_db import TopologyDB


@pytest.mark.parametrize("fab,V,E,H", [
    (lambda: T.fat_tree(8), 80, 512, 128),
    (lambda: T.fat_tree(48), 2880, 110592, 27648),
    (lambda: T.dragonfly(16, 8, 8), 2064, 47472, 16512),
    (lambda: T.torus3d(32, 32, 32), 32768, 196608, 32768),
])
def test_canonical_sizes(fab, V, E, H):
    f = fab()
    c = f.csr()
    assert (c.V, c.E, f.n_hosts) == (V, E, H)


def test_jellyfish_is_regular_and_simple():
    f = T.jellyfish(2000, 16, seed=1)
    c = f.csr()
    deg = np.diff(c.row_ptr)
    assert (deg == 16).all()
    for u in range(0, c.V, 97):
        row = c.col[c.row_ptr[u]:c.row_ptr[u + 1]]
        assert u not in row and len(set(row.tolist())) == 16


def _dfs_hop_hist(f):
    c = f.csr()
    hv, _ = f.host_table()
    srcs = np.unique(hv)
    _, _, hops = O.dfs_tables(c, srcs)
    row = {int(s): i for i, s in enumerate(srcs)}
    h = collections.Counter()
    for a in hv:
        for b in hv:
            h[int(hops[row[int(a)], int(b)])] += 1
    return dict(h)


def test_fat_tree_self_check_histograms():
    """k=8 {0:512, 2:1536, 4:2048, 8:2048, 12:2048, 16:8192},
    k=4 {0:32, 2:32, 4:64, 8:128}; shortest switch pairs (edge->edge) at k=8
    {0:32, 2:96, 4:896}."""
    assert _dfs_hop_hist(T.fat_tree(8)) == {0: 512, 2: 1536, 4: 2048, 8: 2048, 12: 2048, 16: 8192}
    assert _dfs_hop_hist(T.fat_tree(4)) == {0: 32, 2: 32, 4: 64, 8: 128}
    f = T.fat_tree(8)
    c = f.csr()
    edges = np.unique(f.host_table()[0])
    dist, _, _ = O.dest_tables(c, edges)
    h = collections.Counter(int(x) for x in dist[:, edges].ravel())
    assert dict(h) == {0: 32, 2: 96, 4: 896}


@pytest.mark.parametrize("fab", [lambda: T.fat_tree(8), lambda: T.torus3d(5, 3, 2),
                                 lambda: T.dragonfly(4, 2, 2), lambda: T.jellyfish(60, 5, 3),
                                 T.mock_square])
def test_dict_export_equals_direct_csr(fab):
    f = fab()
    db = f.populate(TopologyDB())
    ex = export_graph(db.links, db.switches, db.hosts)
    assert ex.csr.digest() == f.csr().digest()


def test_csr_conventions_parallel_links_last_write_wins():
    # torus 5x3x2: the size-2 dimension creates two links per ordered pair
    f = T.torus3d(5, 3, 2)
    c = f.csr()
    for u in range(c.V):
        row = c.col[c.row_ptr[u]:c.row_ptr[u + 1]]
        assert (np.diff(row) > 0).all()
    assert (np.diff(c.dpids) > 0).all()
    # the later-created link's port survives, as links[src][dst] = link does
    last = {}
    for s, sp, d in zip(f.link_src, f.link_sport, f.link_dst):
        last[(int(s), int(d))] = int(sp)
    for u in range(c.V):
        for e in range(c.row_ptr[u], c.row_ptr[u + 1]):
            assert c.port[e] == last[(int(c.dpids[u]), int(c.dpids[c.col[e]]))]


def test_tree_expansion_helpers():
    f = T.fat_tree(8)
    c = f.csr()
    srcs = np.arange(c.V, dtype=np.int32)
    parent, port, hops = O.dfs_tables(c, srcs)
    rng = np.random.default_rng(0)
    rows = rng.integers(0, c.V, 300)
    dsts = rng.integers(0, c.V, 300)
    off, verts, ports = expand_tree_paths(parent, port, rows, dsts)
    for i, (r, d) in enumerate(zip(rows, dsts)):
        seq = tree_path(parent[r], int(r), int(d))
        assert verts[off[i]:off[i + 1]].tolist() == seq
        assert len(seq) == hops[r, d] + 1
        for k in range(len(seq) - 1):
            assert ports[off[i] + k] == port[r, seq[k + 1]]


def test_shortest_paths_lex_matches_reference_order():
    f = T.fat_tree(4)
    c = f.csr()
    dsts = np.arange(c.V, dtype=np.int32)
    dist, _, _ = O.dest_tables(c, dsts)
    # every enumerated path is shortest, simple, in lexicographic order
    for s in range(0, c.V, 3):
        for d in range(0, c.V, 5):
            seqs = shortest_paths_lex(c.row_ptr, c.col, dist[d], s, d)
            assert seqs == sorted(seqs)
            for q in seqs:
                assert len(q) - 1 == dist[d, s] and len(set(q)) == len(q)


def test_shortest_paths_count_and_limit():
    # the host count equals the enumeration's length (fat-tree, small torus)
    for fab in (T.fat_tree(4), T.torus3d(4, 4, 4)):
        c = fab.csr()
        dist, _, _ = O.dest_tables(c, np.arange(c.V, dtype=np.int32))
        for s in range(0, c.V, 7):
            for d in range(0, c.V, 5):
                if dist[d, s] == 0xFFFF:
                    continue
                n = len(shortest_paths_lex(c.row_ptr, c.col, dist[d], s, d))
                assert count_shortest_paths(c.row_ptr, c.col, dist[d], s, d) == n
    # torus 32^3 antipodal pair: 48!/(16!)^3 ~ 1e21 routes -> MemoryError
    # before enumerating, like the batched device path (RouteEngine.ecmp)
    c = T.torus3d(32, 32, 32).csr()
    dist, _, _ = O.dest_tables(c, np.array([0], np.int32))
    far = 16 * 1024 + 16 * 32 + 16
    assert count_shortest_paths(c.row_ptr, c.col, dist[0], far, 0, ECMP_LIMIT) > ECMP_LIMIT
    with pytest.raises(MemoryError):
        shortest_paths_lex(c.row_ptr, c.col, dist[0], far, 0)


def test_unpack_tree_layout():
    from sdnmpi_amd._native import unpack_tree
    t = np.array([[0x00030002, 0xFFFF0005, 0xFFFFFFFF, 0xFFFE0000]], np.uint32)
    p, q = unpack_tree(t)
    assert p.tolist() == [[2, 5, -1, 0]]
    assert q.tolist() == [[3, -1, -1, 0xFFFE]]


def test_pool_failed_fill_leaves_slots_blank():
    """A fill that writes part of its rows in place and then raises gives
    the slots back blank (free slots must stay all-unreached,
    which drop() and the incremental row tests rely on)."""
    from sdnmpi_amd.engine import _Pool
    V = 8
    pool = _Pool(budget=1 << 20, row_bytes=8 * V, blanks=(-1, -1))
    like = (np.empty((0, V), np.int32), np.empty((0, V), np.int32))

    def bad_fill(out):
        out[0][...] = 7                      # partial in-place write, then a failure
        raise RuntimeError("kernel failed")

    with pytest.raises(RuntimeError):
        pool.add([0, 1, 2], fill=bad_fill, like=like)
    assert len(pool) == 0
    assert all((a == -1).all() for a in pool.arrays)
    pool.add([3, 4], fill=lambda out: [o.fill(5) for o in out], like=like)
    rows = sorted(pool.row.values())
    assert all((a[rows] == 5).all() for a in pool.arrays)
    others = [i for i in range(pool.size) if i not in rows]
    assert all((a[others] == -1).all() for a in pool.arrays)


def test_profile_coalescing_figures():
    """tools/summarize_profile.py's read-coalescing figures:
    tag lookups per VMEM instruction (4 = one line per quarter-wave, the
    floor), L2 requests per load, L1 hit rate -- from per-dispatch counter
    means, here the round-6 headline kernel's own (profiles/r06_dfs48p)."""
    import importlib.util
    import json
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "summarize_profile", os.path.join(root, "tools", "summarize_profile.py"))
    sp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sp)
    c = {"TCP_TOTAL_CACHE_ACCESSES_sum": 400.0, "SQ_INSTS_VMEM_RD": 90.0,
         "SQ_INSTS_VMEM_WR": 10.0, "TCP_TCC_READ_REQ_sum": 45.0, "TCP_TOTAL_READ_sum": 900.0}
    co = sp.coalescing(c)
    assert co["tag_lookups_per_vmem"] == 4.0
    assert co["l2_req_per_vmem_rd"] == 0.5
    assert abs(co["l1_read_hit"] - 0.95) < 1e-12
    assert sp.coalescing({}) == {}
    pmc = json.load(open(os.path.join(root, "profiles", "r06_dfs48p_pmc.json")))
    k = [n for n in pmc if "dfs_async_kernel" in n][0]
    got = sp.coalescing(pmc[k]["counters"])
    assert 4.0 <= got["tag_lookups_per_vmem"] < 4.5        # coalesced: ~one line per quarter-wave
    assert got["l1_read_hit"] > 0.9
