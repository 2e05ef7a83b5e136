"""The drop-in TopologyDB, exercised the way the reference uses it.

* ``TestReferenceSuite`` re-states the reference's own unit tests
  (reference ``tests/test_topologydb.py:13-109``: 4-switch square fixture,
  dicts assigned directly, ``del`` of a links entry) against our class.
* scenario replays (tests/golden/scenarios.json, produced by the reference):
  mutations through the methods AND directly on the dicts, deleted switches
  whose links stay, parallel links, switch-local MACs (OFPP_LOCAL), unknown
  and malformed MACs -- every query's result must equal the reference's.
* every host pair of the small golden fabrics, both route modes.

GPU tests: routes come from the HIP tables.  The CPU-only tests at the end
check the host-side logic (dict tracking / invalidation) with a fake engine.
"""
import numpy as np
import pytest

import golden_util as G
from sdnmpi_amd.objects import Host, Link, Port, Switch
from sdnmpi_amd.util.topology_db import OFPP_LOCAL, TopologyDB

MAC1 = "02:00:00:00:00:01"
MAC2 = "02:00:00:00:00:02"
MAC3 = "02:00:00:00:00:03"
MAC4 = "02:00:00:00:00:04"


def square_db():
    """Reference fixture: tests/test_topologydb.py:14-61."""
    db = TopologyDB()
    p = {(d, n): Port(d, n) for d in (1, 2, 3, 4) for n in (1, 2, 3)}
    db.links = {
        1: {2: Link(p[1, 2], p[2, 2]), 3: Link(p[1, 3], p[3, 3])},
        2: {1: Link(p[2, 2], p[1, 2]), 4: Link(p[2, 3], p[4, 2])},
        3: {1: Link(p[3, 3], p[1, 3]), 4: Link(p[3, 2], p[4, 3])},
        4: {2: Link(p[4, 2], p[2, 3]), 3: Link(p[4, 3], p[3, 2])},
    }
    db.hosts = {MAC1: Host(MAC1, p[1, 1]), MAC2: Host(MAC2, p[2, 1]),
                MAC3: Host(MAC3, p[3, 1]), MAC4: Host(MAC4, p[4, 1])}
    db.switches = {d: Switch(d) for d in (1, 2, 3, 4)}
    return db


@pytest.mark.gpu
class TestReferenceSuite(object):
    def test_find_route_same_switch(self):
        db = square_db()
        for mac, d in ((MAC1, 1), (MAC2, 2), (MAC3, 3), (MAC4, 4)):
            assert db.find_route(mac, mac) == [(d, 1)]

    def test_find_route_unreachable(self):
        db = square_db()
        del db.links[1]
        assert db.find_route(MAC1, MAC2) == []
        assert db.find_route(MAC1, MAC3) == []
        assert db.find_route(MAC1, MAC4) == []

    def test_find_route_between_switches(self):
        db = square_db()
        assert db.find_route(MAC1, MAC2) == [(1, 2), (2, 1)]
        assert db.find_route(MAC1, MAC3) == [(1, 3), (3, 1)]
        assert db.find_route(MAC2, MAC4) == [(2, 3), (4, 1)]
        assert db.find_route(MAC3, MAC4) == [(3, 2), (4, 1)]

    def test_find_multiple_routes(self):
        db = square_db()
        routes = db.find_route(MAC1, MAC4, True)
        assert sorted(routes) == sorted([[(1, 2), (2, 3), (4, 1)], [(1, 3), (3, 2), (4, 1)]])
        assert sorted(db.find_route(MAC3, MAC4, True)) == [[(3, 2), (4, 1)]]

    def test_find_multiple_routes_unreachable(self):
        db = square_db()
        del db.links[1]
        for mac in (MAC2, MAC3, MAC4):
            assert db.find_route(MAC1, mac, True) == []

    def test_dfs_is_not_shortest_and_local_ports(self):
        """SURVEY.md section 4 all-pairs fixture: 1->4 goes via 3 (LIFO takes
        the largest branch), switch-local destinations end in OFPP_LOCAL."""
        db = square_db()
        assert db.find_route(MAC1, MAC4) == [(1, 3), (3, 2), (4, 1)]
        assert db.find_route(MAC4, MAC1) == [(4, 3), (3, 3), (1, 1)]
        assert db.find_route(MAC1, "00:00:00:00:00:04") == [(1, 3), (3, 2), (4, OFPP_LOCAL)]
        assert db.find_route("00:00:00:00:00:04", MAC1) == [(4, 3), (3, 3), (1, 1)]
        assert db.find_route(MAC1, "02:00:00:00:00:99") == []

    def test_return_types_are_python_ints(self):
        db = square_db()
        for hop in db.find_route(MAC1, MAC4) + db.find_route(MAC1, MAC4, True)[0]:
            assert type(hop) is tuple and all(type(x) is int for x in hop)


@pytest.mark.gpu
def test_scenarios_match_reference():
    db = TopologyDB()
    for sc in G.scenarios():
        for op in sc["ops"]:
            G.apply_op(db, op)
        for a, b, multiple, want in sc.get("queries", []):
            assert db.find_route(a, b, multiple) == G.as_tuples(want), (sc["name"], a, b, multiple)
        for a, b, exc in sc.get("raises", []):
            with pytest.raises(Exception) as ei:
                db.find_route(a, b)
            assert type(ei.value).__name__ == exc


@pytest.mark.gpu
@pytest.mark.parametrize("name", G.SMALL)
def test_all_host_pairs_match_reference(name):
    g = G.Golden(name)
    fabric = g.fabric()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    pairs = [(macs[a], macs[b]) for a, b in zip(g.pair_src, g.pair_dst)]
    got = db.find_routes(pairs)
    for i, r in enumerate(got):
        assert r == g.fdb(i), (name, i)
    if g.has_multi():
        for i, (a, b) in enumerate(pairs):
            assert db.find_route(a, b, True) == g.multi(i), (name, i)


@pytest.mark.gpu
def test_route_tables_batched_form():
    from oracle import oracle as O
    fabric = G.Golden("fat_tree_k8").fabric()
    db = fabric.populate(TopologyDB())
    t = db.route_tables("dfs")
    csr = fabric.csr()
    po, to, ho = O.dfs_tables(csr, t["sources"])
    np.testing.assert_array_equal(t["parent"], po)
    np.testing.assert_array_equal(t["port"], to)
    np.testing.assert_array_equal(t["hops"], ho)
    s = db.route_tables("shortest")
    do, nho, nhpo = O.dest_tables(csr, s["destinations"])
    np.testing.assert_array_equal(s["dist"], do)
    np.testing.assert_array_equal(s["nh"], nho)
    np.testing.assert_array_equal(s["nh_port"], nhpo)


# ----------------------------------------------------------------- CPU only --

class _FakeEngine(object):
    """Test double for RouteEngine: oracle tables + a call log."""

    def __init__(self):
        from oracle import oracle as O
        self.O = O
        self.calls = []

    def dfs_tables(self, export, srcs, with_hops=True):
        self.calls.append(("dfs", export.key, tuple(int(x) for x in srcs)))
        return self.O.dfs_tables(export.csr, srcs)

    def shortest_tables(self, export, dsts):
        self.calls.append(("sp", export.key, tuple(int(x) for x in dsts)))
        return self.O.dest_tables(export.csr, dsts)

    def pack_trees(self, export, parent, port, layout):
        # host packing (test double of sdnr_tree_pack)
        from sdnmpi_amd.engine import pack_host_tree
        return pack_host_tree(parent, port, export.csr, layout)

    def empty_rows(self, n, V, dtypes):
        return tuple(np.empty((n, V), d) for d in dtypes)

    def dfs_tree_tables(self, export, srcs, layout, out=None):
        # oracle trees packed on the host (test double of sdnr_dfs_tables_tree)
        from sdnmpi_amd.engine import pack_host_tree
        self.calls.append(("dfs", export.key, tuple(int(x) for x in srcs)))
        par, prt, hop = self.O.dfs_tables(export.csr, srcs)
        tree = pack_host_tree(par, prt, export.csr, layout)
        dep = hop.astype(np.int16 if export.csr.V <= 0xFFFF else np.int32)
        if out is None:
            return tree, dep
        out[0][...] = tree
        out[1][...] = dep
        return out

    def ecmp(self, export, dist, rows, srcs):
        # host walk of the shortest-path DAG (test double only)
        from sdnmpi_amd.engine import shortest_paths_lex
        c = export.csr
        out = []
        for r, s in zip(rows, srcs):
            d = int(np.nonzero(dist[r] == 0)[0][0])
            q = shortest_paths_lex(c.row_ptr, c.col, dist[r], int(s), d)
            out.append(np.asarray(q, np.int32).reshape(len(q), -1))
        return out

    def edge_ports(self, ends, ports):
        # membership test of routes.hip's edge_port_kernel (test double only)
        return ~np.isin(np.asarray(ports, np.uint64), np.asarray(ends, np.uint64))

    def expand(self, export, tables, rows, dsts, last_port):
        # numpy restatement of routes.hip (test double only)
        from sdnmpi_amd.engine import expand_tree_paths
        parent, port, _ = tables
        off, verts, ports = expand_tree_paths(parent, port, rows, dsts)
        ends = off[1:] - 1
        ok = off[1:] > off[:-1]
        ports[ends[ok]] = np.asarray(last_port)[ok]
        return off, verts.astype(np.int32), ports.astype(np.int32)


def test_dict_mutations_invalidate_tables():
    eng = _FakeEngine()
    db = square_db()
    db._engine = eng
    assert db.find_route(MAC1, MAC2) == [(1, 2), (2, 1)]
    n = len(eng.calls)
    assert db.find_route(MAC3, MAC4) == [(3, 2), (4, 1)]     # cached: no new call
    assert len(eng.calls) == n
    del db.links[1][2]                                      # nested dict mutation
    assert db.find_route(MAC1, MAC2) == [(1, 3), (3, 2), (4, 2), (2, 1)]
    assert len(eng.calls) == n + 1
    db.links[1][2] = Link(Port(1, 7), Port(2, 2))            # re-add, new port
    assert db.find_route(MAC1, MAC2) == [(1, 7), (2, 1)]
    db.links = {}                                           # whole-dict assignment
    assert db.find_route(MAC1, MAC2) == []


def test_host_only_changes_keep_tables():
    eng = _FakeEngine()
    db = square_db()
    db._engine = eng
    db.find_route(MAC1, MAC4)
    n = len(eng.calls)
    db.add_host(Host(MAC4, Port(4, 9)))                    # same switch, new port
    assert db.find_route(MAC1, MAC4) == [(1, 3), (3, 2), (4, 9)]
    assert len(eng.calls) == n                             # graph unchanged


def test_find_route_errors_before_engine():
    db = square_db()
    db._engine = None
    with pytest.raises(ValueError):
        db.find_route("zz:00:00:00:00:01", MAC2)
    assert db.find_route("02:00:00:00:00:77", MAC2) == []   # unknown host: no engine needed
    assert db._engine is None


def test_to_dict_snapshot():
    db = square_db()
    d = db.to_dict()
    assert len(d["links"]) == 8 and len(d["hosts"]) == 4 and len(d["switches"]) == 4


def test_tracked_dicts_are_dicts():
    db = square_db()
    assert isinstance(db.links, dict) and isinstance(db.links[1], dict)
    assert sorted(db.links[1].keys()) == [2, 3]
    v = db._versions.key()
    db.links.setdefault(9, {})[1] = Link(Port(9, 1), Port(1, 5))
    assert db._versions.key() != v
    v = db._versions.key()
    db.links[9].pop(1)
    assert db._versions.key() != v


def _link_failure_replay(db, fabric):
    """Routes for every host pair, then a failed agg-core link (Ryu reports
    both directions) and a re-added one; every route must equal the
    reference semantics on the mutated dicts, and only the affected
    sources may be recomputed."""
    from oracle import oracle as O
    macs = fabric.host_macs()
    pairs = [(a, b) for a in macs[::5] for b in macs[::3]]
    assert db.find_routes(pairs) == [O.find_route_pair(db, a, b) for a, b in pairs]
    hosts = len(set(h.port.dpid for h in db.hosts.values()))
    # a tree link of the first source's table: agg -> core 0 where core 0
    # (dpid 1) was first pushed
    t = db.route_tables("dfs")
    dp = t["dpids"]
    a = int(dp[t["parent"][0][0]])     # vertex 0 = core 0
    ab = db.links[a][1]
    ba = db.links[1][a]
    n0 = db._cache.rows_computed
    db.delete_link(ab)
    db.delete_link(ba)
    got = db.find_routes(pairs)
    assert got == [O.find_route_pair(db, a, b) for a, b in pairs]
    c = db._cache
    assert 0 < c.rows_computed - n0 < hosts and c.rows_inherited > 0
    n1 = c.rows_computed
    db.add_link(ab)
    db.add_link(ba)
    assert db.find_routes(pairs) == [O.find_route_pair(db, a, b) for a, b in pairs]
    assert db._cache.rows_computed - n1 < hosts
    # shortest mode keeps its rows across the change too
    sp = [db.find_route(a, b, True) for a, b in pairs[:40]]
    assert sp == [O.find_routes_all_shortest(db, a, b) for a, b in pairs[:40]]


def test_link_failure_incremental_fake_engine():
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(8)
    db = fabric.populate(TopologyDB())
    db._engine = _FakeEngine()
    _link_failure_replay(db, fabric)


@pytest.mark.gpu
def test_link_failure_incremental_gpu():
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(8)
    _link_failure_replay(fabric.populate(TopologyDB()), fabric)


def test_route_entries_batched_fake_engine():
    from oracle import oracle as O
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(4)
    db = fabric.populate(TopologyDB())
    db._engine = _FakeEngine()
    macs = fabric.host_macs() + ["00:00:00:00:00:05", "02:00:00:00:00:77"]   # local, unknown
    pairs = [(a, b) for a in macs for b in macs]
    got = db.find_routes(pairs)
    assert got == [O.find_route_pair(db, a, b) for a, b in pairs]


@pytest.mark.gpu
@pytest.mark.parametrize("walk", ["auto", "seg32", "v1", "v1seg32", "jump16", "serial", "int32",
                                  "p4", "p8", "pipe224", "pipe224seg32"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "torus_5x3x2"])
def test_route_entries_match_reference(monkeypatch, name, walk):
    """GPU flow-entry emission for every host pair (plus switch-local and
    unknown MACs) equals the reference's fdb lists."""
    from oracle import oracle as O
    if walk.startswith("pipe224"):               # walker / storer waves (route_seg_pipe_kernel)
        monkeypatch.setenv("SDNROUTE_ROUTE_PIPE", "2,2,4")
        if walk == "pipe224seg32":
            monkeypatch.setenv("SDNROUTE_ROUTE_OUT", "int32")
    elif walk == "serial":
        monkeypatch.setenv("SDNROUTE_ROUTE_WALK", walk)
    elif walk == "jump16":                       # packed per-entry jump walks
        monkeypatch.setenv("SDNROUTE_ROUTE_SEG", "0")
    elif walk == "seg32":                        # entries as two int32 arrays
        monkeypatch.setenv("SDNROUTE_ROUTE_OUT", "int32")
    elif walk.startswith("v1"):                  # 4-B stores instead of 16-B ones
        monkeypatch.setenv("SDNROUTE_ROUTE_V4", "0")
        if walk == "v1seg32":
            monkeypatch.setenv("SDNROUTE_ROUTE_OUT", "int32")
    elif walk != "auto":                         # int32-table jump kernels
        monkeypatch.setenv("SDNROUTE_ROUTE_PACKED", "0")
        if walk != "int32":
            monkeypatch.setenv("SDNROUTE_ROUTE_P", walk[1:])
    g = G.Golden(name)
    fabric = g.fabric()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    got = db.find_routes([(macs[int(a)], macs[int(b)]) for a, b in zip(g.pair_src, g.pair_dst)])
    assert got == [g.fdb(i) for i in range(len(g))]
    extra = macs[:3] + ["00:00:00:00:00:01", "02:00:00:00:00:77"]
    pairs = [(a, b) for a in extra for b in macs[-20:] + extra] * 4
    assert db.find_routes(pairs) == [O.find_route_pair(db, a, b) for a, b in pairs]


@pytest.mark.gpu
def test_route_entries_k48_many_pairs(monkeypatch):
    """65,536 random k=48 host pairs (paths of ~70 entries, some pairs on one
    switch): the packed 16-lane jump kernel emits the same entries as the
    one-lane-per-pair serial walk."""
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(48)
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    rng = np.random.default_rng(7)
    a = rng.integers(0, len(macs), 65536)
    b = np.where(rng.random(65536) < 0.01, a, rng.integers(0, len(macs), 65536))
    pairs = [(macs[int(x)], macs[int(y)]) for x, y in zip(a, b)]
    monkeypatch.setenv("SDNROUTE_ROUTE_WALK", "serial")
    o0, d0, p0 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_walk_kernel"
    monkeypatch.delenv("SDNROUTE_ROUTE_WALK")
    o1, d1, p1 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024,u32>"
    np.testing.assert_array_equal(o0, o1)
    np.testing.assert_array_equal(d0, d1)
    np.testing.assert_array_equal(p0, p1)
    monkeypatch.setenv("SDNROUTE_ROUTE_OUT", "int32")
    o3, d3, p3 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024>"
    np.testing.assert_array_equal(o0, o3)
    np.testing.assert_array_equal(d0, d3)
    np.testing.assert_array_equal(p0, p3)
    monkeypatch.setenv("SDNROUTE_ROUTE_SEG", "0")
    o2, d2, p2 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_jump_packed_kernel<16>"
    np.testing.assert_array_equal(o0, o2)
    np.testing.assert_array_equal(d0, d2)
    np.testing.assert_array_equal(p0, p2)


@pytest.mark.gpu
@pytest.mark.parametrize("fab", ["fat_tree:48", "torus:16,16,16"])
def test_route_entries_runs_and_long_paths(monkeypatch, fab):
    """The output-centric expansion (route_seg_packed_kernel): pairs in runs
    of one (source switch, destination switch) -- all hosts of a few switch
    pairs, in the all-pairs order -- mixed with scattered and same-switch
    pairs; on the torus the DFS routes (hundreds to thousands of entries)
    overflow the per-wave buffer and take the direct walk.  Entries equal the
    one-lane-per-pair serial walk's."""
    from sdnmpi_amd import topologies as T
    fabric = T.by_name(fab)
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    rng = np.random.default_rng(11)
    sw = fabric.host_table()[0]
    order = np.argsort(sw, kind="stable")
    ms = [macs[int(i)] for i in order]          # hosts grouped by switch
    block = ms[: 3 * 24] if fab.startswith("fat") else ms[:40]
    pairs = [(a, b) for a in block for b in block]
    pairs += [(macs[int(x)], macs[int(y)]) for x, y in rng.integers(0, len(macs), (3000, 2))]
    pairs += [(macs[5], macs[5])] * 70
    monkeypatch.setenv("SDNROUTE_ROUTE_WALK", "serial")
    o0, d0, p0 = db.route_entries(pairs)
    monkeypatch.delenv("SDNROUTE_ROUTE_WALK")
    o1, d1, p1 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024,u32>"
    monkeypatch.setenv("SDNROUTE_ROUTE_OUT", "int32")
    o2, d2, p2 = db.route_entries(pairs)
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024>"
    for a, b in ((o1, o2), (d1, d2), (p1, p2)):
        np.testing.assert_array_equal(a, b)
    # walker / storer shapes, and the one-role kernel, both forms
    for shape in ("0", "4,4,2", "6,2,2", "4,2,3", "4,2,2", "8,4,2", "6,3,2", "2,2,2", "2,2,4",
                  "1,1,4", "3,3,2", "2,1,3"):
        monkeypatch.setenv("SDNROUTE_ROUTE_PIPE", shape)
        for out in ("int32", "u32"):
            monkeypatch.setenv("SDNROUTE_ROUTE_OUT", out)
            o3, d3, p3 = db.route_entries(pairs)
            for a, b in ((o0, o3), (d0, d3), (p0, p3)):
                np.testing.assert_array_equal(a, b)
    monkeypatch.delenv("SDNROUTE_ROUTE_PIPE")
    monkeypatch.setenv("SDNROUTE_ROUTE_V4", "0")         # 4-B stores, both forms
    for out in ("int32", "u32"):
        monkeypatch.setenv("SDNROUTE_ROUTE_OUT", out)
        o3, d3, p3 = db.route_entries(pairs)
        for a, b in ((o1, o3), (d1, d3), (p1, p3)):
            np.testing.assert_array_equal(a, b)
    monkeypatch.delenv("SDNROUTE_ROUTE_V4")
    monkeypatch.delenv("SDNROUTE_ROUTE_OUT")
    if not fab.startswith("fat"):
        assert int(np.diff(o0).max()) > 1024     # some pairs take the direct walk
    np.testing.assert_array_equal(o0, o1)
    np.testing.assert_array_equal(d0, d1)
    np.testing.assert_array_equal(p0, p1)


@pytest.mark.gpu
def test_route_entries_k48_golden_pairs():
    g = G.Golden("fat_tree_k48_sample")
    fabric = g.fabric()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    got = db.find_routes([(macs[int(a)], macs[int(b)]) for a, b in zip(g.pair_src, g.pair_dst)])
    assert got == [g.fdb(i) for i in range(len(g))]


def test_find_routes_multiple_batched_fake_engine():
    from oracle import oracle as O
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(4)
    db = fabric.populate(TopologyDB())
    db._engine = _FakeEngine()
    macs = fabric.host_macs() + ["00:00:00:00:00:05", "02:00:00:00:00:77"]
    pairs = [(a, b) for a in macs[::3] for b in macs]
    assert db.find_routes(pairs, True) == [O.find_routes_all_shortest(db, a, b) for a, b in pairs]


@pytest.mark.gpu
@pytest.mark.parametrize("name", G.MULTI)
def test_ecmp_sets_match_reference(name):
    """GPU-counted and -unranked ECMP sets equal the reference's
    find_route(..., multiple=True) lists (golden fixtures)."""
    g = G.Golden(name)
    fabric = g.fabric()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    pairs = [(macs[int(a)], macs[int(b)]) for a, b in zip(g.pair_src, g.pair_dst)]
    assert db.find_routes(pairs * (1 if len(pairs) >= 16 else 16), True)[:len(pairs)] == \
        [g.multi(i) for i in range(len(g))]


@pytest.mark.gpu
def test_ecmp_sets_k48_sampled():
    """k=48: 576 shortest routes per inter-pod pair, vs the host walk of the
    oracle's shortest-path DAG (the reference itself cannot enumerate them)."""
    from oracle import oracle as O
    g = G.Golden("fat_tree_k48_sample")
    fabric = g.fabric()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    pairs = [(macs[int(a)], macs[int(b)]) for a, b in zip(g.pair_src[:40], g.pair_dst[:40])]
    got = db.find_routes(pairs, True)
    assert got == [O.find_routes_all_shortest(db, a, b) for a, b in pairs]
    assert max(len(r) for r in got) == 576


def test_edge_port_helpers_match_reference_loop():
    _edge_port_replay(_FakeEngine())


@pytest.mark.gpu
def test_edge_port_helpers_gpu():
    """The device flood-port mask (sdnr_edge_ports) against the reference's
    loop through link deletions and whole-entry removal."""
    _edge_port_replay(None)


def _edge_port_replay(engine):
    """is_edge_port / edge_ports / broadcast_ports vs the reference's
    O(links) loop (sdnmpi/topology.py:150-177), before and after link
    changes."""
    from sdnmpi_amd import topologies as T
    from sdnmpi_amd.objects import Switch

    def ref_is_edge(db, port):            # topology.py:150-155, restated
        for nb in db.links.values():
            for lk in nb.values():
                if port == lk.src or port == lk.dst:
                    return False
        return True

    fabric = T.fat_tree(4)
    db = fabric.populate(TopologyDB())
    if engine is not None:
        db._engine = engine
    ports = {}
    for nb in db.links.values():
        for lk in nb.values():
            ports.setdefault(lk.src.dpid, set()).add(lk.src.port_no)
    for h in db.hosts.values():
        ports.setdefault(h.port.dpid, set()).add(h.port.port_no)
    sws = []
    for d in sorted(ports):
        sw = Switch(d)
        sw.ports = [Port(d, n) for n in sorted(ports[d])] + [Port(d, 0xfffe)]
        sws.append(sw)

    def check():
        for sw in sws:
            for p in sw.ports:
                assert db.is_edge_port(p) == ref_is_edge(db, p)
            want = [p for p in sw.ports if ref_is_edge(db, p) and not p.is_reserved()
                    and p.port_no != 3]
            assert db.edge_ports(sw, in_port=3) == want
        # _do_broadcast(data, dpid, in_port) over every switch
        src = sws[1].dp.id
        bc = db.broadcast_ports(src, 1)
        for sw in sws:
            want = [p.port_no for p in sw.ports if ref_is_edge(db, p) and not p.is_reserved()
                    and not (sw.dp.id == src and p.port_no == 1)]
            assert bc[sw.dp.id] == want
        # a port of no switch object (reference: any Port works)
        assert db.is_edge_port(Port(sws[0].dp.id, 999)) is True

    for sw in sws:
        db.add_switch(sw)
    check()
    lk = next(iter(db.links[sws[-1].dp.id].values()))
    db.delete_link(lk)
    check()
    del db.links[lk.dst.dpid]
    check()


@pytest.mark.parametrize("budget_rows", [1, 3, 7])
def test_table_budget_eviction_fake_engine(budget_rows):
    """A table budget of a few rows: batches shrink, old rows are evicted,
    route_entries / find_routes(multiple=True) / route_tables run in chunks of
    sources -- and every answer still equals the reference semantics."""
    from oracle import oracle as O
    from sdnmpi_amd import topologies as T
    from sdnmpi_amd.engine import dfs_row_bytes, sp_row_bytes
    fabric = T.fat_tree(4)
    csr = fabric.csr()
    budget = budget_rows * dfs_row_bytes(csr)          # compact rows: 6 B per entry
    assert dfs_row_bytes(csr) == 6 * csr.V and sp_row_bytes(csr) == 4 * csr.V
    db = fabric.populate(TopologyDB(table_budget=budget))
    eng = _FakeEngine()
    db._engine = eng
    macs = fabric.host_macs()
    pairs = [(a, b) for a in macs for b in macs[::2]]
    assert db.find_routes(pairs) == [O.find_route_pair(db, a, b) for a, b in pairs]
    assert len(db._cache.dfs) <= budget_rows
    assert db._cache.dfs.size <= budget_rows           # the pool never outgrows the budget
    for a, b in pairs[::7]:
        assert db.find_route(a, b) == O.find_route_pair(db, a, b)
    assert db.find_routes(pairs[:40], True) == \
        [O.find_routes_all_shortest(db, a, b) for a, b in pairs[:40]]
    assert len(db._cache.sp) <= max(1, budget // sp_row_bytes(csr))
    t = db.route_tables("dfs")
    po, to, ho = O.dfs_tables(fabric.csr(), t["sources"])
    np.testing.assert_array_equal(t["parent"], po)
    np.testing.assert_array_equal(t["hops"], ho)
    s = db.route_tables("shortest")
    do, _, nhpo = O.dest_tables(fabric.csr(), s["destinations"])
    np.testing.assert_array_equal(s["dist"], do)
    np.testing.assert_array_equal(s["nh_port"], nhpo)


def test_unsigned_64bit_dpids():
    """Ryu datapath ids are unsigned 64-bit: dpids >= 2**63 sort and route as
    the reference's Python ints do."""
    from oracle import oracle as O
    big = [2**63 + 5, 2**64 - 1, 7, 2**63]
    db = TopologyDB()
    db._engine = _FakeEngine()
    for d in big:
        db.add_switch(Switch(d))
    for i, u in enumerate(big):
        for j, v in enumerate(big):
            if u != v and (i + j) % 3 != 0:
                db.add_link(Link(Port(u, 10 + j), Port(v, 10 + i)))
    macs = ["02:00:00:00:01:%02x" % i for i in range(len(big))]
    for m, d in zip(macs, big):
        db.add_host(Host(m, Port(d, 1)))
    ex = db.graph()
    assert [int(x) for x in ex.csr.dpids] == sorted(big)
    for a in macs:
        for b in macs:
            assert db.find_route(a, b) == O.find_route_pair(db, a, b)
            assert db.find_route(a, b, True) == O.find_routes_all_shortest(db, a, b)


def _replay_switch_fdb(db, pairs, keys=None):
    """Reference-shaped replay of Router._add_flows_for_path into a
    SwitchFDB-like dict (sdnmpi/router.py:83-104, util/switch_fdb.py:6-9):
    fdb = find_route(src, dst) per pair, one (dpid, (src, dst)) -> out_port
    per hop, an existing key kept."""
    from oracle import oracle as O
    out = {}
    for i, (a, b) in enumerate(pairs):
        key = keys[i] if keys else (a, b)
        for dpid, port in O.find_route_pair(db, a, b):
            sw = out.setdefault(dpid, {})
            if key not in sw:
                sw[key] = port
    return out


def _grouped_to_dict(dpids, off, keys, port):
    out = {}
    for k in range(dpids.shape[0]):
        sw = out.setdefault(int(dpids[k]), {})
        for j in range(int(off[k]), int(off[k + 1])):
            sw[keys[j]] = int(port[j])
    return out


def _switch_fdb_check(db, fabric, rng):
    macs = fabric.host_macs()
    pairs = [(macs[int(a)], macs[int(b)]) for a, b in rng.integers(0, len(macs), (300, 2))]
    pairs += pairs[:20] + [(macs[0], "02:00:00:00:00:77")]      # repeated keys, unknown host
    dpids, off, pid, port, last = db.switch_fdb_entries(pairs)
    assert np.all(np.diff(dpids) > 0)
    got = _grouped_to_dict(dpids, off, [pairs[int(i)] for i in pid], port)
    assert got == _replay_switch_fdb(db, pairs)
    # the last flag marks each pair's destination switch
    for j in np.nonzero(last)[0][:50]:
        a, b = pairs[int(pid[j])]
        k = int(np.searchsorted(off, j, side="right") - 1)
        assert int(dpids[k]) == db.hosts[b].port.dpid
    # the MPI rank set: every ordered rank pair, keyed by (src rank, dst rank)
    ranks = {r: macs[int(h)] for r, h in enumerate(rng.choice(len(macs), 12, replace=False))}
    dpids, off, sr, dr, port, last = db.mpi_flow_entries(ranks, coll_type=3)
    rp = [(a, b) for a in sorted(ranks) for b in sorted(ranks) if a != b]
    want = _replay_switch_fdb(db, [(ranks[a], ranks[b]) for a, b in rp], keys=rp)
    got = _grouped_to_dict(dpids, off, list(zip(sr.tolist(), dr.tolist())), port)
    assert got == want
    # several ranks per host (ranks take eth.src, process.py:108-109): the
    # router keys each flow by (src MAC, virtual MAC), so rank pairs sharing
    # both hosts still get one flow each (router.py:189-193)
    from oracle import oracle as O
    from sdnmpi_amd.util.topology_db import sdn_mpi_mac
    hosts = rng.choice(len(macs), 4, replace=False)
    ranks = {r: macs[int(hosts[r % 4])] for r in range(10)}
    dpids, off, sr, dr, port, last = db.mpi_flow_entries(ranks, coll_type=2)
    rp = [(a, b) for a in sorted(ranks) for b in sorted(ranks) if a != b]
    keys = [(ranks[a], sdn_mpi_mac(2, a, b)) for a, b in rp]
    want = _replay_switch_fdb(db, [(ranks[a], ranks[b]) for a, b in rp], keys=keys)
    got = _grouped_to_dict(dpids, off, [(ranks[a], sdn_mpi_mac(2, a, b))
                                        for a, b in zip(sr.tolist(), dr.tolist())], port)
    assert got == want
    assert sum(len(v) for v in got.values()) == int(off[-1])   # no pair's entries dropped
    n_hops = sum(len(O.find_route_pair(db, ranks[a], ranks[b])) for a, b in rp)
    assert int(off[-1]) == n_hops


def test_switch_fdb_entries_fake_engine():
    from sdnmpi_amd import topologies as T
    for fabric in (T.fat_tree(4), T.fat_tree(8)):
        db = fabric.populate(TopologyDB())
        db._engine = _FakeEngine()
        _switch_fdb_check(db, fabric, np.random.default_rng(3))


def test_sdn_mpi_mac_matches_router_decoding():
    """sdn_mpi_mac round-trips through the router's decoding (reference
    sdnmpi/router.py:163-178): locally administered bit, collective type,
    little-endian int16 ranks."""
    import struct
    from sdnmpi_amd.util.topology_db import sdn_mpi_mac
    for coll, a, b in [(0, 0, 1), (3, 17, 4095), (63, 32767, 0), (5, 300, 256)]:
        raw = bytes(int(x, 16) for x in sdn_mpi_mac(coll, a, b).split(":"))
        assert raw[0] & 0x02
        assert raw[0] >> 2 == coll
        assert struct.unpack("<h", raw[2:4])[0] == a
        assert struct.unpack("<h", raw[4:6])[0] == b


@pytest.mark.gpu
def test_switch_fdb_entries_gpu():
    from sdnmpi_amd import topologies as T
    for fabric in (T.fat_tree(8), T.fat_tree(48)):
        db = fabric.populate(TopologyDB())
        _switch_fdb_check(db, fabric, np.random.default_rng(4))


@pytest.mark.gpu
def test_route_entries_wide_host_port(monkeypatch):
    """A destination host port above 0xffff cannot ride in the u32 entry
    (switch | port << 16): route_entries must take the int32 expansion and
    still equal the reference's fdbs; the u32 form serves the other pairs."""
    from oracle import oracle as O
    from sdnmpi_amd import topologies as T
    fabric = T.fat_tree(4)
    db = fabric.populate(TopologyDB())
    macs = sorted(db.hosts)
    wide = macs[3]
    h = db.hosts[wide]
    db.add_host(Host(wide, Port(h.port.dpid, 70000)))
    pairs = [(a, b) for a in macs for b in macs]
    want = [O.find_route_pair(db, a, b) for a, b in pairs]
    assert db.find_routes(pairs) == want
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024>"   # int32 form
    narrow = [(a, b) for a, b in pairs if b != wide]
    assert db.find_routes(narrow) == [O.find_route_pair(db, a, b) for a, b in narrow]
    assert db.engine.ctx.last_kernel() == "route_seg_packed_kernel<1024,u32>"


@pytest.mark.gpu
def test_dropin_empty_batches():
    """The batch calls of the drop-in on an empty request list: empty
    results, as the reference's loop over no pairs installs nothing."""
    g = G.Golden("fat_tree_k8")
    db = g.fabric().populate(TopologyDB())
    assert db.find_routes([]) == []
    assert db.find_routes([], multiple=True) == []
    off, dp, pt = db.route_entries([])
    assert list(off) == [0] and len(dp) == 0 and len(pt) == 0
    dpids, soff, pid, opt, last = db.switch_fdb_entries([])
    assert len(dpids) == len(pid) == len(opt) == len(last) == 0 and list(soff) == [0]
    dpids, soff, sr, dr, opt, last = db.mpi_flow_entries({})
    assert len(dpids) == len(sr) == len(dr) == len(opt) == 0 and list(soff) == [0]
    dpids, soff, sr, dr, opt, last = db.mpi_flow_entries({0: g.fabric().host_macs()[0]})
    assert len(dpids) == 0 and list(soff) == [0]          # one rank: no pairs
    macs = g.fabric().host_macs()
    assert db.find_routes([(macs[0], macs[1])]) == [db.find_route(macs[0], macs[1])]
