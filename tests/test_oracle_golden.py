"""Pin the oracle to the reference: every golden vector the reference produced
(tests/golden/make_golden.py) must be reproduced by the C restatement
(per-source tables) and by the per-pair Python restatement.  CPU only."""
import numpy as np
import pytest

import golden_util as G
from oracle import oracle as O
from sdnmpi_amd import topologies as T


class _DictDB(object):
    """The reference's three dicts, nothing else (input of the per-pair oracle)."""

    def __init__(self):
        self.switches, self.links, self.hosts = {}, {}, {}

    def add_switch(self, s):
        self.switches[s.dp.id] = s

    def delete_switch(self, s):
        self.switches.pop(s.dp.id, None)

    def add_link(self, lk):
        self.links.setdefault(lk.src.dpid, {})[lk.dst.dpid] = lk

    def delete_link(self, lk):
        if lk.src.dpid in self.links:
            self.links[lk.src.dpid].pop(lk.dst.dpid, None)

    def add_host(self, h):
        self.hosts[h.mac] = h


def oracle_fdbs_from_tables(g, fabric):
    csr = fabric.csr()
    srcs, hv, hp = G.host_vertex_rows(fabric)
    parent, port, hops = O.dfs_tables(csr, srcs)
    row = {int(s): i for i, s in enumerate(srcs)}
    out = []
    for a, b in zip(g.pair_src, g.pair_dst):
        s, d = int(hv[a]), int(hv[b])
        r = row[s]
        out.append(O.tree_fdb(csr, parent[r], port[r], s, d, hp[b]))
    return out, (parent, port, hops, srcs)


@pytest.mark.parametrize("name", G.SMALL)
def test_dfs_tables_match_reference(name):
    g = G.Golden(name)
    fabric = g.fabric()
    got, (parent, port, hops, srcs) = oracle_fdbs_from_tables(g, fabric)
    for i in range(len(g)):
        assert got[i] == g.fdb(i), (name, i)
    # hop counts: tree depth == len(route) - 1
    hv, _ = fabric.host_table()
    row = {int(s): i for i, s in enumerate(srcs)}
    for i in range(len(g)):
        h = hops[row[int(hv[g.pair_src[i]])], int(hv[g.pair_dst[i]])]
        assert (h < 0 and not g.fdb(i)) or h == len(g.fdb(i)) - 1


@pytest.mark.parametrize("name", G.SMALL)
def test_per_pair_oracle_matches_reference(name):
    g = G.Golden(name)
    fabric = g.fabric()
    db = fabric.populate(_DictDB())
    macs = fabric.host_macs()
    step = max(1, len(g) // 1500)
    for i in range(0, len(g), step):
        a, b = macs[g.pair_src[i]], macs[g.pair_dst[i]]
        assert O.find_route_pair(db, a, b) == g.fdb(i)
        # the path-copying form (the reference's own search shape, timed as
        # bench.py's cpu_reference_path)
        assert O.find_route_pair(db, a, b, copying=True) == g.fdb(i)


@pytest.mark.parametrize("name", ["fat_tree_k48_sample", "dragonfly_a16_h8_p8_sample"])
def test_per_pair_copying_oracle_matches_reference_fullsize(name):
    """The path-copying restatement on the reference's own sampled pairs of
    the full-size fabrics (the bench's CPU reference-path workload)."""
    g = G.Golden(name)
    fabric = g.fabric()
    db = fabric.populate(_DictDB())
    macs = fabric.host_macs()
    for i in range(0, len(g), max(1, len(g) // 40)):
        a, b = macs[g.pair_src[i]], macs[g.pair_dst[i]]
        assert O.find_route_pair(db, a, b, copying=True) == g.fdb(i)


@pytest.mark.parametrize("name", G.MULTI)
def test_multiple_routes_match_reference(name):
    g = G.Golden(name)
    assert g.has_multi()
    fabric = g.fabric()
    db = fabric.populate(_DictDB())
    macs = fabric.host_macs()
    csr = fabric.csr()
    hv, hp = fabric.host_table()
    dsts = np.unique(hv)
    dist, nh, nh_port = O.dest_tables(csr, dsts)
    drow = {int(d): i for i, d in enumerate(dsts)}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        want = g.multi(i)
        assert O.find_routes_all_shortest(db, macs[a], macs[b]) == want
        # routes[0] == greedy smallest-next-hop walk of the dest tables
        s, d = int(hv[a]), int(hv[b])
        r = drow[d]
        if not want:
            assert dist[r, s] == 0xFFFF
            continue
        assert dist[r, s] == len(want[0]) - 1
        x, walk = s, []
        while x != d:
            walk.append((int(csr.dpids[x]), int(nh_port[r, x])))
            x = int(nh[r, x])
        walk.append((int(csr.dpids[d]), int(hp[b])))
        assert walk == want[0]


@pytest.mark.parametrize("name", G.MULTI)
def test_ecmp_counts_match_reference(name):
    """oracle.ecmp_counts == the number of routes the reference returned for
    every multiple=True fixture pair."""
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    hv, _ = fabric.host_table()
    dsts = np.unique(hv)
    dist, _, _ = O.dest_tables(csr, dsts)
    drow = {int(d): i for i, d in enumerate(dsts)}
    counts = {}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        d = int(hv[b])
        if d not in counts:
            counts[d] = O.ecmp_counts(csr, dist[drow[d]])
        assert int(counts[d][int(hv[a])]) == len(g.multi(i)), (name, i)


@pytest.mark.parametrize("name", G.MULTI)
def test_bfs_tree_is_lexmin_shortest(name):
    """Per-source FIFO-BFS tree path == routes[0] of multiple=True."""
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    hv, hp = fabric.host_table()
    srcs = np.unique(hv)
    parent, port, _ = O.bfs_tables(csr, srcs)
    row = {int(s): i for i, s in enumerate(srcs)}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        want = g.multi(i)
        r = row[int(hv[a])]
        got = O.tree_fdb(csr, parent[r], port[r], int(hv[a]), int(hv[b]), hp[b])
        assert got == (want[0] if want else [])


def test_scenarios_per_pair_oracle():
    db = _DictDB()
    for sc in G.scenarios():
        for op in sc["ops"]:
            G.apply_op(db, op)
        for a, b, multiple, want in sc.get("queries", []):
            if multiple:
                got = O.find_routes_all_shortest(db, a, b)
            else:
                got = O.find_route_pair(db, a, b)
                assert O.find_route_pair(db, a, b, copying=True) == got
            assert got == G.as_tuples(want), (sc["name"], a, b, multiple)
        for a, b, exc in sc.get("raises", []):
            with pytest.raises(Exception) as ei:
                O.find_route_pair(db, a, b)
            assert type(ei.value).__name__ == exc


def test_apsp_matches_bfs():
    f = T.dragonfly(4, 2, 2)
    csr = f.csr()
    D = O.apsp(csr)
    dist, _, _ = O.dest_tables(csr, np.arange(csr.V))
    # dest_tables row d = distances x -> d, i.e. column d of APSP
    assert np.array_equal(D.T, dist)


@pytest.mark.slow
@pytest.mark.parametrize("name", sorted(G.LARGE))
def test_large_samples_match_reference(name):
    g = G.Golden(name)
    fabric = g.fabric()              # also checks the generator digest
    csr = fabric.csr()
    hv, hp = fabric.host_table()
    srcs = np.unique(hv[g.pair_src])
    parent, port, _ = O.dfs_tables(csr, srcs, with_hops=False)
    row = {int(s): i for i, s in enumerate(srcs)}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        r = row[int(hv[a])]
        got = O.tree_fdb(csr, parent[r], port[r], int(hv[a]), int(hv[b]), hp[b])
        assert got == g.fdb(i), (name, i)
