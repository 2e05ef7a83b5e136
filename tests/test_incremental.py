"""Incremental table maintenance (sdnmpi_amd.incremental): the row tests
are checked against full recomputation by the oracle.  Soundness: every row
the test keeps is bit-identical after the change.  Exactness for single
events: every row it flags really changes.  CPU only (oracle tables stand in
for the GPU's); the drop-in's use of it runs with the fake engine here and
on the GPU in test_topologydb_dropin.py."""
import numpy as np
import pytest

from oracle import oracle as O
from sdnmpi_amd import topologies as T
from sdnmpi_amd.incremental import dfs_rows_affected, edge_diff, sp_rows_affected
from sdnmpi_amd.topologies import build_csr


def _links(csr):
    src = np.repeat(np.arange(csr.V), np.diff(csr.row_ptr))
    return {(int(a), int(b)): int(p) for a, b, p in zip(src, csr.col, csr.port)}


def _csr(dpids, links):
    ks = sorted(links)
    return build_csr([dpids[a] for a, _ in ks], [dpids[b] for _, b in ks],
                     [links[k] for k in ks], extra_vertices=dpids)


def _tables(csr):
    srcs = np.arange(csr.V, dtype=np.int32)
    p, t, h = O.dfs_tables(csr, srcs, nthreads=4)
    d, nh, nhp = O.dest_tables(csr, srcs, nthreads=4)
    return (p, t, h), (d, nh, nhp)


def _check(old_csr, new_csr, single):
    (p0, t0, h0), (d0, n0, q0) = _tables(old_csr)
    (p1, t1, h1), (d1, n1, q1) = _tables(new_csr)
    diff = edge_diff(old_csr, new_csr)
    assert diff is not None
    srcs = np.arange(old_csr.V)
    fa = dfs_rows_affected(p0, h0, srcs, diff)
    changed = ((p0 != p1) | (t0 != t1) | (h0 != h1)).any(1)
    assert not (changed & ~fa).any(), "kept a DFS row that changed"
    sa = sp_rows_affected(d0, n0, diff)
    schanged = ((d0 != d1) | (n0 != n1) | (q0 != q1)).any(1)
    assert not (schanged & ~sa).any(), "kept a shortest row that changed"
    if single:
        assert not (fa & ~changed).any(), "flagged a DFS row that does not change"
        assert not (sa & ~schanged).any(), "flagged a shortest row that does not change"
    return int(fa.sum()), int(sa.sum())


def _random_directed(V, E, rng):
    links = {}
    while len(links) < E:
        a, b = rng.integers(0, V, 2)
        if a != b:
            links[(int(a), int(b))] = int(rng.integers(1, 60))
    return links


@pytest.mark.parametrize("seed", range(6))
def test_single_link_events_exact(seed):
    rng = np.random.default_rng(seed)
    V = 24
    dpids = list(range(100, 100 + V))
    links = _random_directed(V, 70, rng)
    base = _csr(dpids, links)
    keys = sorted(links)
    for _ in range(8):
        # removal
        k = keys[int(rng.integers(len(keys)))]
        l2 = dict(links)
        del l2[k]
        _check(base, _csr(dpids, l2), single=True)
        # new port on an existing link
        l2 = dict(links)
        l2[k] = links[k] + 100
        _check(base, _csr(dpids, l2), single=True)
        # addition
        while True:
            a, b = (int(x) for x in rng.integers(0, V, 2))
            if (a, b) not in links:
                break
        l2 = dict(links)
        l2[(a, b)] = 77
        _check(base, _csr(dpids, l2), single=True)


@pytest.mark.parametrize("seed", range(4))
def test_batched_events_sound(seed):
    rng = np.random.default_rng(100 + seed)
    V = 30
    dpids = list(range(5, 5 + V))
    links = _random_directed(V, 90, rng)
    base = _csr(dpids, links)
    keys = sorted(links)
    for _ in range(6):
        l2 = dict(links)
        for k in rng.choice(len(keys), 3, replace=False):
            del l2[keys[int(k)]]
        for _ in range(3):
            a, b = (int(x) for x in rng.integers(0, V, 2))
            if a != b:
                l2[(a, b)] = int(rng.integers(1, 9))
        _check(base, _csr(dpids, l2), single=False)


def test_fat_tree_link_failure_touches_few_rows():
    """A failed agg-core link (both directions, as Ryu reports it) on the
    k=8 fat-tree: only the sources whose tree uses it are recomputed."""
    csr = T.fat_tree(8).csr()
    links = _links(csr)
    dp = csr.dpids.tolist()
    core, agg = csr.index_of([1])[0], csr.index_of([1 + 16])[0]   # core 0 <-> agg(0,0)
    l2 = {k: v for k, v in links.items() if k not in ((core, agg), (agg, core))}
    fa, sa = _check(csr, _csr(dp, l2), single=False)
    assert 0 < fa < csr.V and sa > 0      # every shortest row uses core 0 <-> agg(0,0)


def test_vertex_set_change_is_not_incremental():
    a = T.fat_tree(4).csr()
    b = T.fat_tree(6).csr()
    assert edge_diff(a, b) is None
