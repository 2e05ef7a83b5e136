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


# ------------------------------------------------------------------ GPU --
# The drop-in's device pool runs the row test as one kernel
# (sdnr_dfs_rows_affected, csrc/incremental.hip); its verdict must equal the
# host test above -- itself exact / sound against full recomputation -- in
# every row layout the pool keeps, free rows included.

def _device_verdict(ctx, old, csr, p, t, h, srcs, diff, layout):
    import torch
    from sdnmpi_amd import _native
    from sdnmpi_amd.engine import PORT16, SLOT, pack_host_tree
    dev = torch.device("cuda", 0)
    ctx.upload(csr)
    V = csr.V
    if layout == "int32":
        tree, depth, lay = p.astype(np.int32), h.astype(np.int32), _native.TREE_INT32
        blank_t, blank_d = -1, -1
    else:
        lay = _native.TREE_PORT16 if layout == "port16" else _native.TREE_SLOT
        tree = pack_host_tree(p, t, old, PORT16 if layout == "port16" else SLOT)
        tree = np.asarray(tree).view(np.int32) if np.asarray(tree).dtype != np.int32 else tree
        depth = h.astype(np.int16) if V <= 0xFFFF else h.astype(np.int32)
        blank_t, blank_d = -1, -1
    # interleave free rows (source -1, blank tables) with the real ones
    n = len(srcs)
    order = np.arange(2 * n)
    real = order % 2 == 0
    tr = np.full((2 * n, V), blank_t, tree.dtype)
    dp = np.full((2 * n, V), blank_d, depth.dtype)
    rs = np.full(2 * n, -1, np.int32)
    tr[real], dp[real], rs[real] = tree, depth, srcs
    tt = torch.from_numpy(tr).to(dev)
    td = torch.from_numpy(dp).to(dev)
    ts = torch.from_numpy(rs).to(dev)
    rm = [np.concatenate([diff.removed[0], diff.ported[0]]),
          np.concatenate([diff.removed[1], diff.ported[1]])]
    links = np.concatenate([np.stack(rm, 1).reshape(-1),
                            np.stack([diff.added[0], diff.added[1]], 1).reshape(-1)]).astype(np.int32)
    tl = torch.from_numpy(links if links.size else np.zeros(2, np.int32)).to(dev)
    out = torch.full((2 * n,), 7, dtype=torch.uint8, device=dev)
    ctx.dfs_rows_affected_device(tt.data_ptr(), td.data_ptr(), lay, td.element_size(), 2 * n,
                                 ts.data_ptr(), tl.data_ptr(), rm[0].size, diff.added[0].size,
                                 out.data_ptr())
    ctx.synchronize()
    v = out.cpu().numpy()
    assert set(np.unique(v)) <= {0, 1}
    assert not v[~real].any(), "a free row was flagged"
    return v[real].astype(bool)


def _gpu_cases(seed):
    rng = np.random.default_rng(500 + seed)
    V = 40
    dpids = list(range(1000, 1000 + V))
    links = _random_directed(V, 120, rng)
    base = _csr(dpids, links)
    keys = sorted(links)
    out = []
    for _ in range(5):
        k = keys[int(rng.integers(len(keys)))]
        l2 = dict(links)
        del l2[k]
        out.append(_csr(dpids, l2))
        l2 = dict(links)
        l2[k] = links[k] + 50
        out.append(_csr(dpids, l2))
        while True:
            a, b = (int(x) for x in rng.integers(0, V, 2))
            if (a, b) not in links:
                break
        l2 = dict(links)
        l2[(a, b)] = 77
        out.append(_csr(dpids, l2))
        l2 = dict(links)                       # a batch: 2 removed, 3 added
        for j in rng.choice(len(keys), 2, replace=False):
            del l2[keys[int(j)]]
        for _ in range(3):
            a, b = (int(x) for x in rng.integers(0, V, 2))
            l2[(a, b)] = 5
        out.append(_csr(dpids, l2))
    return base, out


@pytest.fixture(scope="module")
def gctx():
    from sdnmpi_amd import _native
    c = _native.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["port16", "slot", "int32"])
@pytest.mark.parametrize("seed", range(3))
def test_device_row_test_equals_host(gctx, seed, layout):
    base, news = _gpu_cases(seed)
    srcs = np.arange(base.V, dtype=np.int32)
    p, t, h = O.dfs_tables(base, srcs, nthreads=4)
    for new in news:
        diff = edge_diff(base, new)
        want = np.asarray(dfs_rows_affected(p, h, srcs, diff), bool)
        got = _device_verdict(gctx, base, new, p, t, h, srcs, diff, layout)
        np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("fab", ["fat_tree:8", "fat_tree:48", "torus:8,8,8", "dragonfly:4,2,2"])
def test_device_row_test_fabrics(gctx, fab):
    """Added and removed links on the structured fabrics (deep trees on the
    torus: the climbs run hundreds of levels), every vertex as a source."""
    rng = np.random.default_rng(7)
    csr = T.by_name(fab).csr()
    links = _links(csr)
    dp = csr.dpids.tolist()
    srcs = np.arange(csr.V, dtype=np.int32)
    if csr.V > 1000:
        srcs = np.unique(rng.integers(0, csr.V, 400)).astype(np.int32)
    p, t, h = O.dfs_tables(csr, srcs, nthreads=8)
    keys = sorted(links)
    for _ in range(4):
        l2 = dict(links)
        a, b = keys[int(rng.integers(len(keys)))]
        del l2[(a, b)]
        l2.pop((b, a), None)                  # Ryu reports both directions
        while True:
            x, y = (int(z) for z in rng.integers(0, csr.V, 2))
            if x != y and (x, y) not in links:
                break
        l2[(x, y)] = 90
        new = _csr(dp, l2)
        diff = edge_diff(csr, new)
        want = np.asarray(dfs_rows_affected(p, h, srcs, diff), bool)
        for layout in ("port16", "slot"):
            got = _device_verdict(gctx, csr, new, p, t, h, srcs, diff, layout)
            np.testing.assert_array_equal(got, want)
