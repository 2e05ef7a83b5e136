"""HIP tables vs the oracle, through the C ABI, on a gfx950 device.

Bit-exact for every table (integer work): parent/port/hops of the default
route, dist/nh/nh_port of the shortest mode, the APSP matrix.  Small fabrics
are checked over ALL vertices as sources/destinations, the full-size
BASELINE fabrics over all host-bearing sources (k=48, dragonfly) or a spread
sample (torus 32^3, Jellyfish 100k) plus the reference's own sampled pairs.
"""
import os

import numpy as np
import pytest

import golden_util as G
from oracle import oracle as O
from sdnmpi_amd import _native
from sdnmpi_amd import topologies as T

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def ctx():
    c = _native.Context(0)
    yield c
    c.close()


def _strategy(monkeypatch, dfs=None, ell=None):
    if dfs == "global-ring128":
        monkeypatch.setenv("SDNROUTE_DFS_RING", "128")
        dfs = "global"
    if dfs == "global-nopack":
        monkeypatch.setenv("SDNROUTE_DFS_PACKED", "0")
        dfs = "global"
    if dfs == "global-nosplit":                  # single-wave lane-packed kernel
        monkeypatch.setenv("SDNROUTE_DFS_SPLIT", "0")
        dfs = "global"
    if dfs == "global-cumap":                    # split kernel, sources by CU chunk
        monkeypatch.setenv("SDNROUTE_DFS_CUMAP", "1")
        dfs = "global"
    if dfs == "global-nodict":                   # split kernel on ELL rows, not dictionary rows
        monkeypatch.setenv("SDNROUTE_DFS_DICT", "0")
        dfs = "global"
    if dfs:
        monkeypatch.setenv("SDNROUTE_DFS_STRATEGY", dfs)
    if ell is not None:
        monkeypatch.setenv("SDNROUTE_ELL", "1" if ell else "0")


def _check_dfs(ctx, csr, srcs, hops=True):
    ctx.upload(csr)
    p, t, h = ctx.dfs_tables(srcs, with_hops=hops)
    po, to, ho = O.dfs_tables(csr, srcs, with_hops=hops, nthreads=NTHREADS)
    np.testing.assert_array_equal(p, po)
    np.testing.assert_array_equal(t, to)
    if hops:
        np.testing.assert_array_equal(h, ho)
    return p, t


def _check_pairs(g, fabric, p, t, srcs):
    csr = fabric.csr()
    hv, hp = fabric.host_table()
    row = {int(s): i for i, s in enumerate(srcs)}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        r = row[int(hv[a])]
        got = O.tree_fdb(csr, p[r], t[r], int(hv[a]), int(hv[b]), hp[b])
        assert got == g.fdb(i), (g.name, i)


@pytest.mark.parametrize("strategy", ["auto", "async", "count", "coop", "lds", "global",
                                      "global-ring128", "global-nopack", "global-nosplit",
                                      "global-cumap", "global-nodict"])
@pytest.mark.parametrize("ell", [True, False])
@pytest.mark.parametrize("name", G.SMALL)
def test_dfs_small_all_sources(ctx, monkeypatch, name, strategy, ell):
    _strategy(monkeypatch, None if strategy == "auto" else strategy, ell)
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    p, t = _check_dfs(ctx, csr, srcs)
    _check_pairs(g, fabric, p, t, srcs)


@pytest.mark.parametrize("layout", ["int32", "hops", "packed", "slots"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "jellyfish_n60_r5", "torus_5x3x2", "torus_4x4x4"])
def test_dfs_dict_rows_small(ctx, monkeypatch, name, layout):
    """The split kernel on dictionary rows (row u = u + D[p(u)] from LDS,
    csrc/capi.hip upload_dict): every small fabric whose rows
    have <= 8 slots takes it under the split strategy, in every table layout,
    bit-exact vs the oracle."""
    _strategy(monkeypatch, "global")
    csr = G.Golden(name).fabric().csr()
    if csr.max_degree() > 8:
        pytest.skip("rows wider than 8 slots: no dictionary rows")
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    po, to, ho = O.dfs_tables(csr, srcs, with_hops=True, nthreads=NTHREADS)
    if layout in ("int32", "hops"):
        p, t, h = ctx.dfs_tables(srcs, with_hops=layout == "hops")
        np.testing.assert_array_equal(p, po)
        np.testing.assert_array_equal(t, to)
        if layout == "hops":
            np.testing.assert_array_equal(h, ho)
    elif layout == "packed":
        np.testing.assert_array_equal(ctx.dfs_tables_packed(srcs), _pack(po, to))
    else:
        np.testing.assert_array_equal(ctx.dfs_tables_slots(srcs), _expected_slots(csr, po))
    assert ctx.last_kernel().startswith("dfs_split_kernel<dict"), ctx.last_kernel()


def test_dfs_dict_rows_fallback(ctx, monkeypatch):
    """An irregular fabric with more than 255 distinct row tuples (a random
    4-regular graph on 600 switches) keeps the ELL rows; the forced-off
    dictionary (SDNROUTE_DFS_DICT=0) does too; both bit-exact."""
    _strategy(monkeypatch, "global")
    csr = T.jellyfish(600, 4, seed=3).csr()
    srcs = np.arange(0, csr.V, 7, dtype=np.int32)
    p, t = _check_dfs(ctx, csr, srcs)
    assert ctx.last_kernel() == "dfs_split_kernel<row16>", ctx.last_kernel()
    monkeypatch.setenv("SDNROUTE_DFS_DICT", "0")
    csr = G.Golden("torus_4x4x4").fabric().csr()
    _check_dfs(ctx, csr, np.arange(csr.V, dtype=np.int32))
    assert ctx.last_kernel() == "dfs_split_kernel<row16>", ctx.last_kernel()


def _pack(p, t):
    return ((p.astype(np.int64) & 0xFFFF) | ((t.astype(np.int64) & 0xFFFF) << 16)).astype(np.uint32)


@pytest.mark.parametrize("strategy", ["auto", "lds", "global", "global-nosplit"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "jellyfish_n60_r5", "torus_5x3x2"])
def test_dfs_packed_small(ctx, monkeypatch, name, strategy):
    _strategy(monkeypatch, None if strategy == "auto" else strategy)
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))
    p, t = _native.unpack_tree(tree)
    np.testing.assert_array_equal(p, po)
    np.testing.assert_array_equal(t, to)


def _expected_slots(csr, po):
    """Slot-tree words from oracle parents: parent | slot << 26, slot = the
    child's position in the parent's ascending CSR row, 63 for the root."""
    S, V = po.shape
    want = np.full((S, V), 0xFFFFFFFF, np.uint64)
    for i in range(S):
        for v in range(V):
            p = int(po[i, v])
            if p < 0:
                continue
            if p == v:
                want[i, v] = p | (63 << 26)
            else:
                row = csr.col[csr.row_ptr[p]:csr.row_ptr[p + 1]]
                want[i, v] = p | (int(np.searchsorted(row, v)) << 26)
    return want.astype(np.uint32)


@pytest.mark.parametrize("strategy", ["auto", "async", "lds", "global", "global-nosplit",
                                      "global-cumap"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "jellyfish_n60_r5", "torus_5x3x2", "random_V60_dense"])
def test_dfs_slots_small(ctx, monkeypatch, name, strategy):
    _strategy(monkeypatch, None if strategy == "auto" else strategy)
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    tree = ctx.dfs_tables_slots(srcs)
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _expected_slots(csr, po))
    p, t = _native.unpack_slots(tree, csr)
    np.testing.assert_array_equal(p, po)
    np.testing.assert_array_equal(t, to)


def _check_tree_depth(csr, srcs, tree, depth, layout, depth_bytes):
    po, to, ho = O.dfs_tables(csr, srcs, nthreads=NTHREADS)
    want = _pack(po, to) if layout == _native.TREE_PORT16 else _expected_slots(csr, po)
    np.testing.assert_array_equal(tree, want)
    if depth_bytes == 2:
        np.testing.assert_array_equal(depth, ho.astype(np.uint16))   # -1 -> 0xFFFF
    else:
        np.testing.assert_array_equal(depth, ho)


@pytest.mark.parametrize("strategy", ["auto", "async", "lds", "global", "global-nosplit"])
@pytest.mark.parametrize("layout", ["port16", "slot"])
@pytest.mark.parametrize("depth_bytes", [2, 4])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "jellyfish_n60_r5", "torus_5x3x2"])
def test_dfs_tree_depth_small(ctx, monkeypatch, name, layout, depth_bytes, strategy):
    """sdnr_dfs_tables_tree: 4-byte tree words + depths straight from every
    DFS strategy (the drop-in's pool rows), bit-exact vs the oracle."""
    _strategy(monkeypatch, None if strategy == "auto" else strategy)
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    lay = _native.TREE_PORT16 if layout == "port16" else _native.TREE_SLOT
    tree, depth = ctx.dfs_tables_tree(srcs, lay, depth_bytes)
    _check_tree_depth(csr, srcs, tree, depth, lay, depth_bytes)


@pytest.mark.parametrize("nsrc", [1, 144, 1152])
def test_dfs_tree_depth_k48(ctx, nsrc):
    """The drop-in's fill on k=48 runs the benched async kernel with hop
    counts (u16 depth plane), no int32 intermediate."""
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)[:nsrc]
    ctx.upload(csr)
    tree, depth = ctx.dfs_tables_tree(srcs, _native.TREE_PORT16, 2)
    assert ctx.last_kernel().startswith("dfs_async_kernel<") and \
        ctx.last_kernel().endswith(",packed,hops>")
    _check_tree_depth(csr, srcs, tree, depth, _native.TREE_PORT16, 2)


def test_dfs_packed_fullsize_k48(ctx, monkeypatch):
    _strategy(monkeypatch, "async")
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    assert ctx.last_kernel() == "dfs_async_kernel<4,packed>"
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


@pytest.mark.parametrize("nsrc", [1, 144, 512, 513])
def test_dfs_packed_k48_worker_count(ctx, monkeypatch, nsrc):
    """At most 2 sources per CU (one GPU's share of a multi-GPU step): the
    async kernel runs 7 decrement workers per source on dword-paired in-rows
    instead of 3 on u16 rows (dfs_async_waves; k=48 in-degree 48 > 32); the
    tables stay bit-exact."""
    import torch
    _strategy(monkeypatch, "async")
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)[:nsrc]
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert ctx.last_kernel() == "dfs_async_kernel<%d,packed>" % (8 if nsrc <= 2 * cus else 4)
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


@pytest.mark.parametrize("spec", ["0", "1"])
@pytest.mark.parametrize("nsrc", [1, 144, 1152])
@pytest.mark.parametrize("name", ["fat_tree_k48", "dragonfly_a16_h8_p8"])
def test_dfs_async_speculative_pop(ctx, monkeypatch, name, nsrc, spec):
    """The async kernel with the next stack candidate (window, counts, row)
    read before the push whenever every fresh child is a leaf
    (SDNROUTE_DFS_SPECPOP), and without: packed trees bit-exact vs the
    oracle at 1, 144 and 1,152 sources (every worker regime)."""
    monkeypatch.setenv("SDNROUTE_DFS_SPECPOP", spec)
    fabric = T.fat_tree(48) if name == "fat_tree_k48" else T.dragonfly(16, 8, 8)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)[:nsrc]
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    assert ctx.last_kernel().startswith("dfs_async_kernel<")
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


@pytest.mark.parametrize("spec", ["default", "1"])
@pytest.mark.parametrize("c16", ["0", "1", "0plain", "1plain"])
@pytest.mark.parametrize("layout", ["int32", "hops"])
@pytest.mark.parametrize("name", G.SMALL)
def test_dfs_async_compact_lds(ctx, monkeypatch, name, layout, c16, spec):
    """dfs_async_kernel with the compact LDS layout (u16 counts in pairs, u16
    parents + u8 slots; the dragonfly default) and without -- with the
    workers' pre-swizzled in-rows (the default) or the plain ones -- every
    source."""
    _strategy(monkeypatch, "async")
    if spec != "default":
        monkeypatch.setenv("SDNROUTE_DFS_SPECPOP", spec)
    monkeypatch.setenv("SDNROUTE_DFS_C16", c16[0])
    if c16.endswith("plain"):
        monkeypatch.setenv("SDNROUTE_DFS_PRESWZ", "0")
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    _check_dfs(ctx, csr, srcs, hops=layout == "hops")


def test_dfs_dragonfly_one_residency_round(ctx):
    """Dragonfly a16 h8: all 2,064 sources at once with the compact layout
    (the default there), bit-exact packed trees."""
    fabric = T.dragonfly(16, 8, 8)
    csr = fabric.csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


@pytest.mark.parametrize("c16", ["0", "1"])
@pytest.mark.parametrize("waves", [2, 3, 4, 5, 6, 8])
@pytest.mark.parametrize("name", ["fat_tree_k8", "jellyfish_n60_r5", "torus_5x3x2"])
def test_dfs_packed_async_waves(ctx, monkeypatch, name, waves, c16):
    _strategy(monkeypatch, "async")
    monkeypatch.setenv("SDNROUTE_DFS_C16", c16)
    monkeypatch.setenv("SDNROUTE_DFS_ASYNC_WAVES", str(waves))
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    assert ctx.last_kernel() == f"dfs_async_kernel<{waves},packed>"
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


def test_dfs_packed_rejects_wide_ports(ctx):
    from sdnmpi_amd.topologies import CSR
    c = CSR(np.array([1, 2]), np.array([0, 1, 2]), np.array([1, 0]), np.array([0xFFFF, 3]))
    ctx.upload(c)
    with pytest.raises(_native.SdnrError) as ei:
        ctx.dfs_tables_packed(np.array([0], np.int32))
    assert ei.value.code == -22
    p, t, _ = ctx.dfs_tables(np.array([0], np.int32))      # int32 layout still works
    assert t[0, 1] == 0xFFFF


def test_dfs_without_hops_and_repeated_sources(ctx):
    csr = T.fat_tree(8).csr()
    srcs = np.array([5, 5, 0, csr.V - 1, 17, 5], np.int32)
    _check_dfs(ctx, csr, srcs, hops=False)


@pytest.mark.parametrize("name", ["fat_tree_k48_sample", "dragonfly_a16_h8_p8_sample"])
def test_dfs_fullsize_all_host_sources(ctx, name):
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    p, t = _check_dfs(ctx, csr, srcs)
    _check_pairs(g, fabric, p, t, srcs)


# "1" is the default (CU-chunked sources, NS by shape: 7 on the torus, 5 on
# the Jellyfish; 8-entry windows); the others force each non-default shape
@pytest.mark.parametrize("split", ["1", "0", "ns3", "ns11-ring256", "cumap0", "j4"])
@pytest.mark.parametrize("name,nsample", [("torus_32x32x32_sample", 384),
                                          ("jellyfish_n100000_r16_sample", 48)])
def test_dfs_fullsize_sampled_sources(ctx, monkeypatch, name, nsample, split):
    if split.startswith("cumap"):                # sources by CU chunk or strided
        monkeypatch.setenv("SDNROUTE_DFS_CUMAP", split[-1])
    elif split.startswith("j"):                  # stack entries per window (rows of 9-16 slots)
        monkeypatch.setenv("SDNROUTE_DFS_SPLIT_J", split[1:])
    elif split.startswith("ns"):                 # search waves per workgroup
        ns, _, ring = split[2:].partition("-ring")
        monkeypatch.setenv("SDNROUTE_DFS_SPLIT_NS", ns)
        if ring:
            monkeypatch.setenv("SDNROUTE_DFS_SPLIT_RING", ring)
    else:
        monkeypatch.setenv("SDNROUTE_DFS_SPLIT", split)
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    hv, _ = fabric.host_table()
    spread = np.linspace(0, csr.V - 1, nsample).astype(np.int32)
    srcs = np.unique(np.concatenate([spread, hv[g.pair_src]])).astype(np.int32)
    p, t = _check_dfs(ctx, csr, srcs, hops=False)
    _check_pairs(g, fabric, p, t, srcs)


def test_dfs_fullsize_tree_properties(ctx):
    """Size-independent checks on the complete k=48 table: every reachable
    vertex's parent chain ends at the source, hop counts are parent + 1,
    ports are real ports of the parent's row."""
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    p, t, h = ctx.dfs_tables(srcs)
    V = csr.V
    assert (p >= 0).all()                       # fat-tree is connected
    r = np.arange(V)
    assert (p[srcs, srcs] == srcs).all() and (h[srcs, srcs] == 0).all()
    nonroot = p != r[None, :].repeat(len(srcs), 0)
    nonroot[srcs, srcs] = False
    hp = np.take_along_axis(h, p.astype(np.int64), 1)
    assert (h[nonroot] == hp[nonroot] + 1).all()
    # (parent, child) is a link and the port matches the CSR
    rows = csr.row_ptr
    for s in (0, 1, 777, V - 1):
        for v in range(V):
            if v == s:
                continue
            u = p[s, v]
            lo, hi = rows[u], rows[u + 1]
            k = lo + np.searchsorted(csr.col[lo:hi], v)
            assert k < hi and csr.col[k] == v and csr.port[k] == t[s, v]


@pytest.mark.parametrize("strategy", ["auto", "msbfs", "lanes", "lanes-csr", "plane",
                                      "plane-opt0", "plane-opt2", "apsp", "apsp-csr"])
@pytest.mark.parametrize("name", G.SMALL)
def test_shortest_small_all_destinations(ctx, monkeypatch, name, strategy):
    if strategy == "apsp-csr":                   # next hops from CSR rows (no ELL copy)
        monkeypatch.setenv("SDNROUTE_ELL", "0")
        strategy = "apsp"
    if strategy == "lanes-csr":                  # no ELL copy: 64-wide rows + CSR ports
        monkeypatch.setenv("SDNROUTE_ELL", "0")
        strategy = "lanes"
    if strategy.startswith("plane-opt"):         # plane updates: read-modify-write / atomic OR
        monkeypatch.setenv("SDNROUTE_PLANE_OPT", strategy[-1])
        strategy = "plane"
    if strategy != "auto":
        monkeypatch.setenv("SDNROUTE_SP_STRATEGY", strategy)
    fabric = G.Golden(name).fabric()
    csr = fabric.csr()
    dsts = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("dsts", ["all", "hosts", "mixed"])
@pytest.mark.parametrize("fab", ["fat_tree:48", "dragonfly:16,8,8", "fat_tree:8"])
def test_shortest_tables_from_apsp(ctx, monkeypatch, fab, dsts):
    """route_tables('shortest') through the APSP distances + next-hop
    extraction (SDNROUTE_SP_STRATEGY=apsp) equals the oracle's BFS tables:
    every vertex as a destination, the host switches, and a mixed list with
    repeats and an unknown id (device path)."""
    import torch
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "apsp")
    fabric = T.by_name(fab)
    csr = fabric.csr()
    V = csr.V
    if dsts == "all":
        d = np.arange(V, dtype=np.int32)
    elif dsts == "hosts":
        d = np.unique(fabric.host_table()[0]).astype(np.int32)
    else:
        d = np.array([3, V - 1, 3, -1, 0, V // 2], np.int32)
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    td = torch.from_numpy(d).to(dev)
    dist = torch.empty((len(d), V), dtype=torch.int16, device=dev)
    nh = torch.empty((len(d), V), dtype=torch.int32, device=dev)
    nhp = torch.empty_like(nh)
    ctx.shortest_tables_device(td.data_ptr(), len(d), dist.data_ptr(), nh.data_ptr(),
                               nhp.data_ptr())
    ctx.synchronize()
    assert ctx.last_kernel() == "apsp+sp_from_apsp_kernel"
    dist = dist.cpu().numpy().view(np.uint16)
    nh, nhp = nh.cpu().numpy(), nhp.cpu().numpy()
    ok = (d >= 0) & (d < V)
    do, nho, nhpo = O.dest_tables(csr, d[ok], nthreads=NTHREADS)
    np.testing.assert_array_equal(dist[ok], do)
    np.testing.assert_array_equal(nh[ok], nho)
    np.testing.assert_array_equal(nhp[ok], nhpo)
    assert (dist[~ok] == 0xFFFF).all() and (nh[~ok] == -1).all()


@pytest.mark.parametrize("name", G.MULTI)
def test_shortest_matches_reference_multiple(ctx, name):
    from sdnmpi_amd.engine import shortest_paths_lex
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    hv, hp = fabric.host_table()
    dsts = np.unique(hv).astype(np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    row = {int(d): i for i, d in enumerate(dsts)}
    for i in range(len(g)):
        a, b = int(g.pair_src[i]), int(g.pair_dst[i])
        s, d = int(hv[a]), int(hv[b])
        seqs = shortest_paths_lex(csr.row_ptr, csr.col, dist[row[d]], s, d)
        want = g.multi(i)
        assert len(seqs) == len(want)
        for q, w in zip(seqs, want):
            assert [int(csr.dpids[x]) for x in q] == [x for x, _ in w]


@pytest.mark.parametrize("strategy", ["auto", "dest", "msbfs", "opt0"])
def test_shortest_fullsize_fat_tree(ctx, monkeypatch, strategy):
    """k=48: rows of 48 slots -- the bit-plane BFS with 6 slot planes (auto:
    plane updates by atomic OR; opt0: by read-modify-write), the
    per-destination BFS and the level + next-hop kernels."""
    if strategy == "opt0":
        monkeypatch.setenv("SDNROUTE_PLANE_OPT", "0")
        strategy = "auto"
    if strategy != "auto":
        monkeypatch.setenv("SDNROUTE_SP_STRATEGY", strategy)
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    dsts = np.unique(fabric.host_table()[0]).astype(np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    if strategy != "msbfs":
        assert ctx.last_kernel().startswith({"auto": "msbfs_plane_level_kernel",
                                             "dest": "bfs_dest_kernel"}[strategy])
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("guess", ["default", "0"])
def test_shortest_plane_depth_cache(ctx, monkeypatch, guess):
    """The bit-plane BFS queues as many levels as the previous call on the
    graph needed before its first host check (SDNROUTE_PLANE_GUESS=0: a
    check every 8 levels).  Calls whose destinations need fewer, then more
    levels than the cached depth, on one context, against the oracle; and a
    repeated k=48 call launches only the levels it needs (4: every (batch,
    vertex) word is complete after level 4, so no empty fifth level runs)."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    if guess == "0":
        monkeypatch.setenv("SDNROUTE_PLANE_GUESS", "0")
    csr = T.torus3d(40, 3, 1).csr()                 # eccentricity 21 from every vertex
    ctx.upload(csr)
    for dsts in (np.arange(0, csr.V, 5), np.arange(3), np.arange(csr.V)[::-1], np.arange(70)):
        dsts = dsts.astype(np.int32)
        dist, nh, nhp = ctx.shortest_tables(dsts)
        do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
        np.testing.assert_array_equal(dist, do)
        np.testing.assert_array_equal(nh, nho)
        np.testing.assert_array_equal(nhp, nhpo)
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    dsts = np.unique(fabric.host_table()[0]).astype(np.int32)
    ctx.upload(csr)
    ctx.shortest_tables(dsts)
    first = ctx.last_launches()
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert ctx.last_launches() == (first if guess == "0" else 4)
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)


@pytest.mark.parametrize("pad", ["0", "1", "64", "1000"])
@pytest.mark.parametrize("name", ["fat_tree_k8", "torus_5x3x2"])
def test_shortest_plane_stride_pad(ctx, monkeypatch, name, pad):
    """The bit-plane BFS with plane strides V + pad (SDNROUTE_PLANE_PAD; 64 is
    the default), two chunks of batches so the batch stride is
    exercised too: tables independent of the pad."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    monkeypatch.setenv("SDNROUTE_PLANE_PAD", pad)
    monkeypatch.setenv("SDNROUTE_PLANE_CHUNK", "1")
    csr = G.Golden(name).fabric().csr()
    dsts = np.concatenate([np.arange(csr.V), np.arange(csr.V)[::-1]]).astype(np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert ctx.last_kernel().startswith("msbfs_plane_level_kernel")
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("dp", ["auto", "8"])
def test_shortest_plane_compact_levels(ctx, monkeypatch, dp):
    """Compact level planes (3 instead of 8) when the previous call on the
    graph ended by level 7, and the redo with 8 when a call then runs
    deeper: random_V40, whose destinations' eccentricities run 4..13 (some
    pairs unreachable), with shallow and deep destination sets in turn on one
    context, against the oracle (SDNROUTE_PLANE_DP=8: always 8 planes)."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    if dp != "auto":
        monkeypatch.setenv("SDNROUTE_PLANE_DP", dp)
    csr = G.Golden("random_V40").fabric().csr()
    ctx.upload(csr)
    for dsts in ([1, 6, 11, 12], [14, 7], [1, 6, 11, 12], [1, 6, 11, 12], [3, 25, 5],
                 [13, 39], list(range(csr.V))):
        dsts = np.asarray(dsts, np.int32)
        dist, nh, nhp = ctx.shortest_tables(dsts)
        do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
        np.testing.assert_array_equal(dist, do)
        np.testing.assert_array_equal(nh, nho)
        np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("init", ["init", "nofuse", "seed"])
@pytest.mark.parametrize("dp", ["auto", "8"])
def test_shortest_plane_repeated_destinations(ctx, monkeypatch, dp, init):
    """Batches whose destinations are all one vertex ([5, 5], a full batch of
    one id) or hold repeats and unknown ids, in compact and 8-plane mode,
    with the one-launch init and the old fill + seed path: the complete-word
    count must see the words complete from the start, and every
    table stays bit-exact vs the oracle."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    if dp != "auto":
        monkeypatch.setenv("SDNROUTE_PLANE_DP", dp)
    if init == "seed":
        monkeypatch.setenv("SDNROUTE_PLANE_INIT", "0")
    if init == "nofuse":
        monkeypatch.setenv("SDNROUTE_PLANE_FUSE1", "0")
    import torch
    csr = T.fat_tree(8).csr()
    ctx.upload(csr)
    V = csr.V
    dev = torch.device("cuda", 0)
    for dsts in ([5, 5], [7] * 64, [7] * 64 + [9] * 64 + [3], [3, 3, -1, 3],
                 list(range(V)) + [11] * 70, [0, V + 5], [2, 2, 2, 2]):
        dsts = np.asarray(dsts, np.int32)
        n = dsts.shape[0]
        td = torch.from_numpy(dsts).to(dev)       # device path: unknown ids give blank rows
        dist = torch.zeros((n, V), dtype=torch.int16, device=dev)
        nh = torch.zeros((n, V), dtype=torch.int32, device=dev)
        nhp = torch.zeros_like(nh)
        torch.cuda.synchronize(dev)      # torch's fills run on torch's stream
        ctx.shortest_tables_device(td.data_ptr(), n, dist.data_ptr(), nh.data_ptr(),
                                   nhp.data_ptr())
        ctx.synchronize()
        dist = dist.cpu().numpy().view(np.uint16)
        nh, nhp = nh.cpu().numpy(), nhp.cpu().numpy()
        ok = (dsts >= 0) & (dsts < V)
        do, nho, nhpo = O.dest_tables(csr, dsts[ok], nthreads=NTHREADS)
        np.testing.assert_array_equal(dist[ok], do)
        np.testing.assert_array_equal(nh[ok], nho)
        np.testing.assert_array_equal(nhp[ok], nhpo)
        assert (dist[~ok] == 0xFFFF).all() and (nh[~ok] == -1).all()


@pytest.mark.parametrize("fuse", ["1", "0"])
@pytest.mark.parametrize("fabric", ["fat_tree:8", "dragonfly:4,2,2", "torus:4,4,4"])
def test_shortest_plane_level1_fold(ctx, monkeypatch, fabric, fuse):
    """Level 1 folded into the plane init (msbfs_plane_init1_kernel): batches
    that are ascending id runs take the index test, others (shuffled,
    descending, strided, a run with a gap, a short last batch) the 64-lane
    match; both, and the separate level-1 launch, bit-exact vs the oracle."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    monkeypatch.setenv("SDNROUTE_PLANE_FUSE1", fuse)
    csr = T.by_name(fabric).csr()
    ctx.upload(csr)
    V = csr.V
    rng = np.random.default_rng(7)
    runs = np.arange(V, dtype=np.int32)
    for dsts in (runs, rng.permutation(V).astype(np.int32), runs[::-1].copy(),
                 runs[::3].copy(), np.r_[runs[:10], runs[12:80]].astype(np.int32),
                 runs[V // 2:V // 2 + 5].copy(), np.asarray([V - 1], np.int32)):
        for _ in range(2):                     # the second call runs on the cached depth
            dist, nh, nhp = ctx.shortest_tables(dsts)
            assert ctx.last_kernel().startswith("msbfs_plane_level_kernel")
            do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
            np.testing.assert_array_equal(dist, do)
            np.testing.assert_array_equal(nh, nho)
            np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("strategy", ["auto", "msbfs", "plane", "lanes"])
def test_shortest_fullsize_torus_sample(ctx, monkeypatch, strategy):
    """torus 32^3 (the BASELINE multi-source BFS config), spread destinations:
    the lane-packed per-destination BFS and the 64-destination bitset BFS."""
    if strategy != "auto":
        monkeypatch.setenv("SDNROUTE_SP_STRATEGY", strategy)
    fabric = T.torus3d(32, 32, 32)
    csr = fabric.csr()
    dsts = np.linspace(0, csr.V - 1, 96).astype(np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert ctx.last_kernel().startswith({"auto": "msbfs_plane_level_kernel",
                                         "lanes": "bfs_dest_lanes_kernel<8,sym>",
                                         "msbfs": "msbfs_level_kernel",
                                         "plane": "msbfs_plane_level_kernel"}[strategy])
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


def test_shortest_global_path_torus(ctx):
    """V > 6400 -> masks in HBM, one launch per level."""
    fabric = T.torus3d(24, 24, 16)
    csr = fabric.csr()
    dsts = np.linspace(0, csr.V - 1, 130).astype(np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("algo", ["squaring", "squaring-norelax", "sq128", "fw"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k8", "dragonfly_a4_h2_p2",
                                  "random_V60_dense", "torus_5x3x2", "random_V40", "random_V9"])
def test_apsp_small(ctx, monkeypatch, name, algo):
    if algo == "squaring-norelax":               # squaring passes only, no sweeps
        monkeypatch.setenv("SDNROUTE_APSP_RELAX", "0")
    elif algo != "squaring":
        monkeypatch.setenv("SDNROUTE_APSP", algo)
        monkeypatch.setenv("SDNROUTE_APSP_RELAX", "0")
    csr = G.Golden(name).fabric().csr()
    ctx.upload(csr)
    np.testing.assert_array_equal(ctx.apsp(), O.apsp(csr))


@pytest.mark.parametrize("strategy", ["auto", "dest"])
def test_shortest_dest_kernel_dragonfly_all_destinations(ctx, monkeypatch, strategy):
    if strategy == "dest":
        monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "dest")
    csr = T.dragonfly(16, 8, 8).csr()
    dsts = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert ctx.last_kernel().startswith("bfs_dest_kernel" if strategy == "dest"
                                        else "msbfs_plane_level_kernel")
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


def test_shortest_unknown_destination_rows_device(ctx):
    torch = pytest.importorskip("torch")
    csr = T.fat_tree(4).csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    td = torch.tensor([-1, 3, csr.V + 5], dtype=torch.int32, device=dev)
    dist = torch.zeros((3, csr.V), dtype=torch.int16, device=dev)
    nh = torch.zeros((3, csr.V), dtype=torch.int32, device=dev)
    nhp = torch.zeros_like(nh)
    torch.cuda.synchronize(dev)          # torch's fills run on torch's stream
    ctx.shortest_tables_device(td.data_ptr(), 3, dist.data_ptr(), nh.data_ptr(), nhp.data_ptr())
    ctx.synchronize()
    d = dist.cpu().numpy().view(np.uint16)
    assert (d[0] == 0xFFFF).all() and (d[2] == 0xFFFF).all() and d[1, 3] == 0
    assert (nh.cpu().numpy()[[0, 2]] == -1).all()


@pytest.mark.parametrize("name", ["random_V40", "random_V12", "random_V60_dense", "torus_5x3x2"])
def test_shortest_plane_incomplete_words(ctx, monkeypatch, name):
    """Plane BFS termination without completion: directed graphs with
    unreachable pairs (and a destination batch of one) keep some (batch,
    vertex) words incomplete, so the BFS ends on an empty level; repeated
    calls reuse the cached depth."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    csr = G.Golden(name).fabric().csr()
    ctx.upload(csr)
    for dsts in (np.arange(csr.V), np.arange(65) % csr.V, np.array([csr.V - 1]), np.arange(csr.V)):
        dsts = dsts.astype(np.int32)
        dist, nh, nhp = ctx.shortest_tables(dsts)
        do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
        np.testing.assert_array_equal(dist, do)
        np.testing.assert_array_equal(nh, nho)
        np.testing.assert_array_equal(nhp, nhpo)


@pytest.mark.parametrize("tiles", ["64", "64-norelax"])       # sq128: test_apsp_dragonfly
def test_apsp_fullsize_k48(ctx, monkeypatch, tiles):
    """k=48 (diameter 4): Bellman-Ford sweeps reach the fixpoint within the
    cap, no squaring pass at all; squaring alone takes 3 passes."""
    if tiles == "sq128":
        monkeypatch.setenv("SDNROUTE_APSP", "sq128")
    if tiles != "64":
        monkeypatch.setenv("SDNROUTE_APSP_RELAX", "0")
    csr = T.fat_tree(48).csr()
    ctx.upload(csr)
    D = ctx.apsp()
    if tiles == "64":
        assert ctx.last_kernel() == "apsp_relax8_kernel"
        assert ctx.last_launches() == 0 and 2 <= ctx.last_sweeps() <= 5
    else:
        assert ctx.last_kernel() == ("minplus_square_kernel" if tiles == "sq128"
                                     else "minplus_square64_kernel")
        assert ctx.last_launches() == 3 and ctx.last_sweeps() == 0
    np.testing.assert_array_equal(D, O.apsp(csr))


@pytest.mark.parametrize("tiles", ["64", "sq128", "64-norelax"])
def test_apsp_long_paths_torus(ctx, monkeypatch, tiles):
    """A high-diameter graph (ring-like torus 40x3x1, diameter 21): squaring
    alone takes many passes; with sweeps, the cap (5 here) runs out and
    squaring passes alternate with sweeps."""
    if tiles == "sq128":
        monkeypatch.setenv("SDNROUTE_APSP", "sq128")
    if tiles != "64":
        monkeypatch.setenv("SDNROUTE_APSP_RELAX", "0")
    csr = T.torus3d(40, 3, 1).csr()
    ctx.upload(csr)
    np.testing.assert_array_equal(ctx.apsp(), O.apsp(csr))
    if tiles == "64":
        assert ctx.last_launches() >= 1 and ctx.last_sweeps() >= 5


@pytest.mark.parametrize("tiles", ["64", "sq128"])
def test_apsp_dragonfly(ctx, monkeypatch, tiles):
    if tiles == "sq128":
        monkeypatch.setenv("SDNROUTE_APSP", "sq128")
        monkeypatch.setenv("SDNROUTE_APSP_RELAX", "0")
    csr = T.dragonfly(16, 8, 8).csr()
    ctx.upload(csr)
    np.testing.assert_array_equal(ctx.apsp(), O.apsp(csr))


def test_device_pointer_path_matches_host_path(ctx):
    torch = pytest.importorskip("torch")
    csr = T.fat_tree(16).csr()
    ctx.upload(csr)
    srcs = np.arange(csr.V, dtype=np.int32)
    p, t, h = ctx.dfs_tables(srcs)
    dev = torch.device("cuda", 0)
    ts = torch.from_numpy(srcs).to(dev)
    tp = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
    tt = torch.empty_like(tp)
    th = torch.empty_like(tp)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    ctx.dfs_tables_device(ts.data_ptr(), len(srcs), tp.data_ptr(), tt.data_ptr(),
                          th.data_ptr(), timing=True)
    ms = ctx.last_kernel_ms()
    torch.cuda.synchronize()
    ctx.set_stream(None)
    assert ms > 0
    np.testing.assert_array_equal(tp.cpu().numpy(), p)
    np.testing.assert_array_equal(tt.cpu().numpy(), t)
    np.testing.assert_array_equal(th.cpu().numpy(), h)


def test_out_of_range_source_rows_device(ctx):
    torch = pytest.importorskip("torch")
    csr = T.fat_tree(4).csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    ts = torch.tensor([-1, 3, csr.V + 5], dtype=torch.int32, device=dev)
    tp = torch.empty((3, csr.V), dtype=torch.int32, device=dev)
    tt = torch.empty_like(tp)
    ctx.dfs_tables_device(ts.data_ptr(), 3, tp.data_ptr(), tt.data_ptr())
    ctx.synchronize()
    p = tp.cpu().numpy()
    assert (p[0] == -1).all() and (p[2] == -1).all() and p[1, 3] == 3


def test_host_path_rejects_bad_source(ctx):
    ctx.upload(T.fat_tree(4).csr())
    with pytest.raises(_native.SdnrError) as ei:
        ctx.dfs_tables(np.array([0, 999], np.int32))
    assert ei.value.code == -22


def test_upload_rejects_unsorted_rows(ctx):
    from sdnmpi_amd.topologies import CSR
    bad = CSR(np.array([1, 2, 3]), np.array([0, 2, 2, 2]), np.array([2, 1]), np.array([1, 2]))
    with pytest.raises(_native.SdnrError):
        ctx.upload(bad)


def test_edge_graphs(ctx):
    from sdnmpi_amd.topologies import CSR
    # isolated vertices only
    c = CSR(np.array([4, 9]), np.array([0, 0, 0]), np.zeros(0, np.int32), np.zeros(0, np.int32))
    ctx.upload(c)
    p, t, h = ctx.dfs_tables(np.array([0, 1], np.int32))
    np.testing.assert_array_equal(p, [[0, -1], [-1, 1]])
    np.testing.assert_array_equal(h, [[0, -1], [-1, 0]])
    dist, nh, nhp = ctx.shortest_tables(np.array([1], np.int32))
    np.testing.assert_array_equal(dist, [[0xFFFF, 0]])
    # a star with 130 leaves: rows wider than one wavefront (CSR chunks)
    V = 131
    rp = np.zeros(V + 1, np.int64)
    rp[1] = V - 1
    rp[2:] = V - 1 + np.arange(1, V)
    col = np.concatenate([np.arange(1, V), np.zeros(V - 1, np.int64)])
    port = np.arange(len(col))
    star = CSR(np.arange(1, V + 1), rp, col, port)
    _check_dfs(ctx, star, np.arange(V, dtype=np.int32))


def test_new_paths_on_edge_graphs(ctx):
    """Isolated vertices, a one-way link and an unreachable destination
    through the route expansion, ECMP and APSP entry points."""
    from sdnmpi_amd.topologies import CSR
    # 0 -> 1 (port 5), 2 isolated
    c = CSR(np.array([3, 7, 9]), np.array([0, 1, 1, 1]), np.array([1]), np.array([5]))
    ctx.upload(c)
    p, t, h = ctx.dfs_tables(np.arange(3, dtype=np.int32))
    off, sw, hp = ctx.expand_routes(p, t, h, np.array([0, 0, 1, 2]), np.array([1, 2, 0, 2]),
                                    np.array([11, 12, 13, 14]))
    assert off.tolist() == [0, 2, 2, 2, 3]
    assert sw.tolist() == [0, 1, 2] and hp.tolist() == [5, 11, 14]
    dist, nh, nhp = ctx.shortest_tables(np.arange(3, dtype=np.int32))
    paths = ctx.ecmp_counts(dist)
    assert paths[1].tolist() == [1, 1, 0] and paths[2].tolist() == [0, 0, 1]
    r = ctx.ecmp_routes(dist, paths, np.array([1, 1, 0]), np.array([0, 2, 1]),
                        np.array([0, 0, 0], np.uint64), 3)
    assert r.tolist() == [[0, 1, -1], [-1, -1, -1], [-1, -1, -1]]
    np.testing.assert_array_equal(ctx.apsp(), O.apsp(c))


def test_ecmp_counts_dragonfly(ctx):
    csr = T.dragonfly(4, 2, 2).csr()
    ctx.upload(csr)
    dsts = np.arange(csr.V, dtype=np.int32)
    dist, _, _ = ctx.shortest_tables(dsts)
    do, _, _ = O.dest_tables(csr, dsts)
    np.testing.assert_array_equal(dist, do)
    paths = ctx.ecmp_counts(dist)
    for d in range(0, csr.V, 3):
        np.testing.assert_array_equal(paths[d], O.ecmp_counts(csr, do[d]))


@pytest.mark.parametrize("case", ["fat_tree:8", "random", "ladder", "star"])
def test_ecmp_counts_vs_level_dp(ctx, case):
    """ECMP counts against the oracle's DP: ecmp_count_rows_kernel (64-wide rows)
    including counts past 2**64 (a 70-rung ladder has 2**68 shortest routes
    end to end: saturated), and the CSR kernel on a star of degree 130 (no
    64-wide rows)."""
    from sdnmpi_amd.topologies import CSR
    if case == "fat_tree:8":
        csr = T.by_name("fat_tree:8").csr()
    elif case == "random":
        rng = np.random.default_rng(7)
        V = 300
        adj = [sorted(set(rng.choice(V, size=rng.integers(1, 9), replace=False).tolist()) - {u})
               for u in range(V)]
        rp = np.concatenate([[0], np.cumsum([len(a) for a in adj])])
        col = np.array([v for a in adj for v in a], np.int64)
        csr = CSR(np.arange(1, V + 1), rp, col, np.concatenate([np.arange(1, len(a) + 1) for a in adj]))
    elif case == "star":
        V = 131                                  # hub 0 joined to 1..130, leaves 1-2 linked
        nb = [list(range(1, V))] + [[0] for _ in range(1, V)]
        nb[1].append(2)
        nb[2].append(1)
        rp = np.concatenate([[0], np.cumsum([len(a) for a in nb])])
        col = np.array([v for a in nb for v in a], np.int64)
        csr = CSR(np.arange(1, V + 1), rp, col, np.concatenate([np.arange(1, len(a) + 1) for a in nb]))
    else:
        R = 70                                   # rungs: vertices 2i, 2i+1
        V = 2 * R
        nb = [[] for _ in range(V)]
        for i in range(R - 1):
            for a in (2 * i, 2 * i + 1):
                for b in (2 * i + 2, 2 * i + 3):
                    nb[a].append(b)
                    nb[b].append(a)
        nb = [sorted(x) for x in nb]
        rp = np.concatenate([[0], np.cumsum([len(a) for a in nb])])
        col = np.array([v for a in nb for v in a], np.int64)
        csr = CSR(np.arange(1, V + 1), rp, col, np.concatenate([np.arange(1, len(a) + 1) for a in nb]))
    ctx.upload(csr)
    dsts = np.arange(0, csr.V, 5 if case != "ladder" else 1, dtype=np.int32)
    dist, _, _ = ctx.shortest_tables(dsts)
    do, _, _ = O.dest_tables(csr, dsts)
    np.testing.assert_array_equal(dist, do)
    paths = ctx.ecmp_counts(dist)
    for i in range(0, len(dsts), 3 if case != "ladder" else 7):
        np.testing.assert_array_equal(paths[i], O.ecmp_counts(csr, do[i]))
    if case == "ladder":
        assert int(paths[0, csr.V - 1]) == 2**64 - 1



def test_shortest_plane_too_deep_falls_back(ctx, monkeypatch):
    """A ring of 700 switches (BFS depth 350 > the 255 levels the bit planes
    hold): the plane path hands over to the level + next-hop kernels."""
    monkeypatch.setenv("SDNROUTE_SP_STRATEGY", "plane")
    csr = T.torus3d(700, 1, 1).csr()
    dsts = np.arange(0, csr.V, 7, dtype=np.int32)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert not ctx.last_kernel().startswith("msbfs_plane")
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=NTHREADS)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)


def test_route_expand_packed_rejects_wide_last_port(ctx):
    """sdnr_route_expand_packed keeps a 16-bit port per u32 entry: a last
    (host) port above 0xFFFF, or negative, fails the call (the device sets
    the watchdog word; sdnr_synchronize reports EINVAL) instead of keeping
    its low bits -- ADVICE r4.  In-range ports expand as before."""
    import torch
    csr = T.fat_tree(4).csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    srcs = np.arange(csr.V, dtype=np.int32)
    par, prt, hop = O.dfs_tables(csr, srcs, nthreads=NTHREADS)
    tp, tt, th = (torch.from_numpy(a).to(dev) for a in (par, prt, hop))
    rows = torch.tensor([0, 1, 2], dtype=torch.int32, device=dev)
    dsts = torch.tensor([5, 6, 7], dtype=torch.int32, device=dev)
    off = torch.empty(4, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ctx.route_offsets_device(th.data_ptr(), rows.data_ptr(), dsts.data_ptr(), 3, off.data_ptr(),
                             nrows=csr.V)
    ctx.synchronize()
    ent = torch.zeros(int(off[-1].item()), dtype=torch.int32, device=dev)
    for bad, ok in (([1, 70000, 2], False), ([1, -1, 2], False), ([1, 0xFFFE, 2], True)):
        last = torch.tensor(bad, dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)      # torch's copies / fills run on torch's stream
        ctx.expand_routes_packed_device(tp.data_ptr(), tt.data_ptr(), csr.V, rows.data_ptr(),
                                        dsts.data_ptr(), last.data_ptr(), 3, off.data_ptr(),
                                        ent.data_ptr())
        if ok:
            ctx.synchronize()
            o = off.cpu().numpy()
            e = ent.cpu().numpy().view(np.uint32)
            assert e[o[2] - 1] == 6 | (0xFFFE << 16)
        else:
            with pytest.raises(_native.SdnrError) as ei:
                ctx.synchronize()
            assert ei.value.code == -22 and "last port" in str(ei.value)


@pytest.mark.parametrize("packed", [True, False])
def test_route_expand_same_tables(ctx, packed):
    """SDNR_SAME_TABLES: chunks of pairs over one set of tables reuse the
    walk tables the first chunk built; tables at other addresses, or the same
    addresses without the flag, are rebuilt.  Every chunk's entries equal the
    host path's (which always rebuilds)."""
    import torch
    csr = T.fat_tree(8).csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    srcs = np.arange(csr.V, dtype=np.int32)
    tabs = []
    for perm in (srcs, rng.permutation(srcs).astype(np.int32)):
        par, prt, hop = O.dfs_tables(csr, perm, nthreads=NTHREADS)
        tabs.append((par, prt, hop))

    def run(t_host, t_dev, same, n=5000):
        par, prt, hop = t_host
        rows = rng.integers(0, csr.V, n).astype(np.int32)
        dsts = rng.integers(0, csr.V, n).astype(np.int32)
        last = rng.integers(1, 200, n).astype(np.int32)
        off, sw, hp = ctx.expand_routes(par, prt, hop, rows, dsts, last)
        r, d, l = (torch.from_numpy(a).to(dev) for a in (rows, dsts, last))
        doff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)      # torch's copies / fills run on torch's stream
        ctx.route_offsets_device(t_dev[2].data_ptr(), r.data_ptr(), d.data_ptr(), n,
                                 doff.data_ptr(), nrows=csr.V)
        tot = int(off[-1])
        if packed:
            ent = torch.zeros(tot, dtype=torch.int32, device=dev)
            torch.cuda.synchronize(dev)
            ctx.expand_routes_packed_device(t_dev[0].data_ptr(), t_dev[1].data_ptr(), csr.V,
                                            r.data_ptr(), d.data_ptr(), l.data_ptr(), n,
                                            doff.data_ptr(), ent.data_ptr(), same_tables=same)
            ctx.synchronize()
            e = ent.cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(e & 0xFFFF, sw)
            np.testing.assert_array_equal(e >> 16, hp)
        else:
            dsw = torch.zeros(tot, dtype=torch.int32, device=dev)
            dhp = torch.zeros(tot, dtype=torch.int32, device=dev)
            torch.cuda.synchronize(dev)
            ctx.expand_routes_device(t_dev[0].data_ptr(), t_dev[1].data_ptr(), csr.V,
                                     r.data_ptr(), d.data_ptr(), l.data_ptr(), n,
                                     doff.data_ptr(), dsw.data_ptr(), dhp.data_ptr(),
                                     same_tables=same)
            ctx.synchronize()
            np.testing.assert_array_equal(dsw.cpu().numpy(), sw)
            np.testing.assert_array_equal(dhp.cpu().numpy(), hp)
        np.testing.assert_array_equal(doff.cpu().numpy(), off)

    da = [torch.from_numpy(a).to(dev) for a in tabs[0]]
    db = [torch.from_numpy(a).to(dev) for a in tabs[1]]
    run(tabs[0], da, False)
    for _ in range(3):
        run(tabs[0], da, True)                   # reused
    run(tabs[1], db, True)                       # other addresses: rebuilt
    run(tabs[1], db, True)
    for i in range(3):                           # same addresses, new contents, no flag
        da[i].copy_(db[i])
    torch.cuda.synchronize(dev)
    run(tabs[1], da, False)
    run(tabs[1], da, True)


@pytest.mark.parametrize("pipe", ["default", "0"])
def test_route_expand_k48_large_batch(ctx, monkeypatch, pipe):
    """A 4.3 M-pair batch on k=48 -- the all-pairs order of the materialised
    flows (runs of 24 hosts per destination switch, DFS routes of ~70
    entries) followed by random pairs and same-switch pairs: the u32 entries
    of the default large-batch kernel (route_seg_pipe_kernel, walker and
    storer waves), of another shape and of the one-role kernel
    (SDNROUTE_ROUTE_PIPE=0) equal the int32 switch / port arrays of
    route_seg_packed_kernel, and a sample of pairs equals the host path's
    entries."""
    import torch
    if pipe != "default":
        monkeypatch.setenv("SDNROUTE_ROUTE_PIPE", pipe)
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    hv, hp = fabric.host_table()
    srcs = np.unique(hv).astype(np.int32)
    H = len(hv)
    par, prt, hop = ctx.dfs_tables(srcs)
    tp, tt, th = (torch.from_numpy(a).to(dev) for a in (par, prt, hop))
    rng = np.random.default_rng(5)
    n_ord = (1 << 22) + 4321
    idx = np.arange(3 * H + 17, 3 * H + 17 + n_ord, dtype=np.int64)
    a = np.concatenate([idx // H, rng.integers(0, H, 200_000), np.full(500, 7)])
    b = np.concatenate([idx % H, rng.integers(0, H, 200_000), np.full(500, 7)])
    rows = np.searchsorted(srcs, hv[a]).astype(np.int32)
    dsts = hv[b].astype(np.int32)
    last = hp[b].astype(np.int32)
    n = len(rows)
    r, d, l = (torch.from_numpy(x).to(dev) for x in (rows, dsts, last))
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ctx.route_offsets_device(th.data_ptr(), r.data_ptr(), d.data_ptr(), n, off.data_ptr(),
                             nrows=len(srcs))
    ctx.synchronize()
    tot = int(off[-1].item())
    ent = torch.zeros(tot, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)          # torch's fill runs on its own stream, not the context's
    ctx.expand_routes_packed_device(tp.data_ptr(), tt.data_ptr(), len(srcs), r.data_ptr(),
                                    d.data_ptr(), l.data_ptr(), n, off.data_ptr(), ent.data_ptr())
    ctx.synchronize()
    assert ctx.last_kernel() == ("route_seg_packed_kernel<1024,u32>" if pipe == "0"
                                 else "route_seg_pipe_kernel<u32>")
    sw = torch.zeros(tot, dtype=torch.int32, device=dev)
    pt = torch.zeros(tot, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    monkeypatch.delenv("SDNROUTE_ROUTE_PIPE", raising=False)   # the int32 one-role kernel
    ctx.expand_routes_device(tp.data_ptr(), tt.data_ptr(), len(srcs), r.data_ptr(), d.data_ptr(),
                             l.data_ptr(), n, off.data_ptr(), sw.data_ptr(), pt.data_ptr())
    ctx.synchronize()
    assert ctx.last_kernel() == "route_seg_packed_kernel<1024>"
    e = ent.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(e & 0xFFFF, sw.cpu().numpy())
    np.testing.assert_array_equal(e >> 16, pt.cpu().numpy())
    o = off.cpu().numpy()
    pick = np.concatenate([rng.integers(0, n, 3000), [0, n - 1, n_ord - 1, n_ord]])
    so, ssw, shp = ctx.expand_routes(par, prt, hop, rows[pick], dsts[pick], last[pick])
    for j, i in enumerate(pick):
        np.testing.assert_array_equal(e[o[i]:o[i + 1]] & 0xFFFF, ssw[so[j]:so[j + 1]])
        np.testing.assert_array_equal(e[o[i]:o[i + 1]] >> 16, shp[so[j]:so[j + 1]])


@pytest.mark.parametrize("fab", ["fat_tree:48", "torus:16,16,16"])
def test_route_expand_pipe_edges(ctx, monkeypatch, fab):
    """route_seg_pipe_kernel (walker / storer waves, line-aligned store
    heads) on a request stream that puts every kind of pair next to slot and
    group boundaries -- runs of one route, stretches of same-switch pairs (one
    entry each), pairs with no entries (row -1), random pairs and, on the
    torus, DFS routes longer than a slot (the direct walk) -- written at
    several phases of the entry array against the 128-B lines, by three
    walker / storer shapes.  The u32 entries equal the int32 one-role
    kernel's, and nothing outside the output range is written.  (Also the
    parity test of the line-owned slots measured in round 6,
    tools/diag/flows_line_owned.patch.)"""
    import torch
    fabric = T.by_name(fab)
    csr = fabric.csr()
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    hv, hp = fabric.host_table()
    srcs = np.unique(hv).astype(np.int32)
    H = len(hv)
    order = np.argsort(hv, kind="stable")        # hosts grouped by switch
    par, prt, hop = ctx.dfs_tables(srcs)
    tp, tt, th = (torch.from_numpy(x).to(dev) for x in (par, prt, hop))
    rng = np.random.default_rng(13)
    A, B, R = [], [], []
    for _ in range(600):
        kind = int(rng.integers(0, 6))
        if kind in (0, 5):                       # a run: one source, hosts of few switches
            cnt = int(rng.integers(1, 60 if kind == 0 else 300))
            b0 = int(rng.integers(0, H))
            a = np.full(cnt, rng.integers(0, H))
            b = order[(b0 + np.arange(cnt)) % H]
        elif kind == 1:                          # same-switch pairs: one entry each
            cnt = int(rng.integers(1, 45))
            a = rng.integers(0, H, cnt)
            b = a.copy()
        elif kind == 2:                          # random pairs
            cnt = int(rng.integers(1, 30))
            a, b = rng.integers(0, H, cnt), rng.integers(0, H, cnt)
        else:                                    # no entries (unknown row)
            cnt = int(rng.integers(1, 20))
            a, b = rng.integers(0, H, cnt), rng.integers(0, H, cnt)
        A.append(a)
        B.append(b)
        R.append(np.full(cnt, kind == 3 or kind == 4))
    a, b, none = np.concatenate(A), np.concatenate(B), np.concatenate(R)
    rows = np.where(none, -1, np.searchsorted(srcs, hv[a])).astype(np.int32)
    dsts = hv[b].astype(np.int32)
    last = hp[b].astype(np.int32)
    n = len(rows)
    r, d, l = (torch.from_numpy(x).to(dev) for x in (rows, dsts, last))
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ctx.route_offsets_device(th.data_ptr(), r.data_ptr(), d.data_ptr(), n, off.data_ptr(),
                             nrows=len(srcs))
    ctx.synchronize()
    tot = int(off[-1].item())
    o = off.cpu().numpy()
    assert (np.diff(o) == 0).sum() >= 100 and (np.diff(o) == 1).sum() >= 100
    sw = torch.zeros(tot, dtype=torch.int32, device=dev)
    pt = torch.zeros(tot, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    monkeypatch.setenv("SDNROUTE_ROUTE_PIPE", "0")
    ctx.expand_routes_device(tp.data_ptr(), tt.data_ptr(), len(srcs), r.data_ptr(), d.data_ptr(),
                             l.data_ptr(), n, off.data_ptr(), sw.data_ptr(), pt.data_ptr())
    ctx.synchronize()
    assert ctx.last_kernel() == "route_seg_packed_kernel<1024>"
    want = (sw.cpu().numpy().astype(np.uint32) & 0xFFFF) | (pt.cpu().numpy().astype(np.uint32) << 16)
    for shape in ("2,2,4", "1,1,4", "8,4,2"):
        monkeypatch.setenv("SDNROUTE_ROUTE_PIPE", shape)
        for phase in (0, 1, 7, 13, 31, 37):      # entries past a 128-B boundary
            buf = torch.zeros(tot + 96, dtype=torch.int32, device=dev)
            assert buf.data_ptr() % 128 == 0
            torch.cuda.synchronize(dev)
            ctx.expand_routes_packed_device(tp.data_ptr(), tt.data_ptr(), len(srcs), r.data_ptr(),
                                            d.data_ptr(), l.data_ptr(), n, off.data_ptr(),
                                            buf[phase:].data_ptr())
            ctx.synchronize()
            assert ctx.last_kernel() == "route_seg_pipe_kernel<u32>"
            e = buf.cpu().numpy().view(np.uint32)
            np.testing.assert_array_equal(e[phase:phase + tot], want, err_msg="%s %d" % (shape, phase))
            assert not e[:phase].any() and not e[phase + tot:].any()


@pytest.mark.parametrize("scan", ["fused", "4"])
@pytest.mark.parametrize("npairs", [1, 8191, 8192, 8193, 3_000_000])
def test_route_offsets_scan(ctx, monkeypatch, scan, npairs):
    """sdnr_route_offsets: the one-pass look-back scan (default) and the
    four-kernel form give offsets[i] = sum of (hops + 1) of the pairs before
    i (0 for an unreachable pair or an unknown row / destination), on tile
    boundaries and over hundreds of tiles (look-back windows past 64)."""
    import torch
    if scan == "4":
        monkeypatch.setenv("SDNROUTE_ROUTE_SCAN", "4")
    csr = T.fat_tree(8).csr()
    ctx.upload(csr)
    V = csr.V
    srcs = np.arange(V, dtype=np.int32)
    _, _, hop = O.dfs_tables(csr, srcs, nthreads=NTHREADS)
    hop[3, 7] = -1                                # an unreachable pair
    rng = np.random.default_rng(npairs)
    rows = rng.integers(0, V, npairs).astype(np.int32)
    dsts = rng.integers(0, V, npairs).astype(np.int32)
    dsts[::97] = -1                               # unknown destinations
    rows[5::101] = -1                             # unknown rows
    ok = (rows >= 0) & (dsts >= 0)
    h = np.full(npairs, -1, np.int64)
    h[ok] = hop[rows[ok], dsts[ok]]
    lens = np.where(h < 0, 0, h + 1)
    want = np.concatenate([[0], np.cumsum(lens)])
    dev = torch.device("cuda", 0)
    th = torch.from_numpy(hop).to(dev)
    tr, td = torch.from_numpy(rows).to(dev), torch.from_numpy(dsts).to(dev)
    off = torch.full((npairs + 1,), -7, dtype=torch.int64, device=dev)
    ctx.route_offsets_device(th.data_ptr(), tr.data_ptr(), td.data_ptr(), npairs, off.data_ptr(),
                             nrows=V)
    ctx.synchronize()
    np.testing.assert_array_equal(off.cpu().numpy(), want)


def test_empty_batches(ctx):
    """Zero sources, destinations and pairs through every batch entry point:
    empty results and no error (the C ABI returns SDNR_OK and launches
    nothing; the offsets of zero pairs are [0])."""
    csr = T.fat_tree(8).csr()
    ctx.upload(csr)
    V = csr.V
    e = np.empty(0, np.int32)
    p, t, h = ctx.dfs_tables(e)
    assert p.shape == t.shape == h.shape == (0, V)
    assert ctx.dfs_tables_packed(e).shape == (0, V)
    assert ctx.dfs_tables_slots(e).shape == (0, V)
    d, nh, nhp = ctx.shortest_tables(e)
    assert d.shape == nh.shape == nhp.shape == (0, V)
    assert ctx.ecmp_counts(np.empty((0, V), np.uint16)).shape == (0, V)
    par, prt, hop = ctx.dfs_tables(np.array([0, 1], np.int32))
    off, sw, hp = ctx.expand_routes(par, prt, hop, e, e, e)
    assert off.tolist() == [0] and sw.size == 0 and hp.size == 0
    # and one source still computes afterwards
    np.testing.assert_array_equal(ctx.dfs_tables(np.array([1], np.int32))[0], par[1:2])
