"""Parity of the DIAGNOSTIC DFS variants (tools/diag/dfs_runs.hip,
dfs_bits.hip: measured slower than the shipped kernels, DESIGN.md 4.1a /
4.1b).  They are not in libsdnroute.so; build the diagnostic library with
tools/diag/build_diag.sh, then run on a GPU box:

    SDNROUTE_LIB=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_diag.so \
        python -m pytest tools/diag/test_diag_variants.py -x -q

Not part of tests/ (the driver's suites): these kernels are never selected
by the product."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "sdn-mpi-router_amd"), os.path.join(ROOT, "tests")]

import golden_util as G  # noqa: E402
from oracle import oracle as O  # noqa: E402
from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402
from test_gpu_parity import NTHREADS, _check_dfs, _check_pairs, _pack, _strategy  # noqa: E402

if "diag" not in os.path.basename(os.environ.get("SDNROUTE_LIB", "")):
    pytest.skip("needs SDNROUTE_LIB=<libsdnroute_diag.so> (tools/diag/build_diag.sh)",
                allow_module_level=True)


@pytest.fixture(scope="module")
def ctx():
    c = _native.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("waves", ["auto", "2", "3", "8"])
@pytest.mark.parametrize("name", ["mock", "fat_tree_k4", "fat_tree_k8", "dragonfly_a4_h2_p2",
                                  "random_V40", "random_V12", "random_V9", "jellyfish_n60_r5",
                                  "torus_5x3x2", "torus_4x4x4", "random_V60_dense"])
def test_dfs_bits_small(ctx, monkeypatch, name, waves):
    """dfs_bits_kernel (visited set in registers, bitmap rows, frame log):
    int32 tables with hops, packed trees, tree + u16 depth, all bit-exact vs
    the oracle on every vertex as a source -- directed graphs, sparse dpids,
    isolated switches included."""
    _strategy(monkeypatch, "bits")
    if waves != "auto":
        monkeypatch.setenv("SDNROUTE_DFS_BITS_WAVES", waves)
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    ctx.upload(csr)
    p, t, h = ctx.dfs_tables(srcs)
    assert ctx.last_kernel() == "dfs_bits_kernel<hops>"
    po, to, ho = O.dfs_tables(csr, srcs, nthreads=NTHREADS)
    np.testing.assert_array_equal(p, po)
    np.testing.assert_array_equal(t, to)
    np.testing.assert_array_equal(h, ho)
    if csr.E and int(csr.port.max()) < 0xFFFF:
        tree = ctx.dfs_tables_packed(srcs)
        assert ctx.last_kernel() == "dfs_bits_kernel<packed>"
        np.testing.assert_array_equal(tree, _pack(po, to))
        tree, depth = ctx.dfs_tables_tree(srcs, _native.TREE_PORT16, 2)
        assert ctx.last_kernel() == "dfs_bits_kernel<packed,hops>"
        np.testing.assert_array_equal(tree, _pack(po, to))
        np.testing.assert_array_equal(depth, ho.astype(np.uint16))


@pytest.mark.parametrize("name", ["fat_tree_k48", "dragonfly_a16_h8_p8"])
@pytest.mark.parametrize("nsrc", [1, 144, 0])
def test_dfs_bits_fullsize(ctx, monkeypatch, name, nsrc):
    """The bits kernel on the BASELINE small-V fabrics: every host source
    (k=48: 1,152; dragonfly: 2,064), or the first 1 / 144 (one GPU's share
    at N=8), packed trees bit-exact vs the oracle."""
    _strategy(monkeypatch, "bits")
    fabric = T.fat_tree(48) if name == "fat_tree_k48" else T.dragonfly(16, 8, 8)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    if nsrc:
        srcs = srcs[:nsrc]
    ctx.upload(csr)
    tree = ctx.dfs_tables_packed(srcs)
    assert ctx.last_kernel() == "dfs_bits_kernel<packed>"
    po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=NTHREADS)
    np.testing.assert_array_equal(tree, _pack(po, to))


@pytest.mark.parametrize("V", [4000, 4096])
def test_dfs_bits_log_spill(ctx, monkeypatch, V):
    """Graphs whose frame log, frame headers and stack outgrow their LDS
    parts (768 / 384 / 192): a long path with branches (deep stack, many
    frames) -- the spill to global memory stays bit-exact."""
    _strategy(monkeypatch, "bits")
    rng = np.random.default_rng(V)
    src, dst = [], []
    for u in range(V - 1):                       # a chain 0-1-2-..., both ways
        src += [u, u + 1]
        dst += [u + 1, u]
    for _ in range(V // 2):                      # plus random chords
        a, b = (int(x) for x in rng.integers(0, V, 2))
        if a != b:
            src += [a, b]
            dst += [b, a]
    from sdnmpi_amd.topologies import build_csr
    e = np.unique(np.stack([src, dst], 1), axis=0)
    csr = build_csr(e[:, 0] + 1, e[:, 1] + 1, np.arange(e.shape[0]) % 60 + 1)
    srcs = np.array([0, 1, V // 2, V - 1], np.int32)
    ctx.upload(csr)
    p, t, h = ctx.dfs_tables(srcs)
    assert ctx.last_kernel() == "dfs_bits_kernel<hops>"
    po, to, ho = O.dfs_tables(csr, srcs, nthreads=NTHREADS)
    np.testing.assert_array_equal(p, po)
    np.testing.assert_array_equal(t, to)
    np.testing.assert_array_equal(h, ho)


def _max_runs(csr):
    """Most arithmetic runs a sorted row (out or in) needs -- the encoding of
    capi.hip's encode_runs (strides <= 511)."""
    def runs(row):
        n, i, k = len(row), 0, 0
        while i < n:
            j = i
            if i + 1 < n and row[i + 1] - row[i] <= 511:
                st = row[i + 1] - row[i]
                j = i + 1
                while j + 1 < n and row[j + 1] - row[j] == st:
                    j += 1
            k += 1
            i = j + 1
        return k
    V = csr.V
    ins = [[] for _ in range(V)]
    most = 0
    for u in range(V):
        row = [int(x) for x in csr.col[csr.row_ptr[u]:csr.row_ptr[u + 1]]]
        most = max(most, runs(row))
        for v in row:
            ins[v].append(u)
    return max([most] + [runs(r) for r in ins])


# LDS-row kernel (dfs_runs.hip): every slot count / worker count / layout on
# every small fabric whose rows encode in <= 4 runs
@pytest.mark.parametrize("slots,workers", [(1, 1), (1, 3), (2, 2), (3, 3), (4, 3), (5, 2),
                                           (8, 1)])
@pytest.mark.parametrize("layout", ["int32", "hops", "packed"])
@pytest.mark.parametrize("name", G.SMALL)
def test_dfs_runs_small(ctx, monkeypatch, name, slots, workers, layout):
    _strategy(monkeypatch, "runs")
    monkeypatch.setenv("SDNROUTE_DFS_RUNS_SLOTS", str(slots))
    monkeypatch.setenv("SDNROUTE_DFS_RUNS_S", str(workers))
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    srcs = np.concatenate([srcs, srcs[::-1], srcs[:3]])      # more sources than slots
    ctx.upload(csr)
    po, to, ho = O.dfs_tables(csr, srcs, with_hops=True, nthreads=NTHREADS)
    if layout == "packed":
        got = ctx.dfs_tables_packed(srcs)
        np.testing.assert_array_equal(got, _pack(po, to))
    else:
        p, t, h = ctx.dfs_tables(srcs, with_hops=layout == "hops")
        np.testing.assert_array_equal(p, po)
        np.testing.assert_array_equal(t, to)
        if layout == "hops":
            np.testing.assert_array_equal(h, ho)
    if _max_runs(csr) <= 4:
        assert ctx.last_kernel().startswith("dfs_runs_kernel"), ctx.last_kernel()


@pytest.mark.parametrize("slots", [1, 5])
@pytest.mark.parametrize("name", ["fat_tree_k48_sample", "dragonfly_a16_h8_p8_sample"])
def test_dfs_runs_fullsize(ctx, monkeypatch, name, slots):
    _strategy(monkeypatch, "runs")
    monkeypatch.setenv("SDNROUTE_DFS_RUNS_SLOTS", str(slots))
    g = G.Golden(name)
    fabric = g.fabric()
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    p, t = _check_dfs(ctx, csr, srcs)
    assert ctx.last_kernel() == "dfs_runs_kernel<hops>"
    _check_pairs(g, fabric, p, t, srcs)


