"""Single-process multi-device context (sdnr_create_multi): the table calls
shard their ids over the listed devices and assemble the rows; the result
must equal the one-device tables bit for bit.  On a one-GPU box the devices
are logical shards on device 0 (the list may repeat a device), which runs the
same fork / peer-copy / join code as distinct GPUs.  Reference call site:
the controller's one TopologyDB (sdnmpi/topology.py:67, find_route at
:138-142)."""
import numpy as np
import pytest

import golden_util as G
from oracle import oracle as O
from sdnmpi_amd import _native
from sdnmpi_amd import topologies as T

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def one():
    c = _native.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("nshards", [2, 3, 8])
@pytest.mark.parametrize("name", ["fat_tree_k8", "dragonfly_a4_h2_p2", "random_V40",
                                  "torus_5x3x2", "jellyfish_n60_r5"])
def test_sharded_host_tables_equal_single(one, name, nshards):
    csr = G.Golden(name).fabric().csr()
    srcs = np.arange(csr.V, dtype=np.int32)
    one.upload(csr)
    p1, t1, h1 = one.dfs_tables(srcs)
    d1, n1, q1 = one.shortest_tables(srcs)
    with _native.Context([0] * nshards) as m:
        assert m.device_list() == [0] * nshards
        m.upload(csr)
        p, t, h = m.dfs_tables(srcs)
        np.testing.assert_array_equal(p, p1)
        np.testing.assert_array_equal(t, t1)
        np.testing.assert_array_equal(h, h1)
        d, n, q = m.shortest_tables(srcs)
        np.testing.assert_array_equal(d, d1)
        np.testing.assert_array_equal(n, n1)
        np.testing.assert_array_equal(q, q1)
        np.testing.assert_array_equal(m.dfs_tables_packed(srcs), one.dfs_tables_packed(srcs))
        # fewer ids than shards: empty shards are skipped
        few = srcs[:2]
        p, t, h = m.dfs_tables(few)
        np.testing.assert_array_equal(p, p1[:2])
        m.synchronize()


@pytest.mark.parametrize("nshards", [2, 4])
def test_sharded_device_tables_k48(one, nshards):
    """Device buffers on the primary: peers pull their ids and push their
    rows with peer copies, the primary stream joins them; packed k=48 tables
    of all host sources equal the oracle's."""
    torch = pytest.importorskip("torch")
    fabric = T.fat_tree(48)
    csr = fabric.csr()
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    dev = torch.device("cuda", 0)
    with _native.Context([0] * nshards) as m:
        m.upload(csr)
        stream = torch.cuda.Stream(dev)
        m.set_stream(stream.cuda_stream)
        ts = torch.from_numpy(srcs).to(dev)
        torch.cuda.synchronize(dev)
        tree = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
        m.dfs_tables_packed_device(ts.data_ptr(), len(srcs), tree.data_ptr(), timing=True)
        ms = m.last_kernel_ms()
        m.synchronize()
        assert ms > 0
        po, to, _ = O.dfs_tables(csr, srcs, with_hops=False)
        p, t = _native.unpack_tree(tree.cpu().numpy().view(np.uint32))
        np.testing.assert_array_equal(p, po)
        np.testing.assert_array_equal(t, to)
        dist = torch.empty((len(srcs), csr.V), dtype=torch.int16, device=dev)
        nh = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
        nhp = torch.empty_like(nh)
        m.shortest_tables_device(ts.data_ptr(), len(srcs), dist.data_ptr(), nh.data_ptr(),
                                 nhp.data_ptr())
        m.synchronize()
        do, nho, nhpo = O.dest_tables(csr, srcs)
        np.testing.assert_array_equal(dist.cpu().numpy().view(np.uint16), do)
        np.testing.assert_array_equal(nh.cpu().numpy(), nho)
        np.testing.assert_array_equal(nhp.cpu().numpy(), nhpo)


def test_dropin_over_devices_k48_golden():
    """TopologyDB(devices=[...]) answers the reference's k=48 pairs."""
    from sdnmpi_amd.util.topology_db import TopologyDB
    g = G.Golden("fat_tree_k48_sample")
    fabric = g.fabric()
    db = fabric.populate(TopologyDB(devices=[0, 0, 0]))
    macs = fabric.host_macs()
    pairs = [(macs[int(a)], macs[int(b)]) for a, b in zip(g.pair_src, g.pair_dst)]
    assert db.find_routes(pairs) == [g.fdb(i) for i in range(len(g))]
    assert [db.find_route(a, b) for a, b in pairs[:50]] == [g.fdb(i) for i in range(50)]
    assert db.engine.devices == [0, 0, 0]
