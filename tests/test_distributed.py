"""Multi-rank table assembly on CPU (gloo, world_size 2 and 3): each rank
builds its shard of the per-source tables (oracle stands in for the GPU
kernel here), one all-gather assembles them, and the result must equal the
single-process table bit for bit -- including the -1 padding of the last
shard and uneven source counts."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fabric_name, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "sdn-mpi-router_amd")]
    from oracle import oracle as O
    from sdnmpi_amd import distributed as D
    from sdnmpi_amd import topologies as T
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fabric = T.by_name(fabric_name)
        csr = fabric.csr()
        srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
        mine = D.padded_shard(srcs, world, rank).numpy()
        # stand-in for the kernel: rows of -1 for padded (-1) sources
        ok = mine >= 0
        parent = np.full((len(mine), csr.V), -1, np.int32)
        port = np.full((len(mine), csr.V), -1, np.int32)
        if ok.any():
            p, t, _ = O.dfs_tables(csr, mine[ok], with_hops=False, nthreads=1)
            parent[ok], port[ok] = p, t
        gp = D.unpad(D.all_gather_rows(torch.from_numpy(parent)), len(srcs))
        # the bench's double-buffered form: async gathers into preallocated outputs
        out = torch.empty((world * len(mine), csr.V), dtype=torch.int32)
        D.all_gather_rows_async(torch.from_numpy(port), out).wait()
        gt = D.unpad(out, len(srcs))
        if rank == 0:
            po, to, _ = O.dfs_tables(csr, srcs, with_hops=False, nthreads=1)
            q.put(bool(np.array_equal(gp.numpy(), po) and np.array_equal(gt.numpy(), to)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fabric", [(2, "fat_tree:8"), (3, "dragonfly:4,2,2")])
def test_sharded_tables_assemble_exactly(world, fabric):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fabric, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_shard_bounds_cover_everything():
    from sdnmpi_amd.distributed import shard_bounds
    for n in (0, 1, 7, 1152, 1153):
        for world in (1, 2, 3, 8):
            rows = []
            for r in range(world):
                lo, hi, per = shard_bounds(n, world, r)
                assert hi - lo <= per
                rows += list(range(lo, hi))
            assert rows == list(range(n))


def _db_worker(rank, world, port, fabric_name, q):
    """Each rank: its own drop-in TopologyDB over the same topology events,
    the oracle standing in for the GPU engine (CPU test), its shard of the
    route tables, one all-gather per table."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "sdn-mpi-router_amd"), os.path.join(root, "tests")]
    from test_topologydb_dropin import _FakeEngine
    from sdnmpi_amd import distributed as D
    from sdnmpi_amd import topologies as T
    from sdnmpi_amd.util.topology_db import TopologyDB
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fabric = T.by_name(fabric_name)
        db = fabric.populate(TopologyDB())
        db._engine = _FakeEngine()
        res = []
        for mode in ("dfs", "shortest"):
            got = D.sharded_route_tables(db, mode)
            if rank == 0:
                ref = fabric.populate(TopologyDB())
                ref._engine = _FakeEngine()
                want = ref.route_tables(mode)
                res.append(all(np.array_equal(got[k], want[k]) for k in want))
        if rank == 0:
            q.put(all(res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fabric", [(2, "fat_tree:8"), (3, "torus:4,3,2")])
def test_sharded_topologydb_route_tables(world, fabric):
    """distributed.sharded_route_tables over per-rank TopologyDBs equals one
    TopologyDB's route_tables, both modes (gloo, world size 2 and 3)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_db_worker, args=(r, world, port, fabric, q))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def _rccl_worker(port, q):
    """One-rank RCCL process group on cuda:0: the table dtypes (int32 packed
    trees, int16 distances) through the bench's all-gather helpers."""
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path[:0] = [os.path.join(root, "sdn-mpi-router_amd")]
        from sdnmpi_amd import distributed as D
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        ok = []
        for dt in (torch.int32, torch.int16):
            loc = torch.arange(6 * 10, dtype=torch.int32, device="cuda").view(6, 10).to(dt) - 7
            out = torch.empty_like(loc)
            D.all_gather_rows_async(loc, out).wait()
            torch.cuda.synchronize()
            ok.append(bool(torch.equal(out, loc)))
        # sharded_route_tables on the nccl backend over a subgroup: the shard
        # travels as a device tensor, the gather uses the group passed in
        import numpy as np
        from sdnmpi_amd import topologies as T
        from sdnmpi_amd.util.topology_db import TopologyDB
        sub = dist.new_group([0])
        db = T.fat_tree(4).populate(TopologyDB())
        for mode in ("dfs", "shortest"):
            got = D.sharded_route_tables(db, mode, group=sub)
            want = db.route_tables(mode)
            ok.append(all(np.array_equal(got[k], want[k]) for k in want))
        dist.destroy_process_group()
        q.put(ok)
    except Exception as e:   # noqa: BLE001 -- reported to the parent
        q.put(repr(e))


@pytest.mark.gpu
def test_rccl_all_gather_table_dtypes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(60)
    assert res == [True, True, True, True], res


def _check_worker(rank, world, port, broken, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "sdn-mpi-router_amd")]
    from sdnmpi_amd import distributed as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if broken == "root":                # every rank's root-gather raises
            def boom(*a, **k):
                raise RuntimeError("p2p unavailable")
            D.gather_rows_to_root = boom
        elif broken == "wrong":             # the all-gather returns wrong rows on rank 1
            real = D.all_gather_rows_async

            def bad(local, out, group=None):
                w = real(local, out, group)
                w.wait()
                if dist.get_rank() == 1:
                    out.zero_()
                return w
            D.all_gather_rows_async = bad
        res = D.check_assembly()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("broken", ["none", "root", "wrong"])
def test_check_assembly_preflight(broken):
    """distributed.check_assembly, the preflight bench.py runs before an
    N > 1 line: both forms ok on a healthy group; a form that raises is
    reported as an error on every rank; wrong rows seen by ANY rank are
    reported on every rank (the verdict is all-reduced), so all ranks take
    the same fallback decision."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, world, port, broken, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        res = got[r]
        if broken == "none":
            assert res == {"root": "ok", "all": "ok"}
        elif broken == "root":
            assert res["root"].startswith("error") and res["all"] == "ok"
        else:
            assert res["root"] == "ok" and res["all"] == "wrong rows assembled"
