#!/usr/bin/env python3
"""GPU check: the bit-plane BFS forced on the k=48 fat-tree (rows of 48
slots, 6 slot planes) against the C oracle's destination tables."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
os.environ["SDNROUTE_SP_STRATEGY"] = "plane"
import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402
from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

for fab in ("fat_tree:48", "fat_tree:8"):
    csr = T.by_name(fab).csr()
    dsts = np.unique(T.by_name(fab).host_table()[0]).astype(np.int32)
    ctx = _native.Context(0)
    ctx.upload(csr)
    dist, nh, nhp = ctx.shortest_tables(dsts)
    assert ctx.last_kernel().startswith("msbfs_plane"), ctx.last_kernel()
    do, nho, nhpo = O.dest_tables(csr, dsts, nthreads=16)
    np.testing.assert_array_equal(dist, do)
    np.testing.assert_array_equal(nh, nho)
    np.testing.assert_array_equal(nhp, nhpo)
    print(fab, "plane BFS bit-exact vs oracle,", len(dsts), "destinations")
    ctx.close()
