#!/usr/bin/env python3
"""Diagnostic: kernel time vs number of sources/destinations on one fabric
(latency-bound chains stay flat until the GPU fills; throughput-bound
kernels grow linearly).  Usage: python tools/scaling_probe.py dfs|shortest FABRIC"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "dfs"
fab = T.by_name(sys.argv[2] if len(sys.argv) > 2 else "fat_tree:48")
csr = fab.csr()
srcs_all = np.unique(fab.host_table()[0]).astype(np.int32)
dev = torch.device("cuda", 0)
ctx = _native.Context(0)
ctx.upload(csr)
stream = torch.cuda.Stream(dev)
torch.cuda.set_stream(stream)
ctx.set_stream(stream.cuda_stream)
for n in (32, 128, 256, 512, 768, 1024, len(srcs_all)):
    srcs = srcs_all[np.linspace(0, len(srcs_all) - 1, n).astype(int)]
    ts = torch.from_numpy(np.ascontiguousarray(srcs)).to(dev)
    ms = []
    if mode == "dfs":
        a = torch.empty((n, csr.V), dtype=torch.int32, device=dev)
        for i in range(6):
            ctx.dfs_tables_packed_device(ts.data_ptr(), n, a.data_ptr(), timing=True)
            ms.append(ctx.last_kernel_ms())
    else:
        a = torch.empty((n, csr.V), dtype=torch.int16, device=dev)
        b = torch.empty((n, csr.V), dtype=torch.int32, device=dev)
        c = torch.empty_like(b)
        for i in range(6):
            ctx.shortest_tables_device(ts.data_ptr(), n, a.data_ptr(), b.data_ptr(), c.data_ptr(),
                                       timing=True)
            ms.append(ctx.last_kernel_ms())
    print("%s %s n=%5d  %.4f ms  (%s)" % (mode, sys.argv[2] if len(sys.argv) > 2 else "fat_tree:48",
                                           n, float(np.median(ms[1:])), ctx.last_kernel()), flush=True)
