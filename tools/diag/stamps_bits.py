#!/usr/bin/env python3
"""Diagnostic (stamps build, tools/build_stamps.sh): anatomy of the
register-visited DFS kernel (dfs_bits.hip) -- explores vs false explores
(stale non-leaf bits), frame returns, row-prefetch misses, cycles per phase.
Never used for timing claims."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
os.environ["SDNROUTE_LIB"] = os.path.join(ROOT, "sdn-mpi-router_amd", "sdnmpi_amd",
                                          "libsdnroute_stamps.so")
os.environ["SDNROUTE_DFS_STRATEGY"] = "bits"
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

fab = T.by_name(sys.argv[1] if len(sys.argv) > 1 else "fat_tree:48")
csr = fab.csr()
srcs = np.unique(fab.host_table()[0]).astype(np.int32)
for n in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,144,1152").split(",")]:
    sub = srcs[:: max(1, len(srcs) // n)][:n]
    L = _native.library()
    L.sdnr_debug_bits_stamps.argtypes = [ctypes.c_void_p]
    ctx = _native.Context(0)
    ctx.upload(csr)
    dev = torch.device("cuda", 0)
    ts = torch.from_numpy(sub).to(dev)
    tree = torch.empty((len(sub), csr.V), dtype=torch.int32, device=dev)
    buf = (ctypes.c_ulonglong * 16)()
    for waves in os.environ.get("BITS_WAVES", "2,4,6").split(","):
        os.environ["SDNROUTE_DFS_BITS_WAVES"] = waves
        for rep in range(2):
            L.sdnr_debug_bits_stamps(buf)
            ctx.dfs_tables_packed_device(ts.data_ptr(), len(sub), tree.data_ptr(), timing=True)
            ms = ctx.last_kernel_ms()
            ctx.synchronize()
            L.sdnr_debug_bits_stamps(buf)
        S = max(1, buf[7])
        print("%d sources, %s waves: %.3f ms | per source: life %.0fk cyc, explores %.1f "
              "(false %.1f, prefetch misses %.1f), returns %.1f, explore %.0f cyc/explore, "
              "select %.0f cyc/explore" % (
                  len(sub), waves, ms, buf[0] / S / 1e3, buf[1] / S, buf[2] / S, buf[6] / S,
                  buf[3] / S, buf[4] / max(buf[1], 1), buf[5] / max(buf[1], 1)), flush=True)
    ctx.close()
