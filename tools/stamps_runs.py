#!/usr/bin/env python3
"""Diagnostic (stamps build): anatomy of the LDS-row DFS kernel's search
(dfs_runs.hip) -- candidates, false candidates (stale counts), candidates
found among the newest children, skip steps, cycles per phase, and the lag
of the decrement workers behind the search (children published but not yet
decremented, averaged over candidates).
Usage: stamps_runs.py [FABRIC] [NSOURCES]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
os.environ.setdefault("SDNROUTE_LIB", os.path.join(ROOT, "sdn-mpi-router_amd", "sdnmpi_amd",
                                                 "libsdnroute_stamps.so"))
os.environ.setdefault("SDNROUTE_DFS_STRATEGY", "runs")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

fab = T.by_name(sys.argv[1] if len(sys.argv) > 1 else "fat_tree:48")
csr = fab.csr()
srcs = np.unique(fab.host_table()[0]).astype(np.int32)
if len(sys.argv) > 2:
    srcs = srcs[:: max(1, len(srcs) // int(sys.argv[2]))][: int(sys.argv[2])]
L = _native.library()
L.sdnr_debug_stamps_runs.argtypes = [ctypes.c_void_p]
ctx = _native.Context(0)
ctx.upload(csr)
dev = torch.device("cuda", 0)
ts = torch.from_numpy(srcs).to(dev)
tree = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
buf = (ctypes.c_ulonglong * 16)()
for rep in range(3):
    L.sdnr_debug_stamps_runs(buf)
    ctx.dfs_tables_packed_device(ts.data_ptr(), len(srcs), tree.data_ptr(), timing=True)
    ms = ctx.last_kernel_ms()
    ctx.synchronize()
    L.sdnr_debug_stamps_runs(buf)
S = len(srcs)
cand = max(buf[1], 1)
print("%s %d sources %.4f ms | per source: life %.1fk cyc, candidates %.1f (false %.1f, "
      "children-first %.1f), skip steps %.1f | cycles per candidate: find %.0f, row+gather %.0f, "
      "push %.0f (per true candidate) | worker lag %.1f children" % (
          ctx.last_kernel(), S, ms, buf[0] / S / 1e3, buf[1] / S, buf[2] / S, buf[4] / S,
          buf[3] / S, buf[5] / cand, buf[6] / cand, buf[7] / max(buf[1] - buf[2], 1),
          buf[8] / cand))
