#!/usr/bin/env python3
"""Diagnostic (stamps build): anatomy of the asynchronous DFS kernel's search
wave on a fabric -- candidates vs false candidates (stale counts), prefetch
misses, back-pressure sleeps, skip steps, cycles per candidate."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
os.environ["SDNROUTE_LIB"] = os.path.join(ROOT, "sdn-mpi-router_amd", "sdnmpi_amd",
                                          "libsdnroute_stamps.so")
os.environ.setdefault("SDNROUTE_DFS_STRATEGY", "async")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

fab = T.by_name(sys.argv[1] if len(sys.argv) > 1 else "fat_tree:48")
csr = fab.csr()
srcs = np.unique(fab.host_table()[0]).astype(np.int32)
if len(sys.argv) > 2:                       # subset: fewer workgroups per CU
    srcs = srcs[:: max(1, len(srcs) // int(sys.argv[2]))][: int(sys.argv[2])]
L = _native.library()
L.sdnr_debug_stamps.argtypes = [ctypes.c_void_p]
ctx = _native.Context(0)
ctx.upload(csr)
dev = torch.device("cuda", 0)
ts = torch.from_numpy(srcs).to(dev)
p = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
t = torch.empty_like(p)
buf = (ctypes.c_ulonglong * 16)()
for nw in [int(x) for x in os.environ.get("STAMPS_WAVES", "3,4,5").split(",")]:
    os.environ["SDNROUTE_DFS_ASYNC_WAVES"] = str(nw)
    for rep in range(2):
        L.sdnr_debug_stamps(buf)
        if os.environ.get("STAMPS_PACKED") == "1":      # the headline's packed tables
            ctx.dfs_tables_packed_device(ts.data_ptr(), len(srcs), p.data_ptr(), timing=True)
        else:
            ctx.dfs_tables_device(ts.data_ptr(), len(srcs), p.data_ptr(), t.data_ptr(),
                                  timing=True)
        ms = ctx.last_kernel_ms()
        ctx.synchronize()
        L.sdnr_debug_stamps(buf)
    S = len(srcs)
    cand = buf[2] / S
    print("%s %.3f ms | per source: life %.0fk cyc, candidates %.1f (false %.1f), "
          "row+gather %.0f cyc/cand, skip %.0f cyc/cand, push %.0f cyc/push, bp sleeps %.1f, "
          "skip steps %.1f, prefetch misses %.1f" % (
              ctx.last_kernel(), ms, buf[0] / S / 1e3, cand, buf[3] / S, buf[1] / max(buf[2], 1),
              buf[6] / max(buf[2], 1), buf[7] / max(buf[2] - buf[3], 1),
              buf[4] / S, (buf[5] // 1000000) / S, (buf[5] % 1000000) / S))
    span = buf[11] - (~buf[12] & 0xFFFFFFFFFFFFFFFF)
    print("    per source: init %.1fk cyc, search+worker tail %.1fk cyc, flush %.1fk cyc; "
          "launch span %.1fk cyc" % (buf[8] / S / 1e3, buf[9] / S / 1e3, buf[10] / S / 1e3,
                                     span / 1e3))
