#!/usr/bin/env python3
"""Diagnostic (stamps build): anatomy of the split DFS kernel's search waves
on a large fabric -- cycles per iteration in the stack+row+visited read, the
record-queue wait, the push, spills and refills.  Never used for timing
claims: the stamps' waits change the schedule; read the SHARES."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
os.environ["SDNROUTE_LIB"] = os.path.join(ROOT, "sdn-mpi-router_amd", "sdnmpi_amd",
                                          "libsdnroute_stamps.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

fab = T.by_name(sys.argv[1] if len(sys.argv) > 1 else "torus:32,32,32")
csr = fab.csr()
L = _native.library()
L.sdnr_debug_stamps.argtypes = [ctypes.c_void_p]
ctx = _native.Context(0)
ctx.upload(csr)
dev = torch.device("cuda", 0)
buf = (ctypes.c_ulonglong * 16)()
packed = csr.V <= 65535
for nsrc in [int(x) for x in (sys.argv[2:] or ["256", "8192"])]:
    srcs = np.linspace(0, csr.V - 1, nsrc).astype(np.int32)
    ts = torch.from_numpy(srcs).to(dev)
    if packed:
        tr = torch.empty((nsrc, csr.V), dtype=torch.int32, device=dev)
    else:
        p = torch.empty((nsrc, csr.V), dtype=torch.int32, device=dev)
        t = torch.empty_like(p)
    for rep in range(2):
        L.sdnr_debug_stamps(buf)
        if packed:
            ctx.dfs_tables_packed_device(ts.data_ptr(), nsrc, tr.data_ptr(), timing=True)
        else:
            ctx.dfs_tables_device(ts.data_ptr(), nsrc, p.data_ptr(), t.data_ptr(), timing=True)
        ms = ctx.last_kernel_ms()
        ctx.synchronize()
        L.sdnr_debug_stamps(buf)
    S = nsrc
    it = max(buf[2], 1)
    print("%s %d sources %.3f ms | per source: life %.0fk cyc, iterations %.0f (non-leaf %.0f), "
          "read %.0f cyc/it, queue wait %.0f cyc/push, push %.0f cyc/push, spills %.0f, "
          "refills %.0f (%.0f cyc each)" % (
              ctx.last_kernel(), nsrc, ms, buf[0] / S / 1e3, buf[2] / S, buf[3] / S,
              buf[1] / it, buf[4] / max(buf[3], 1), buf[5] / max(buf[3], 1), buf[6] / S,
              buf[7] / S, buf[8] / max(buf[7], 1)), flush=True)
    del ts
