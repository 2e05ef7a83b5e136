#!/usr/bin/env python3
"""Diagnostic: phase anatomy of the counted-pop DFS kernel (stamps build).

Loads libsdnroute_stamps.so (built with -DSDNR_STAMPS), runs the k=48
all-pairs DFS a few times and prints the mean s_memtime cycles per non-leaf
pop for each phase.  Never used for timing claims: the stamps' waits change
the schedule; read the SHARES.
"""
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

fab = T.by_name(sys.argv[1] if len(sys.argv) > 1 else "fat_tree:48")
csr = fab.csr()
srcs = np.unique(fab.host_table()[0]).astype(np.int32)
L = _native.library()
L.sdnr_debug_stamps.argtypes = [ctypes.c_void_p]
ctx = _native.Context(0)
ctx.upload(csr)
dev = torch.device("cuda", 0)
ts = torch.from_numpy(srcs).to(dev)
p = torch.empty((len(srcs), csr.V), dtype=torch.int32, device=dev)
t = torch.empty_like(p)
buf = (ctypes.c_ulonglong * 16)()
for rep in range(3):
    L.sdnr_debug_stamps(buf)            # reset
    ctx.dfs_tables_device(ts.data_ptr(), len(srcs), p.data_ptr(), t.data_ptr(), timing=True)
    ms = ctx.last_kernel_ms()
    L.sdnr_debug_stamps(buf)
    it = max(buf[5], 1)
    names = ["skip", "row+gather", "barrierA", "push+decrement", "barrierB"]
    print("rep %d  kernel %.3f ms  %s  non-leaf pops/source %.1f" % (
        rep, ms, ctx.last_kernel(), it / len(srcs)))
    tot = sum(buf[k] for k in range(5))
    for k, n in enumerate(names):
        print("   %-15s %7.0f cycles/pop  %4.1f%%" % (n, buf[k] / it, 100.0 * buf[k] / tot))
