#!/usr/bin/env python3
"""Torus 32^3 shortest tables: does the 11.7 / 14.8 ms split
follow the process or the allocation?  One process, R rounds; each round
allocates a different-sized pad first, then a fresh Context (new device
scratch) and fresh tables, and times 5 calls with HIP events on the
kernels' stream.
    python tools/bimodal_probe.py [R]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402


def main(R):
    dev = torch.device("cuda", 0)
    csr = T.by_name("torus:32,32,32").csr()
    V = csr.V
    hv, _ = T.by_name("torus:32,32,32").host_table()
    srcs = torch.from_numpy(np.unique(hv).astype(np.int32)).to(dev)
    S = len(srcs)
    keep = []
    for r in range(R):
        pad = torch.empty(((r * 37) % 257 + 1) << 20, dtype=torch.uint8, device=dev)
        keep.append(pad)                           # shifts every later allocation
        ctx = _native.Context(0)
        ctx.upload(csr)
        st = torch.cuda.Stream(dev)
        torch.cuda.set_stream(st)
        ctx.set_stream(st.cuda_stream)
        dist = torch.empty((S, V), dtype=torch.int16, device=dev)
        nh = torch.empty((S, V), dtype=torch.int32, device=dev)
        port = torch.empty((S, V), dtype=torch.int32, device=dev)
        for _ in range(2):
            ctx.shortest_tables_device(srcs.data_ptr(), S, dist.data_ptr(), nh.data_ptr(),
                                       port.data_ptr())
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            ctx.shortest_tables_device(srcs.data_ptr(), S, dist.data_ptr(), nh.data_ptr(),
                                       port.data_ptr())
            e1.record(st)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1))
        print("round %d pad %3d MiB tables@%#x: %s ms" % (
            r, pad.numel() >> 20, dist.data_ptr(), " ".join("%.2f" % t for t in ts)), flush=True)
        ctx.close()
        del dist, nh, port
        torch.cuda.set_stream(torch.cuda.default_stream(dev))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8)
