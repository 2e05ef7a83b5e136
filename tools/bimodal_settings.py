#!/usr/bin/env python3
"""Torus 32^3 shortest tables: the time depends on where the allocation lands
(tools/bimodal_probe.py: 11.4-14.9 ms across fresh allocations in ONE
process).  Which setting removes the dependence?  R rounds, each with a
different pad before a fresh Context and tables; per round every setting
given (environment assignments read by the library at each call, e.g.
SDNROUTE_PLANE_CHUNK=48 or SDNROUTE_PLANE_PAD=64) is timed back to back,
3 calls each (HIP events on the kernels' stream).
    python tools/bimodal_chunk.py R NAME=VALUE[,NAME=VALUE] ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402


def main(R, chunks):
    base = {k: os.environ.get(k) for c in chunks for k, _ in (a.split("=") for a in c.split(","))}
    dev = torch.device("cuda", 0)
    fab = T.by_name("torus:32,32,32")
    csr = fab.csr()
    V = csr.V
    hv, _ = fab.host_table()
    srcs = torch.from_numpy(np.unique(hv).astype(np.int32)).to(dev)
    S = len(srcs)
    keep = []
    res = {c: [] for c in chunks}
    for r in range(R):
        keep.append(torch.empty(((r * 37) % 257 + 1) << 20, dtype=torch.uint8, device=dev))
        ctx = _native.Context(0)
        ctx.upload(csr)
        st = torch.cuda.Stream(dev)
        torch.cuda.set_stream(st)
        ctx.set_stream(st.cuda_stream)
        dist = torch.empty((S, V), dtype=torch.int16, device=dev)
        nh = torch.empty((S, V), dtype=torch.int32, device=dev)
        port = torch.empty((S, V), dtype=torch.int32, device=dev)
        line = []
        for c in chunks:
            for k, v in base.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            for a in c.split(","):
                k, v = a.split("=")
                os.environ[k] = v
            ctx.shortest_tables_device(srcs.data_ptr(), S, dist.data_ptr(), nh.data_ptr(),
                                       port.data_ptr())
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                ctx.shortest_tables_device(srcs.data_ptr(), S, dist.data_ptr(), nh.data_ptr(),
                                           port.data_ptr())
                e1.record(st)
                torch.cuda.synchronize(dev)
                ts.append(e0.elapsed_time(e1))
            res[c].append(min(ts))
            line.append("%s: %.2f" % (c, min(ts)))
        print("round %d: %s" % (r, " | ".join(line)), flush=True)
        ctx.close()
        del dist, nh, port
        torch.cuda.set_stream(torch.cuda.default_stream(dev))
    for c in chunks:
        v = np.array(res[c])
        print("%-40s min %.2f median %.2f max %.2f ms" % (c, v.min(), np.median(v), v.max()))


if __name__ == "__main__":
    main(int(sys.argv[1]), sys.argv[2:] or ["SDNROUTE_PLANE_CHUNK=64", "SDNROUTE_PLANE_CHUNK=32"])
