#!/usr/bin/env python3
"""Host time of one sdnr_graph_upload (CSR validation + ELL / u16 rows /
in-rows / runs derivation + H2D) per BASELINE fabric: what the drop-in pays
on the first query after a link event (the export itself is O(change),
DESIGN.md 2)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdn-mpi-router_amd"), ROOT]
import torch  # noqa: E402,F401

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

ctx = _native.Context(0)
for name in ("fat_tree:48", "dragonfly:16,8,8", "torus:32,32,32", "jellyfish:100000,16,1"):
    csr = T.by_name(name).csr()
    ctx.upload(csr)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        ctx.upload(csr)
        ts.append(time.perf_counter() - t)
    print("%-24s V=%6d E=%8d upload %.1f ms (min of 3)" % (name, csr.V, csr.E, min(ts) * 1e3))
