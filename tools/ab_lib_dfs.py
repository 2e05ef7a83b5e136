#!/usr/bin/env python3
"""A/B of the k=48 packed DFS tables between library builds (diagnostic).

    python tools/ab_lib_dfs.py [--fabric NAME] [--shortest] LIB[:ENV=VALUE] ...

Each library is loaded through plain ctypes (no build-identity check, so an
older build of the product library works too), the k=48 CSR uploaded, and
sdnr_dfs_tables_packed timed with HIP events on 1, 144 and 1,152 host
sources, libraries interleaved per repetition so box drift hits all alike.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "sdn-mpi-router_amd"))
from sdnmpi_amd import topologies as T  # noqa: E402


def open_lib(path):
    L = ctypes.CDLL(path)
    vp, i32, u32 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32
    L.sdnr_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.sdnr_graph_upload.argtypes = [vp, i32, i32, vp, vp, vp]
    L.sdnr_dfs_tables_packed.argtypes = [vp, vp, i32, vp, u32]
    L.sdnr_shortest_tables.argtypes = [vp, vp, i32, vp, vp, vp, u32]
    L.sdnr_set_stream.argtypes = [vp, vp]
    L.sdnr_synchronize.argtypes = [vp]
    h = vp()
    assert L.sdnr_create(0, ctypes.byref(h)) == 0
    return L, h


def main():
    print("torch imported", file=sys.stderr, flush=True)
    args = sys.argv[1:]
    fab = "fat_tree:48"
    if args and args[0] == "--fabric":
        fab, args = args[1], args[2:]
    shortest = bool(args) and args[0] == "--shortest"
    if shortest:
        args = args[1:]
    specs = [(a.split(":", 1) + [""])[:2] for a in args]    # (library, "ENV=VALUE" or "")
    libs = [a for a in args]
    fabric = T.by_name(fab)
    csr = fabric.csr()
    rp = np.ascontiguousarray(csr.row_ptr, np.int32)
    col = np.ascontiguousarray(csr.col, np.int32)
    port = np.ascontiguousarray(csr.port, np.int32)
    srcs = np.unique(fabric.host_table()[0]).astype(np.int32)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    opened = []
    cache = {}
    for p, (path, env) in zip(libs, specs):
        if path not in cache:
            cache[path] = open_lib(path)
        L, h = cache[path]
        assert L.sdnr_graph_upload(h, csr.V, csr.E, rp.ctypes.data, col.ctypes.data,
                                   port.ctypes.data) == 0
        L.sdnr_set_stream(h, ctypes.c_void_p(stream.cuda_stream))
        opened.append((p, L, h, env))
        print("opened %s" % p, file=sys.stderr, flush=True)
    res = {p: {} for p in libs}
    only = os.environ.get("AB_NS")            # e.g. "144,1152": these counts only
    ns = [n for n in (1, 8, 32, 144, 258, 288, 516, 576, 1152, len(srcs)) if n <= len(srcs)]
    if only:
        ns = [n for n in ns if str(n) in only.split(",") or (n == len(srcs) and "all" in only)]
    for n in sorted(set(ns)):
        pick = srcs[np.linspace(0, len(srcs) - 1, n).astype(np.int64)]
        ts = torch.from_numpy(pick).to(dev)
        out = torch.empty((n, csr.V), dtype=torch.int32, device=dev)
        o2, o3 = torch.empty_like(out), torch.empty_like(out)
        torch.cuda.synchronize(dev)
        for rep in range(6):
            for p, L, h, env in opened:
                k, _, v = env.partition("=")
                if k:
                    os.environ[k] = v
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    if shortest:
                        assert L.sdnr_shortest_tables(h, ts.data_ptr(), n, out.data_ptr(),
                                                      o2.data_ptr(), o3.data_ptr(), 1) == 0
                    else:
                        assert L.sdnr_dfs_tables_packed(h, ts.data_ptr(), n, out.data_ptr(),
                                                        1) == 0
                e1.record(stream)
                torch.cuda.synchronize(dev)
                assert L.sdnr_synchronize(h) == 0
                if k:
                    del os.environ[k]
                if rep:
                    res[p].setdefault(n, []).append(e0.elapsed_time(e1) / 10 * 1e3)
        print("done n=%d" % n, file=sys.stderr, flush=True)      # progress (a silent run looks hung)
    for p in libs:
        print(fab, "shortest" if shortest else "dfs", os.path.basename(p), {n: round(float(np.median(v)), 1) for n, v in res[p].items()})


if __name__ == "__main__":
    main()
