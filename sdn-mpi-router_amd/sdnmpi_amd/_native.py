"""ctypes binding of libsdnroute.so (C ABI: include/sdnroute.h).

This is the only way the product reaches the route kernels; there is no CPU
fallback.  If the library is missing or no gfx950 device is visible the
calls fail loudly (:class:`NativeUnavailable` / :class:`SdnrError`).

PyTorch ROCm bundles its own ``libamdhip64.so.7``; when torch is importable
it is imported first so that this library binds to the same HIP runtime
(shared soname) and device pointers / streams can be exchanged with torch.
"""

import ctypes
import os
import threading

import numpy as np

__all__ = ["NativeUnavailable", "SdnrError", "library", "library_path",
           "Context", "DEVICE_PTRS", "TIMING", "UNREACHED", "DIST_INF", "TREE_NONE",
           "EXPORTED_SYMBOLS", "unpack_tree"]

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_NAME = "libsdnroute.so"

DEVICE_PTRS = 0x1
TIMING = 0x2
SAME_TABLES = 0x4        # route expansion: the previous call's parent / port tables
UNREACHED = -1
DIST_INF = 0xFFFF
TREE_NONE = 0xFFFFFFFF
TREE_INT32 = 0           # int32 parents (sdnr_dfs_rows_affected)
TREE_PORT16 = 1          # parent | port << 16 (sdnr_dfs_tables_packed)
TREE_SLOT = 2            # parent | slot << 26 (sdnr_dfs_tables_slots)
ABI_VERSION = 1

# every entry point declared in include/sdnroute.h
EXPORTED_SYMBOLS = (
    "sdnr_abi_version", "sdnr_build_id", "sdnr_last_error", "sdnr_device_count", "sdnr_create",
    "sdnr_create_multi", "sdnr_device_list", "sdnr_destroy", "sdnr_set_stream", "sdnr_synchronize", "sdnr_graph_upload",
    "sdnr_graph_info", "sdnr_dfs_tables", "sdnr_dfs_tables_packed", "sdnr_dfs_tables_slots",
    "sdnr_dfs_tables_tree", "sdnr_tree_pack", "sdnr_shortest_tables", "sdnr_route_expand_packed",
    "sdnr_apsp", "sdnr_route_offsets", "sdnr_route_expand", "sdnr_ecmp_counts",
    "sdnr_ecmp_routes",
    "sdnr_last_kernel_ms", "sdnr_last_kernel", "sdnr_last_launches", "sdnr_last_sweeps",
    "sdnr_edge_ports", "sdnr_dfs_rows_affected",
)


class NativeUnavailable(RuntimeError):
    """libsdnroute.so could not be loaded (not built, or no HIP runtime)."""


class SdnrError(RuntimeError):
    def __init__(self, code, msg):
        super(SdnrError, self).__init__("sdnroute error %d: %s" % (code, msg))
        self.code = code


_lib = None
_lock = threading.Lock()


def library_path():
    return os.environ.get("SDNROUTE_LIB", os.path.join(_HERE, _LIB_NAME))


def _bind(L):
    c_int, i32, u32, vp = ctypes.c_int, ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p
    sig = {
        "sdnr_abi_version": ([], c_int),
        "sdnr_build_id": ([], ctypes.c_char_p),
        "sdnr_last_error": ([], ctypes.c_char_p),
        "sdnr_device_count": ([ctypes.POINTER(c_int)], c_int),
        "sdnr_create": ([c_int, ctypes.POINTER(vp)], c_int),
        "sdnr_create_multi": ([ctypes.POINTER(c_int), c_int, ctypes.POINTER(vp)], c_int),
        "sdnr_device_list": ([vp, ctypes.POINTER(c_int), c_int, ctypes.POINTER(c_int)], c_int),
        "sdnr_destroy": ([vp], c_int),
        "sdnr_set_stream": ([vp, vp], c_int),
        "sdnr_synchronize": ([vp], c_int),
        "sdnr_graph_upload": ([vp, i32, i32, vp, vp, vp], c_int),
        "sdnr_graph_info": ([vp, ctypes.POINTER(i32), ctypes.POINTER(i32),
                             ctypes.POINTER(i32)], c_int),
        "sdnr_dfs_tables": ([vp, vp, i32, vp, vp, vp, u32], c_int),
        "sdnr_dfs_tables_packed": ([vp, vp, i32, vp, u32], c_int),
        "sdnr_dfs_tables_slots": ([vp, vp, i32, vp, u32], c_int),
        "sdnr_tree_pack": ([vp, vp, vp, ctypes.c_int64, vp, i32, u32], c_int),
        "sdnr_dfs_tables_tree": ([vp, vp, i32, vp, vp, i32, i32, u32], c_int),
        "sdnr_route_expand_packed": ([vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, u32], c_int),
        "sdnr_shortest_tables": ([vp, vp, i32, vp, vp, vp, u32], c_int),
        "sdnr_apsp": ([vp, vp, u32], c_int),
        "sdnr_route_offsets": ([vp, vp, i32, vp, vp, i32, vp, u32], c_int),
        "sdnr_ecmp_counts": ([vp, vp, i32, vp, u32], c_int),
        "sdnr_ecmp_routes": ([vp, vp, vp, i32, vp, vp, vp, i32, i32, vp, u32], c_int),
        "sdnr_route_expand": ([vp, vp, vp, i32, vp, vp, vp, i32, vp, vp, vp, u32], c_int),
        "sdnr_last_kernel_ms": ([vp, ctypes.POINTER(ctypes.c_float)], c_int),
        "sdnr_last_kernel": ([vp], ctypes.c_char_p),
        "sdnr_last_launches": ([vp, ctypes.POINTER(i32)], c_int),
        "sdnr_last_sweeps": ([vp, ctypes.POINTER(i32)], c_int),
        "sdnr_edge_ports": ([vp, vp, i32, vp, i32, vp, u32], c_int),
        "sdnr_dfs_rows_affected": ([vp, vp, vp, i32, i32, i32, vp, vp, i32, i32, vp, u32], c_int),
    }
    # an A/B build named by SDNROUTE_LIB may predate some entry points: those
    # stay unbound (calling one raises AttributeError); the in-tree library
    # must export every one
    older_ok = "SDNROUTE_LIB" in os.environ
    for name, (args, res) in sig.items():
        if older_ok and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


def library():
    """Load (once) and return the bound library."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if not os.path.exists(path):
            raise NativeUnavailable(
                "%s not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                "in the repository root" % path)
        try:   # share torch's HIP runtime when torch is around
            import torch  # noqa: F401
        except Exception:   # noqa: BLE001 - torch is optional plumbing
            pass
        try:
            L = ctypes.CDLL(path)
        except OSError as e:
            raise NativeUnavailable("cannot load %s: %s" % (path, e))
        _bind(L)
        if L.sdnr_abi_version() != ABI_VERSION:
            raise NativeUnavailable("ABI mismatch: library %d, binding %d"
                                    % (L.sdnr_abi_version(), ABI_VERSION))
        if "SDNROUTE_LIB" not in os.environ:     # A/B and diagnostic builds are named explicitly
            verify_build(L)
        _lib = L
        return L


def verify_build(L, csrc=None, include=None):
    """Refuse a library that was not built from the tree beside it: its
    sdnr_build_id() must equal the SHA-256 of the current sources, headers
    and flags (_buildinfo.tree_build_id).  Skipped when the sources are not
    there (a package installed without csrc/)."""
    from . import _buildinfo as B
    want = B.tree_build_id(csrc or B.CSRC, include or B.INCLUDE)
    if want is None:
        return
    got = L.sdnr_build_id().decode("ascii", "replace")
    if got != want:
        raise NativeUnavailable(
            "stale %s: built from sources %s, the tree is %s -- rebuild with "
            "`python -c 'import __graft_entry__ as g; g.build()'`" % (library_path(), got[:16],
                                                                    want[:16]))


def _check(rc):
    if rc != 0:
        msg = library().sdnr_last_error().decode("utf-8", "replace")
        raise SdnrError(rc, msg)


def device_count():
    n = ctypes.c_int(0)
    _check(library().sdnr_device_count(ctypes.byref(n)))
    return n.value


def unpack_tree(tree):
    """Packed tree rows -> (parent, port) int32, -1 where the packed half is
    0xFFFF (unreached vertex / the root's port)."""
    t = np.asarray(tree, np.uint32)
    parent = (t & 0xFFFF).astype(np.int32)
    port = (t >> 16).astype(np.int32)
    parent[parent == 0xFFFF] = -1
    port[port == 0xFFFF] = -1
    return parent, port


def unpack_slots(tree, csr):
    """Slot tree rows (parent | slot << 26) -> (parent, port) int32 with the
    CSR's port of each tree link; -1 for unreached vertices and the root's
    port."""
    t = np.asarray(tree, np.uint32)
    none = t == TREE_NONE
    parent = (t & 0x3FFFFFF).astype(np.int64)
    slot = (t >> 26).astype(np.int64)
    root = slot == 63
    rp = np.asarray(csr.row_ptr, np.int64)
    idx = np.where(none | root, 0, rp[np.where(none, 0, parent)] + slot)
    port = np.asarray(csr.port, np.int32)[idx]
    port[none | root] = -1
    parent = parent.astype(np.int32)
    parent[none] = -1
    return parent, port


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class Context(object):
    """A route-engine context (owns graph + scratch) on one HIP device, or --
    ``device`` a sequence -- over several (sdnr_create_multi: the table calls
    are sharded by source/destination over the devices, device-pointer
    buffers live on the first one)."""

    def __init__(self, device=0):
        self._lib = library()
        h = ctypes.c_void_p()
        if isinstance(device, (list, tuple)):
            devs = [int(d) for d in device]
            arr = (ctypes.c_int * len(devs))(*devs)
            _check(self._lib.sdnr_create_multi(arr, len(devs), ctypes.byref(h)))
            self.devices = devs
        else:
            _check(self._lib.sdnr_create(int(device), ctypes.byref(h)))
            self.devices = [int(device)]
        self._h = h
        self.device = self.devices[0]
        self.V = -1
        self.E = 0

    def device_list(self):
        n = ctypes.c_int()
        _check(self._lib.sdnr_device_list(self._h, None, 0, ctypes.byref(n)))
        arr = (ctypes.c_int * n.value)()
        _check(self._lib.sdnr_device_list(self._h, arr, n.value, ctypes.byref(n)))
        return list(arr)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.sdnr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:   # noqa: BLE001 - interpreter shutdown
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- setup --------------------------------------------------------
    def set_stream(self, stream_handle):
        _check(self._lib.sdnr_set_stream(self._h, ctypes.c_void_p(stream_handle or 0)
                                         if stream_handle else None))

    def synchronize(self):
        _check(self._lib.sdnr_synchronize(self._h))

    def upload(self, csr):
        rp = np.ascontiguousarray(csr.row_ptr, np.int32)
        col = np.ascontiguousarray(csr.col, np.int32)
        port = np.ascontiguousarray(csr.port, np.int32)
        V, E = int(rp.shape[0] - 1), int(col.shape[0])
        _check(self._lib.sdnr_graph_upload(self._h, V, E, _ptr(rp),
                                           _ptr(col) if E else None,
                                           _ptr(port) if E else None))
        self.V, self.E = V, E

    def info(self):
        V, E, D = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _check(self._lib.sdnr_graph_info(self._h, ctypes.byref(V), ctypes.byref(E),
                                         ctypes.byref(D)))
        return V.value, E.value, D.value

    # -- host-buffer (synchronous) calls ------------------------------
    def dfs_tables(self, srcs, with_hops=True):
        srcs = np.ascontiguousarray(srcs, np.int32)
        S, V = int(srcs.shape[0]), self.V
        parent = np.empty((S, V), np.int32)
        port = np.empty((S, V), np.int32)
        hops = np.empty((S, V), np.int32) if with_hops else None
        _check(self._lib.sdnr_dfs_tables(self._h, _ptr(srcs), S, _ptr(parent),
                                         _ptr(port), _ptr(hops), 0))
        return parent, port, hops

    def dfs_tables_packed(self, srcs):
        """Packed trees: uint32 [S, V], parent | port << 16 (see unpack_tree)."""
        srcs = np.ascontiguousarray(srcs, np.int32)
        S, V = int(srcs.shape[0]), self.V
        tree = np.empty((S, V), np.uint32)
        _check(self._lib.sdnr_dfs_tables_packed(self._h, _ptr(srcs), S, _ptr(tree), 0))
        return tree

    def dfs_tables_slots(self, srcs):
        """Slot trees: uint32 [S, V], parent | slot << 26 (see unpack_slots)."""
        srcs = np.ascontiguousarray(srcs, np.int32)
        S, V = int(srcs.shape[0]), self.V
        tree = np.empty((S, V), np.uint32)
        _check(self._lib.sdnr_dfs_tables_slots(self._h, _ptr(srcs), S, _ptr(tree), 0))
        return tree

    def shortest_tables(self, dsts, with_nexthop=True):
        dsts = np.ascontiguousarray(dsts, np.int32)
        D, V = int(dsts.shape[0]), self.V
        dist = np.empty((D, V), np.uint16)
        nh = np.empty((D, V), np.int32) if with_nexthop else None
        nhp = np.empty((D, V), np.int32) if with_nexthop else None
        _check(self._lib.sdnr_shortest_tables(self._h, _ptr(dsts), D, _ptr(dist),
                                              _ptr(nh), _ptr(nhp), 0))
        return dist, nh, nhp

    def expand_routes(self, parent, port, hops, rows, dsts, last_port):
        """Flow entries of many pairs from host tables: (offsets int64
        [n+1], hop_switch int32, hop_port int32); see sdnr_route_expand."""
        parent = np.ascontiguousarray(parent, np.int32)
        port = np.ascontiguousarray(port, np.int32)
        hops = np.ascontiguousarray(hops, np.int32)
        rows = np.ascontiguousarray(rows, np.int32)
        dsts = np.ascontiguousarray(dsts, np.int32)
        last = np.ascontiguousarray(last_port, np.int32)
        n, nrows = int(rows.shape[0]), int(parent.shape[0])
        off = np.empty(n + 1, np.int64)
        _check(self._lib.sdnr_route_offsets(self._h, _ptr(hops), nrows, _ptr(rows), _ptr(dsts),
                                            n, _ptr(off), 0))
        total = int(off[-1])
        sw = np.empty(total, np.int32)
        hp = np.empty(total, np.int32)
        _check(self._lib.sdnr_route_expand(self._h, _ptr(parent), _ptr(port), nrows, _ptr(rows),
                                           _ptr(dsts), _ptr(last), n, _ptr(off), _ptr(sw),
                                           _ptr(hp), 0))
        return off, sw, hp

    def ecmp_counts(self, dist):
        """Shortest-route counts uint64 [D, V] from dist rows (saturating)."""
        dist = np.ascontiguousarray(dist, np.uint16)
        paths = np.empty(dist.shape, np.uint64)
        _check(self._lib.sdnr_ecmp_counts(self._h, _ptr(dist), int(dist.shape[0]), _ptr(paths), 0))
        return paths

    def ecmp_counts_device(self, dist_ptr, ndst, paths_ptr, timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_ecmp_counts(self._h, ctypes.c_void_p(dist_ptr), int(ndst),
                                          ctypes.c_void_p(paths_ptr), flags))

    def ecmp_routes(self, dist, paths, rows, srcs, ranks, max_len):
        """Vertex sequences int32 [n, max_len] (-1 padded) of the ranks[k]-th
        lexicographic shortest route from srcs[k] in row rows[k]."""
        dist = np.ascontiguousarray(dist, np.uint16)
        paths = np.ascontiguousarray(paths, np.uint64)
        rows = np.ascontiguousarray(rows, np.int32)
        srcs = np.ascontiguousarray(srcs, np.int32)
        ranks = np.ascontiguousarray(ranks, np.uint64)
        n = int(rows.shape[0])
        out = np.empty((n, int(max_len)), np.int32)
        _check(self._lib.sdnr_ecmp_routes(self._h, _ptr(dist), _ptr(paths), int(dist.shape[0]),
                                          _ptr(rows), _ptr(srcs), _ptr(ranks), n, int(max_len),
                                          _ptr(out), 0))
        return out

    def ecmp_routes_device(self, dist_ptr, paths_ptr, ndst, rows_ptr, srcs_ptr, ranks_ptr,
                           nroutes, max_len, out_ptr):
        _check(self._lib.sdnr_ecmp_routes(self._h, ctypes.c_void_p(dist_ptr),
                                          ctypes.c_void_p(paths_ptr), int(ndst),
                                          ctypes.c_void_p(rows_ptr), ctypes.c_void_p(srcs_ptr),
                                          ctypes.c_void_p(ranks_ptr), int(nroutes), int(max_len),
                                          ctypes.c_void_p(out_ptr), DEVICE_PTRS))

    def route_offsets_device(self, hops_ptr, rows_ptr, dsts_ptr, npairs, off_ptr, nrows=0):
        _check(self._lib.sdnr_route_offsets(self._h, ctypes.c_void_p(hops_ptr), int(nrows),
                                            ctypes.c_void_p(rows_ptr), ctypes.c_void_p(dsts_ptr),
                                            int(npairs), ctypes.c_void_p(off_ptr), DEVICE_PTRS))

    def expand_routes_device(self, parent_ptr, port_ptr, nrows, rows_ptr, dsts_ptr, last_ptr,
                             npairs, off_ptr, sw_ptr, hp_ptr, timing=False, same_tables=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0) | (SAME_TABLES if same_tables else 0)
        _check(self._lib.sdnr_route_expand(self._h, ctypes.c_void_p(parent_ptr),
                                           ctypes.c_void_p(port_ptr), int(nrows),
                                           ctypes.c_void_p(rows_ptr),
                                           ctypes.c_void_p(dsts_ptr), ctypes.c_void_p(last_ptr),
                                           int(npairs), ctypes.c_void_p(off_ptr),
                                           ctypes.c_void_p(sw_ptr), ctypes.c_void_p(hp_ptr), flags))

    def expand_routes_packed_device(self, parent_ptr, port_ptr, nrows, rows_ptr, dsts_ptr,
                                    last_ptr, npairs, off_ptr, ent_ptr, timing=False,
                                    same_tables=False):
        """Flow entries as one u32 each, switch | port << 16
        (sdnr_route_expand_packed, device pointers).  same_tables: the
        parent / port tables of the previous expansion on this context
        (SDNR_SAME_TABLES: its walk tables are reused)."""
        flags = DEVICE_PTRS | (TIMING if timing else 0) | (SAME_TABLES if same_tables else 0)
        _check(self._lib.sdnr_route_expand_packed(
            self._h, ctypes.c_void_p(parent_ptr), ctypes.c_void_p(port_ptr), int(nrows),
            ctypes.c_void_p(rows_ptr), ctypes.c_void_p(dsts_ptr), ctypes.c_void_p(last_ptr),
            int(npairs), ctypes.c_void_p(off_ptr), ctypes.c_void_p(ent_ptr), flags))

    def edge_ports(self, ends, ports):
        """bool [n_ports]: ports (uint64 keys) that are no link end (``ends``:
        sorted uint64 keys), see sdnr_edge_ports."""
        ends = np.ascontiguousarray(ends, np.uint64)
        ports = np.ascontiguousarray(ports, np.uint64)
        out = np.empty(ports.shape[0], np.uint8)
        _check(self._lib.sdnr_edge_ports(self._h, _ptr(ends), int(ends.shape[0]), _ptr(ports),
                                         int(ports.shape[0]), _ptr(out), 0))
        return out.astype(bool)

    def dfs_rows_affected_device(self, tree_ptr, depth_ptr, layout, depth_bytes, nrows,
                                 row_src_ptr, links_ptr, nremoved, nadded, affected_ptr,
                                 timing=False):
        """uint8 verdicts: which [nrows][V] tree rows the link changes alter
        (sdnr_dfs_rows_affected, device pointers, asynchronous)."""
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_dfs_rows_affected(
            self._h, ctypes.c_void_p(tree_ptr), ctypes.c_void_p(depth_ptr), int(layout),
            int(depth_bytes), int(nrows), ctypes.c_void_p(row_src_ptr),
            ctypes.c_void_p(links_ptr) if links_ptr else None, int(nremoved), int(nadded),
            ctypes.c_void_p(affected_ptr), flags))

    def apsp(self):
        dist = np.empty((self.V, self.V), np.uint16)
        _check(self._lib.sdnr_apsp(self._h, _ptr(dist), 0))
        return dist

    # -- device-pointer (asynchronous) calls --------------------------
    def dfs_tables_device(self, src_ptr, nsrc, parent_ptr, port_ptr, hops_ptr=0,
                          timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_dfs_tables(
            self._h, ctypes.c_void_p(src_ptr), int(nsrc), ctypes.c_void_p(parent_ptr),
            ctypes.c_void_p(port_ptr), ctypes.c_void_p(hops_ptr) if hops_ptr else None,
            flags))

    def dfs_tables_packed_device(self, src_ptr, nsrc, tree_ptr, timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_dfs_tables_packed(self._h, ctypes.c_void_p(src_ptr), int(nsrc),
                                                ctypes.c_void_p(tree_ptr), flags))

    def dfs_tables_slots_device(self, src_ptr, nsrc, tree_ptr, timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_dfs_tables_slots(self._h, ctypes.c_void_p(src_ptr), int(nsrc),
                                               ctypes.c_void_p(tree_ptr), flags))

    def dfs_tables_tree_device(self, src_ptr, nsrc, tree_ptr, depth_ptr, layout, depth_bytes,
                               timing=False):
        """Trees in a 4-byte layout (TREE_PORT16 / TREE_SLOT) plus depths
        (u16 or int32, ``depth_bytes`` 2 / 4; depth_ptr 0: none) straight
        from the DFS kernels (sdnr_dfs_tables_tree)."""
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_dfs_tables_tree(
            self._h, ctypes.c_void_p(src_ptr), int(nsrc), ctypes.c_void_p(tree_ptr),
            ctypes.c_void_p(depth_ptr) if depth_ptr else None, int(layout), int(depth_bytes),
            flags))

    def dfs_tables_tree(self, srcs, layout, depth_bytes=2):
        """Host-buffer form of dfs_tables_tree_device: (tree uint32 [S, V],
        depth uint16 / int32 [S, V])."""
        srcs = np.ascontiguousarray(srcs, np.int32)
        S, V = int(srcs.shape[0]), self.V
        tree = np.empty((S, V), np.uint32)
        depth = np.empty((S, V), np.uint16 if depth_bytes == 2 else np.int32)
        _check(self._lib.sdnr_dfs_tables_tree(self._h, _ptr(srcs), S, _ptr(tree), _ptr(depth),
                                              int(layout), int(depth_bytes), 0))
        return tree, depth

    def tree_pack_device(self, parent_ptr, port_ptr, n, tree_ptr, layout):
        """int32 parent/port tables (device) -> 4-byte trees (sdnr_tree_pack)."""
        _check(self._lib.sdnr_tree_pack(self._h, ctypes.c_void_p(parent_ptr),
                                        ctypes.c_void_p(port_ptr) if port_ptr else None,
                                        int(n), ctypes.c_void_p(tree_ptr), int(layout),
                                        DEVICE_PTRS))

    def shortest_tables_device(self, dst_ptr, ndst, dist_ptr, nh_ptr=0, nh_port_ptr=0,
                               timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_shortest_tables(
            self._h, ctypes.c_void_p(dst_ptr), int(ndst), ctypes.c_void_p(dist_ptr),
            ctypes.c_void_p(nh_ptr) if nh_ptr else None,
            ctypes.c_void_p(nh_port_ptr) if nh_port_ptr else None, flags))

    def apsp_device(self, dist_ptr, timing=False):
        flags = DEVICE_PTRS | (TIMING if timing else 0)
        _check(self._lib.sdnr_apsp(self._h, ctypes.c_void_p(dist_ptr), flags))

    def last_kernel(self):
        return self._lib.sdnr_last_kernel(self._h).decode()

    def last_launches(self):
        n = ctypes.c_int32()
        _check(self._lib.sdnr_last_launches(self._h, ctypes.byref(n)))
        return n.value

    def last_sweeps(self):
        """Bellman-Ford sweeps of the last APSP call (sdnr_last_sweeps)."""
        n = ctypes.c_int32()
        _check(self._lib.sdnr_last_sweeps(self._h, ctypes.byref(n)))
        return n.value

    def last_kernel_ms(self):
        ms = ctypes.c_float()
        _check(self._lib.sdnr_last_kernel_ms(self._h, ctypes.byref(ms)))
        return ms.value
