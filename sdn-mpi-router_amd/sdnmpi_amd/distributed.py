"""Source-sharded route tables over the GPUs of one node.

Every source tree (DFS mode) / destination table (shortest mode) is
independent, so the table rows shard with no communication in the compute:
rank r builds rows [r*per, (r+1)*per) of the padded source list on its own
GPU, and ONE all-gather (RCCL over xGMI with the "nccl" backend, gloo on CPU
for tests) assembles the full [sources][V] tables on every rank -- the
exchange step the controller needs to answer any (src, dst) from any rank.

The padded tail of the last shard uses source id -1, which the kernels turn
into an all-(-1) row; ``unpad`` drops it after the gather.
"""

import torch
import torch.distributed as dist

__all__ = ["shard_bounds", "padded_shard", "all_gather_rows", "all_gather_rows_async", "unpad",
           "sharded_route_tables", "gather_rows_to_root", "check_assembly"]


def shard_bounds(n, world, rank):
    """(lo, hi, per): rank's rows [lo, hi) of n, every rank padded to per."""
    per = (n + world - 1) // world if world > 0 else n
    lo = min(n, rank * per)
    hi = min(n, lo + per)
    return lo, hi, per


def padded_shard(ids, world, rank):
    """This rank's source ids, padded with -1 to the common shard length."""
    lo, hi, per = shard_bounds(len(ids), world, rank)
    out = torch.full((per,), -1, dtype=torch.int32)
    if hi > lo:
        out[: hi - lo] = torch.as_tensor(ids[lo:hi], dtype=torch.int32)
    return out


def all_gather_rows(local, group=None):
    """[per, V] on every rank -> [world*per, V] on every rank, rank order.

    One collective per table; on the nccl backend this is RCCL's all-gather
    over xGMI, writing straight into the assembled tensor.
    """
    world = dist.get_world_size(group)
    if world == 1:
        return local
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]),
                      dtype=local.dtype, device=local.device)
    if dist.get_backend(group) == "nccl":
        src, dst = local.contiguous(), out
        if src.dtype == torch.int16:         # RCCL has no 16-bit integers: move bytes
            src, dst = src.view(torch.uint8), out.view(torch.uint8)
        dist.all_gather_into_tensor(dst, src, group=group)
    else:   # gloo has no all_gather_into_tensor for every dtype
        parts = list(out.chunk(world, 0))
        dist.all_gather(parts, local.contiguous(), group=group)
    return out


def all_gather_rows_async(local, out, group=None):
    """Asynchronous all-gather of [per, V] rows into ``out`` [world*per, V]
    (rank order); returns the work handle.  On the nccl backend it runs on
    RCCL's stream, after the work already queued on the current stream, so
    the next kernel launched on the current stream overlaps it; ``wait()``
    before ``local`` or ``out`` is reused."""
    if dist.get_backend(group) == "nccl":
        src = local.contiguous()
        if src.dtype == torch.int16:         # RCCL has no 16-bit integers: move bytes
            src, out = src.view(torch.uint8), out.view(torch.uint8)
        return dist.all_gather_into_tensor(out, src, group=group, async_op=True)
    if local.is_cuda:        # gloo with device tensors (rehearsal): through host memory
        host = torch.empty(out.shape, dtype=out.dtype)
        src = local.contiguous().cpu()
        if src.dtype == torch.int16:         # gloo has no 16-bit integers: move bytes
            src, hv = src.view(torch.uint8), host.view(torch.uint8)
        else:
            hv = host
        dist.all_gather(list(hv.chunk(dist.get_world_size(group), 0)), src, group=group)
        out.copy_(host)
        return _Done()
    parts = list(out.chunk(dist.get_world_size(group), 0))
    return dist.all_gather(parts, local.contiguous(), group=group, async_op=True)


class _Done(object):
    def wait(self):
        return True


class _Works(object):
    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True


def gather_rows_to_root(local, out, group=None, root=0):
    """Rows [per, V] of every rank into ``out`` [world*per, V] on ``root`` only
    (rank order; ``out`` is ignored elsewhere): the tables assembled on the
    controller's GPU, SURVEY.md 8(e)'s "or on GPU 0 only" -- world-1 point-to-
    point transfers into the root instead of a ring all-gather to everyone.
    Returns a handle to ``wait()`` on."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    src = local.contiguous()
    if src.dtype == torch.int16:             # no 16-bit integers in the collectives: bytes
        src = src.view(torch.uint8)
        out = out.view(torch.uint8) if out is not None else None
    per = src.shape[0]
    groot = dist.get_global_rank(group, root) if group is not None else root
    if dist.get_backend(group) == "nccl":
        if rank == root:
            out[root * per:(root + 1) * per].copy_(src)
            ops = [dist.P2POp(dist.irecv, out[r * per:(r + 1) * per],
                              dist.get_global_rank(group, r) if group is not None else r,
                              group=group)
                   for r in range(world) if r != root]
        else:
            ops = [dist.P2POp(dist.isend, src, groot, group=group)]
        return _Works(dist.batch_isend_irecv(ops)) if ops else _Done()
    # gloo (CPU, rehearsal): through host memory
    host = src.cpu()
    parts = [torch.empty_like(host) for _ in range(world)] if rank == root else None
    dist.gather(host, parts, dst=groot, group=group)
    if rank == root:
        out.copy_(torch.cat(parts).to(out.device))
    return _Done()


def check_assembly(device=None, group=None, forms=("root", "all")):
    """Preflight of the two assembly forms on a small table (a few rows of
    rank-specific values): {"root": "ok" | error, "all": "ok" | error}.  A
    form that raises, or that assembles the wrong rows, is reported instead
    of failing the caller; bench.py runs this before its timed loop and
    falls back to the other form when the headline one is broken."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    rows, cols = 3, 5
    local = (torch.arange(rows * cols, dtype=torch.int32).view(rows, cols) + 1000 * rank)
    want = torch.cat([torch.arange(rows * cols, dtype=torch.int32).view(rows, cols) + 1000 * r
                      for r in range(world)])
    if device is not None:
        local = local.to(device)
    res = {}
    for form in forms:
        try:
            out = torch.full((world * rows, cols), -7, dtype=torch.int32, device=local.device)
            (all_gather_rows_async(local, out, group) if form == "all"
             else gather_rows_to_root(local, out, group)).wait()
            if local.is_cuda:
                torch.cuda.synchronize(local.device)
            if form == "all" or rank == 0:
                ok = bool(torch.equal(out.cpu(), want))
            else:
                ok = True
            # every rank learns whether the root (or any rank) saw a wrong table
            flag = torch.tensor([0 if ok else 1], dtype=torch.int32,
                                device=local.device if dist.get_backend(group) == "nccl"
                                else "cpu")
            dist.all_reduce(flag, group=group)
            res[form] = "ok" if int(flag.item()) == 0 else "wrong rows assembled"
        except Exception as e:   # noqa: BLE001 -- reported to the caller
            res[form] = "error: " + repr(e)[:200]
    return res


def unpad(table, n):
    return table[:n]


def sharded_route_tables(db, mode="dfs", group=None):
    """``db.route_tables(mode)`` computed by every rank of ``group`` together:
    one process per GPU, each with its own TopologyDB over the same dicts
    (e.g. replayed from the same Ryu events); rank r computes the rows of its
    contiguous shard of the host-bearing switches on its own device, and one
    all-gather per table assembles every row on every rank.  Same dict as
    ``db.route_tables(mode)``."""
    import numpy as np
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ex = db.graph()
    hv = db._host_vertices(ex)
    lo, hi, per = shard_bounds(len(hv), world, rank)
    t = db.route_tables(mode, vertices=hv[lo:hi])
    names = ("parent", "port", "hops") if mode == "dfs" else ("dist", "nh", "nh_port")
    out = dict(t)
    # RCCL moves device tensors only: the rank's shard goes to its GPU (one
    # process per GPU, torch's current device) and the gathered table back
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if nccl else None
    for name in names:
        a = t[name]
        pad = np.full((per, a.shape[1]), 0xFFFF if a.dtype == np.uint16 else -1, a.dtype)
        pad[: a.shape[0]] = a
        loc = torch.from_numpy(pad.view(np.int16) if a.dtype == np.uint16 else pad)
        if dev is not None:
            loc = loc.to(dev)
        if loc.dtype == torch.int16:                        # no 16-bit integers: move bytes
            g = all_gather_rows(loc.view(torch.uint8), group=group).view(torch.int16)
        else:
            g = all_gather_rows(loc, group=group)
        g = unpad(g, len(hv)).cpu().numpy()
        out[name] = g.view(np.uint16) if a.dtype == np.uint16 else g
    out["sources" if mode == "dfs" else "destinations"] = np.asarray(hv, np.int32)
    return out
