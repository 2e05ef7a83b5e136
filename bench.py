#!/usr/bin/env python3
"""All-pairs route tables on MI355X -- the BASELINE.json metric.

Workload (BASELINE.json configs[2], the metric's config): the k=48 fat-tree
(2,880 switches, 110,592 directed links, 27,648 hosts).  One step computes the
reference's default route (``TopologyDB.find_route``, LIFO search of
``sdnmpi/util/topology_db.py:59-84``) for EVERY host pair as per-source
tables: one tree (parent + out-port per switch) for each of the 1,152
host-bearing edge switches = 27,648^2 = 7.64e8 host-pair routes.  Inputs
(CSR, source list) are resident in HBM before the timed region; outputs stay
in HBM.

Multi-GPU (one rank per GPU, RCCL; ``--gpus N`` starts the N ranks itself
when no launcher did): the sources are split into contiguous blocks, each
rank builds its block, and the blocks are assembled over RCCL -- by default
on rank 0, the controller's GPU (point-to-point receives, SURVEY.md 8(e)'s
"or on GPU 0 only"), with ``--assemble all`` by an all-gather onto every
rank; the other form is timed beside it.  At N > 1 three consecutive steps
are kept in flight on their own streams (``--inflight``) when a rank's share
is under 4 sources per CU (k=48), so that it fills its GPU; the N = 1 line runs one step at a time (its roofline is
per launch) and reports the same GPU with 3 steps in flight as
``pipelined``, the like-for-like base for an N > 1 line.  Fixed total work
per step -> "scaling": "strong".

The JSON line also carries
  roofline      algorithmic bytes of the DFS kernel per launch
                (B_src = 4(V+1) + 4E + 4(V-1) + 8V per source)
                / its mean duration from HIP events on its stream, vs 8 TB/s;
  cpu_baseline  the oracle's per-source C restatement on the host cores
                (rank 0, N = 1), same workload;
  cpu_reference_path  the per-pair Python restatement of find_route (the
                reference's own algorithm shape) on a bounded pair sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "sdn-mpi-router_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sdnmpi_amd import _native  # noqa: E402
from sdnmpi_amd import distributed as D  # noqa: E402
from sdnmpi_amd import topologies as T  # noqa: E402

METRIC = "all-pairs routes/sec + % HBM roofline, k=48 fat-tree, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 steps: the timed region's fixed cost (barrier, synchronisation,
    # the first launch's latency; ~0.1 ms) was 5 % of a 20-step k=48 run
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--fabric", default="fat_tree:48")
    ap.add_argument("--mode", choices=["dfs", "shortest", "flows", "ecmp", "apsp", "matflows"],
                    default="dfs")
    ap.add_argument("--ranks", type=int, default=1024,
                    help="flows mode: MPI ranks placed on random hosts; every ordered "
                         "rank pair's flow entries are emitted per step")
    ap.add_argument("--layout", choices=["auto", "packed", "slots", "int32"], default="auto",
                    help="dfs tables: packed u32 (parent | port << 16) when the fabric "
                         "allows it (V <= 65535, 16-bit ports), else slot trees (parent | "
                         "slot << 26, sdnr_dfs_tables_slots) when rows have <= 63 links, "
                         "else int32 parent + port")
    ap.add_argument("--max-sources", type=int, default=0,
                    help="dfs/shortest: only the first N sources/destinations (probes; the "
                         "config then says so and value counts only their routes)")
    ap.add_argument("--all-vertices", action="store_true",
                    help="dfs/shortest: every switch as a source/destination (V x V switch "
                         "pairs, e.g. route_tables('shortest', vertices=all)) instead of the "
                         "host-bearing ones; value counts switch pairs")
    ap.add_argument("--event-every", type=int, default=10,
                    help="bracket every k-th timed launch with HIP events (kernel time; "
                         "the events themselves cost a few us per step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-flows", action="store_true",
                    help="dfs mode: skip the materialised flow-entry rate of every host pair")
    ap.add_argument("--cpu-budget-s", type=float, default=20.0,
                    help="bound on the CPU baseline's work")
    ap.add_argument("--assemble", choices=["all", "root", "none"], default="root",
                    help="N > 1: tables assembled on rank 0, the controller's GPU (RCCL "
                         "point-to-point receives into the root, default), or on every "
                         "rank (RCCL all-gather); the other form is measured beside it in "
                         "the multi_gpu block.  none: each rank keeps its shard (the "
                         "line's own fallback when neither form passes the preflight)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="steps kept in flight on their own streams (0: auto -- 3 at N > 1 "
                         "when one rank's share is under 4 sources per CU and leaves most of "
                         "its GPU idle (k=48), else 1; 1 at N = 1, "
                         "whose line then also reports the same GPU with 3 in flight as "
                         "'pipelined').  Every step still computes and assembles all tables")
    ap.add_argument("--profile", action="store_true",
                    help="profiling runs (tools/profile_gpu.sh): only the warmup + timed steps "
                         "run -- no single-step latency, no extra blocks -- so that a kernel's "
                         "dispatches per step are its dispatch count / (warmup + steps)")
    ap.add_argument("--rehearse", action="store_true",
                    help="launcher rehearsal on CPU: the N ranks form a gloo group, shard "
                         "the sources and assemble them, and rank 0 prints the line's "
                         "multi-rank keys -- no GPU call, no kernel (tests only)")
    return ap.parse_args()


def _traffic(key):
    """PMC-measured HBM bytes per launch recorded by tools/summarize_profile.py
    (profiles/traffic.json), or None."""
    try:
        return json.load(open(TRAFFIC_FILE)).get(key)
    except Exception:   # noqa: BLE001 -- missing / unreadable file: unmeasured
        return None


def _measured(traffic, kern_ms):
    """Measured HBM side of a roofline: the PMC traffic per launch
    (profiles/traffic.json, FETCH_SIZE / WRITE_SIZE with the factors
    tools/calib_traffic.py measured) over the live kernel time, and its
    fraction of the HBM peak -- beside the algorithmic frac."""
    if not traffic or not kern_ms:
        return {"hbm_gbs": None, "hbm_frac": None}
    gbs = traffic / (kern_ms / 1e3) / 1e9
    return {"hbm_gbs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS}


def algorithmic_bytes_per_source(V, E, mode, packed=False):
    if mode == "dfs":
        # row_ptr + col (CSR read per source) + tree-edge port reads + table writes
        # (parent + port: 8 B per vertex as int32, 4 B packed)
        return 4 * (V + 1) + 4 * E + 4 * (V - 1) + (4 if packed else 8) * V
    # shortest: CSR read + dist (2 B) + nh/nh_port (8 B) writes per destination
    return 4 * (V + 1) + 4 * E + 10 * V


def cpu_baseline(fabric, csr, srcs, hosts_per_src, H, budget_s):
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    # calibrate on a few sources, then run a bounded sample: the whole source
    # set repeated (or a prefix of it) for about budget_s/4 seconds
    probe = srcs[: max(1, min(len(srcs), threads))]
    t0 = time.perf_counter()
    O.dfs_tables(csr, probe, with_hops=False, nthreads=threads)
    per_src = (time.perf_counter() - t0) / len(probe) * threads
    target = budget_s / 4
    n = int(min(len(srcs), max(threads, target * threads / max(per_src, 1e-9))))
    sample = srcs[:n]
    reps, dt = 0, 0.0
    t0 = time.perf_counter()
    while reps == 0 or (time.perf_counter() - t0 < target and reps < 1000):
        O.dfs_tables(csr, sample, with_hops=False, nthreads=threads)
        reps += 1
    dt = time.perf_counter() - t0
    routes = float(hosts_per_src[:n].sum()) * H * reps
    out = {"value": routes / dt, "unit": "routes/s", "cores": threads, "kind": "port",
           "sample": "oracle/sdnroute_oracle.c per-source DFS trees (same algorithm, "
                     "pthreads, %d threads) for %d of %d sources x %d repetitions, %.2f s"
                     % (threads, n, len(srcs), reps, dt)}
    # the reference's own shape: one Python stack search per host pair, with
    # the reference's path copies (topology_db.py:59-84), and beside it the
    # same search keeping predecessor links (a faster restatement)
    db = _DictDB()
    fabric.populate(db)
    macs = fabric.host_macs()
    res = []
    for copying in (True, False):
        rng = np.random.default_rng(0)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < min(5.0, budget_s / 4):
            a, b = rng.integers(0, len(macs), 2)
            O.find_route_pair(db, macs[a], macs[b], copying=copying)
            k += 1
        dt = time.perf_counter() - t0
        res.append({"value": k / dt, "unit": "routes/s", "cores": 1, "kind": "port",
                    "sample": "oracle.find_route_pair(copying=%s): per-pair Python LIFO search "
                              "%s on %d random host pairs, %.2f s" % (
                                  copying, "copying the path list on every push, as "
                                  "topology_db.py:79 does" if copying else
                                  "keeping predecessor links (not the reference's cost)", k, dt)})
    return out, res[0], res[1]


_MP_DB = None


def _mp_pairs(args):
    """Worker of the multi-process per-pair baseline: random pairs for
    `secs` seconds over the fork-inherited _MP_DB."""
    from oracle import oracle as O
    seed, secs = args
    db, macs = _MP_DB
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < secs:
        a, b = rng.integers(0, len(macs), 2)
        O.find_route_pair(db, macs[a], macs[b], copying=True)
        k += 1
    return k, time.perf_counter() - t0


def cpu_reference_path_mp(fabric, secs=5.0):
    """SURVEY.md 8(d) CPU baseline (ii) on all host cores: the per-pair Python
    restatement in one process per core (fork, BEFORE any GPU call -- the
    children never touch the GPU), rate = sum of the per-process rates."""
    import multiprocessing as mp
    global _MP_DB
    procs = max(1, min(16, os.cpu_count() or 1))
    db = _DictDB()
    fabric.populate(db)
    _MP_DB = (db, fabric.host_macs())
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_mp_pairs, [(1000 + i, secs) for i in range(procs)])
    _MP_DB = None
    rate = sum(k / dt for k, dt in res)
    return {"value": rate, "unit": "routes/s", "cores": procs, "kind": "port",
            "sample": "oracle.find_route_pair(copying=True) (the reference's path-copying "
                      "search) in %d forked processes, %d random host pairs in %.1f s each" % (
                          procs, sum(k for k, _ in res), secs)}


class _DictDB(object):
    def __init__(self):
        self.switches, self.links, self.hosts = {}, {}, {}

    def add_switch(self, s):
        self.switches[s.dp.id] = s

    def add_link(self, lk):
        self.links.setdefault(lk.src.dpid, {})[lk.dst.dpid] = lk

    def add_host(self, h):
        self.hosts[h.mac] = h


def dropin_block(fabric, queries=10000, seed=5):
    """The drop-in as the controller calls it (reference sdnmpi/topology.py:
    138-142: one find_route per packet-in; :184-202: link events), timed on
    the host clock: TopologyDB (sdnmpi_amd.util.topology_db) over this GPU.

    cold_ms        first find_route: CSR export + upload + the trees of every
                   host-bearing switch into the device pool + one row to host;
    warm_us        mean per find_route over `queries` random host pairs
                   (one tree row copied to host per source miss, host LRU);
    batched_us     the same pairs through find_routes (route_entries: one
                   device expansion for all of them), per pair;
    event_ms       delete_link of a link on a cached route + the requery (the
                   rows the link can change recomputed), then add_link back
                   + requery."""
    from sdnmpi_amd.util.topology_db import TopologyDB
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    rng = np.random.default_rng(seed)
    pairs = [(macs[int(a)], macs[int(b)]) for a, b in rng.integers(0, len(macs), (queries, 2))]
    t0 = time.perf_counter()
    route = db.find_route(*pairs[0])
    cold = (time.perf_counter() - t0) * 1e3
    kernel = db.engine.ctx.last_kernel()
    rows = len(db._cache.dfs)
    t0 = time.perf_counter()
    for a, b in pairs:
        db.find_route(a, b)
    warm = (time.perf_counter() - t0) / len(pairs) * 1e6
    t0 = time.perf_counter()
    batch = db.find_routes(pairs)
    batched_first = (time.perf_counter() - t0) / len(pairs) * 1e6
    t0 = time.perf_counter()                 # steady state: the expansion kernels loaded
    batch = db.find_routes(pairs)
    batched = (time.perf_counter() - t0) / len(pairs) * 1e6
    assert batch[0] == route
    i = next(k for k in range(len(pairs)) if len(batch[k]) >= 3)   # a multi-switch route
    route = batch[i]
    pairs[0] = pairs[i]
    u, v = route[1][0], None
    for w, lk in db.links[u].items():
        if lk.src.port_no == route[1][1]:
            v = w
    link = db.links[u][v]
    t0 = time.perf_counter()
    db.delete_link(link)
    db.find_route(*pairs[0])
    t_del = (time.perf_counter() - t0) * 1e3
    recomputed = db._cache.rows_computed
    t0 = time.perf_counter()
    db.add_link(link)
    back = db.find_route(*pairs[0])
    t_add = (time.perf_counter() - t0) * 1e3
    assert back == route
    out = {"cold_ms": cold, "cold_rows": rows, "kernel": kernel, "warm_us": warm,
           "batched_us": batched, "batched_first_us": batched_first, "queries": len(pairs),
           "delete_link_requery_ms": t_del, "add_link_requery_ms": t_add,
           "rows_computed_total": recomputed,
           "note": "TopologyDB.find_route as the controller calls it (host clock): cold = "
                   "first query (export, upload, all host-switch trees into the device "
                   "pool); warm = mean per query over random host pairs; batched = "
                   "find_routes over the same pairs (second call; batched_first: the "
                   "first, with the expansion kernels' first launches); link event + "
                   "requery"}
    db.engine.close()
    return out


def materialised_flows(ctx, dev, stream, csr, fabric, srcs,
                       chunk=int(os.environ.get("BENCH_FLOWS_CHUNK", 1 << 24)), packed=False,
                       overlap=os.environ.get("BENCH_FLOWS_OVERLAP", "1") != "0"):
    """The fdb of EVERY host pair (Router._add_flows_for_path's input,
    reference sdnmpi/router.py:83-104; _route_to_fdb, topology_db.py:127-138)
    materialised in HBM from the default-route tables: the headline counts
    pairs whose route the tables determine, this counts pairs whose flow
    entries were actually written.  Requests (tree row, destination switch,
    host port) of all H^2 pairs are built once, untimed; then chunks of
    `chunk` pairs are sized (offsets) and expanded into a reused output
    buffer, timed with HIP events on the kernels' stream.  packed: each entry
    one u32 word, switch | port << 16 (sdnr_route_expand_packed), instead of
    two int32 arrays.  overlap: chunk c+1's offsets are computed on a second
    stream (a second library context, two offset buffers) while chunk c is
    expanded -- the offsets pass (~0.2 ms per chunk) then hides under the
    entry stores instead of adding to them."""
    V, H = csr.V, fabric.n_hosts
    hv, hp = fabric.host_table()
    S = len(srcs)
    ctx.set_stream(stream.cuda_stream)       # the events below bracket the library's work
    t_src = torch.from_numpy(srcs).to(dev)
    par = torch.empty((S, V), dtype=torch.int32, device=dev)
    prt = torch.empty_like(par)
    hop = torch.empty_like(par)
    ctx.dfs_tables_device(t_src.data_ptr(), S, par.data_ptr(), prt.data_ptr(), hop.data_ptr())
    ctx.synchronize()
    max_len = int(hop.max().item()) + 1
    row_of_host = torch.from_numpy(np.searchsorted(srcs, hv).astype(np.int32)).to(dev)
    sw_of_host = torch.from_numpy(hv.astype(np.int32)).to(dev)
    port_of_host = torch.from_numpy(hp.astype(np.int32)).to(dev)
    npairs = H * H
    offs = [torch.empty(chunk + 1, dtype=torch.int64, device=dev) for _ in range(2)]
    off = offs[0]
    sw = torch.empty(chunk * max_len, dtype=torch.int32, device=dev)
    octx, ostream = ctx, stream                  # where the offsets run
    if overlap:
        ostream = torch.cuda.Stream(dev)
        octx = _native.Context(dev.index)
        octx.upload(csr)
        octx.set_stream(ostream.cuda_stream)
    ev_off = [torch.cuda.Event() for _ in range(2)]      # offsets of buffer b written
    ev_use = [torch.cuda.Event() for _ in range(2)]      # expansion done reading buffer b
    hpo = sw if packed else torch.empty_like(sw)

    def expand(rows, dsts, last, n, same=False, off=off):
        # same: the tables of the previous chunk -- the walk tables derived
        # from them (packed trees + ancestor tables) are built once per pass
        if packed:
            ctx.expand_routes_packed_device(par.data_ptr(), prt.data_ptr(), S, rows.data_ptr(),
                                            dsts.data_ptr(), last.data_ptr(), n, off.data_ptr(),
                                            sw.data_ptr(), same_tables=same)
        else:
            ctx.expand_routes_device(par.data_ptr(), prt.data_ptr(), S, rows.data_ptr(),
                                     dsts.data_ptr(), last.data_ptr(), n, off.data_ptr(),
                                     sw.data_ptr(), hpo.data_ptr(), same_tables=same)
    reqs = []                                   # (rows, dsts, last) per chunk, untimed
    for p0 in range(0, npairs, chunk):
        idx = torch.arange(p0, min(npairs, p0 + chunk), dtype=torch.int64, device=dev)
        a, b = idx // H, idx % H
        reqs.append((row_of_host[a].contiguous(), sw_of_host[b].contiguous(),
                     port_of_host[b].contiguous()))
    # untimed: one chunk through the whole output buffer first (first-touch
    # page mapping of the 2 x chunk x max_len words happens here, not in the
    # timed loop)
    rows, dsts, last = reqs[0]
    ctx.route_offsets_device(hop.data_ptr(), rows.data_ptr(), dsts.data_ptr(), rows.shape[0],
                             off.data_ptr(), nrows=S)
    expand(rows, dsts, last, rows.shape[0])
    sw.fill_(0)
    hpo.fill_(0)
    # the timed loop's one torch op too: its first launch loads the kernel's
    # code object (measured: the first materialisation in a process took
    # ~130 ms against ~70 ms after, whichever entry form went first)
    entries = torch.zeros((), dtype=torch.int64, device=dev)
    entries += off[rows.shape[0]]
    entries.zero_()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for c, (rows, dsts, last) in enumerate(reqs):
        n = rows.shape[0]
        b = c % 2
        if overlap:                              # chunk c's offsets on the second stream,
            ostream.wait_event(ev_use[b])        # once chunk c-2 no longer reads buffer b
            if c == 0:
                ostream.wait_event(e0)
        octx.route_offsets_device(hop.data_ptr(), rows.data_ptr(), dsts.data_ptr(), n,
                                  offs[b].data_ptr(), nrows=S)
        if overlap:
            ev_off[b].record(ostream)
            stream.wait_event(ev_off[b])
        expand(rows, dsts, last, n, same=c > 0, off=offs[b])   # walk tables: first chunk
        entries += offs[b][n]                    # stream-ordered, no host sync
        if overlap:
            ev_use[b].record(stream)             # buffer b read by the expansion and the sum
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall_ms = (time.perf_counter() - t0) * 1e3
    ctx.synchronize()
    if overlap:
        octx.synchronize()
        octx.close()
    ms = e0.elapsed_time(e1)
    total = int(entries.item())
    # rate from the host clock around the whole loop (synchronised on both
    # sides; includes the launch overhead of every chunk), events beside it
    return {"value": npairs / (wall_ms / 1e3), "unit": "routes/s", "pairs": npairs,
            "entries": total, "entries_per_s": total / (wall_ms / 1e3), "ms": wall_ms,
            "event_ms": ms,
            "kernel": ctx.last_kernel(), "chunk_pairs": chunk,
            "entry_bytes": 4 if packed else 8,
            "form": "u32 switch | port << 16" if packed else "int32 switch + int32 port",
            "offsets_overlapped": overlap,
            "note": "flow entries (dpid, out_port) of all %d^2 host pairs written to HBM "
                    "(offsets + output-centric expansion per %d-pair chunk, one reused output "
                    "buffer), tables and requests resident; compare the headline, which "
                    "counts pairs whose route the tables determine" % (H, chunk)}


def main_matflows(args, world, rank, local, dev):
    """The default line's materialised_flows block alone (profiling): every
    host pair's fdb written to HBM, --steps repetitions."""
    fabric = T.by_name(args.fabric)
    csr = fabric.csr()
    hv, _ = fabric.host_table()
    srcs = np.unique(hv).astype(np.int32)
    ctx = _native.Context(local)
    ctx.upload(csr)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    resp = [materialised_flows(ctx, dev, stream, csr, fabric, srcs, packed=True)
            for _ in range(max(1, args.steps))]
    bestp = min(resp, key=lambda r: r["ms"])
    res = [materialised_flows(ctx, dev, stream, csr, fabric, srcs)
           for _ in range(max(1, args.steps))]
    best = min(res, key=lambda r: r["ms"])
    if rank == 0:
        print(json.dumps({"metric": "materialised flow entries of all host pairs, pairs/sec",
                          "value": bestp["value"], "unit": "routes/s", "n_gpus": 1,
                          "ms_per_step": bestp["ms"], "all_ms": [r["ms"] for r in resp],
                          "steps": len(resp), "higher_is_better": True,
                          "config": {"workload": "%s materialised flows" % args.fabric},
                          "materialised_flows": bestp, "int32_all_ms": [r["ms"] for r in res],
                          "materialised_flows_int32": best}), flush=True)
    ctx.close()


def main_flows(args, world, rank, local, dev):
    """Flow-entry emission: for R ranks on seeded random
    hosts, every ordered rank pair's fdb (Router._add_flows_for_path,
    reference sdnmpi/router.py:83-104) from default-route tables already
    resident in HBM.  One step = offsets (lengths + scan) + the tree walks
    for this rank's share of the pairs; value = pairs per second."""
    fabric = T.by_name(args.fabric)
    csr = fabric.csr()
    V = csr.V
    hv, hp = fabric.host_table()
    rng = np.random.default_rng(7)
    R = min(args.ranks, fabric.n_hosts)
    host = rng.choice(fabric.n_hosts, R, replace=False)
    srcs = np.unique(hv[host]).astype(np.int32)
    row_of = {int(v): i for i, v in enumerate(srcs.tolist())}
    a_idx = np.repeat(np.arange(R), R)
    b_idx = np.tile(np.arange(R), R)
    npairs_all = R * R
    lo, hi, _ = D.shard_bounds(npairs_all, world, rank)
    rows = np.asarray([row_of[int(v)] for v in hv[host[a_idx[lo:hi]]]], np.int32)
    dsts = hv[host[b_idx[lo:hi]]].astype(np.int32)
    last = hp[host[b_idx[lo:hi]]].astype(np.int32)
    n = hi - lo

    ctx = _native.Context(local)
    ctx.upload(csr)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    S = len(srcs)
    t_src = torch.from_numpy(srcs).to(dev)
    par = torch.empty((S, V), dtype=torch.int32, device=dev)
    prt = torch.empty_like(par)
    hop = torch.empty_like(par)
    ctx.dfs_tables_device(t_src.data_ptr(), S, par.data_ptr(), prt.data_ptr(), hop.data_ptr())
    t_rows = torch.from_numpy(rows).to(dev)
    t_dsts = torch.from_numpy(dsts).to(dev)
    t_last = torch.from_numpy(last).to(dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.route_offsets_device(hop.data_ptr(), t_rows.data_ptr(), t_dsts.data_ptr(), n, off.data_ptr())
    torch.cuda.synchronize(dev)
    total = int(off[-1].item())
    sw = torch.empty(total, dtype=torch.int32, device=dev)
    hpo = torch.empty(total, dtype=torch.int32, device=dev)

    def step(timing=False):
        ctx.route_offsets_device(hop.data_ptr(), t_rows.data_ptr(), t_dsts.data_ptr(), n,
                                 off.data_ptr())
        ctx.expand_routes_device(par.data_ptr(), prt.data_ptr(), S, t_rows.data_ptr(),
                                 t_dsts.data_ptr(), t_last.data_ptr(), n, off.data_ptr(),
                                 sw.data_ptr(), hpo.data_ptr(), timing=timing)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timing=True)
        kms.append(ctx.last_kernel_ms())        # waits for this step's walk kernel
    torch.cuda.synchronize(dev)
    ctx.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    kern_ms = float(np.mean(kms))
    # expansion: per entry parent + port read (8 B) and (switch, port)
    # written (8 B); per pair row/dst/last_port (12 B) + offsets pair (16 B)
    bytes_launch = 16 * total + 28 * n
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    traffic = None
    if os.path.exists(TRAFFIC_FILE):
        try:
            traffic = json.load(open(TRAFFIC_FILE)).get("%s/flows/N%d" % (args.fabric, world))
        except Exception:   # noqa: BLE001
            traffic = None
    out = {
        "metric": "flow entries for all MPI rank pairs (Router._add_flows_for_path), pairs/sec",
        "value": float(npairs_all) / (ms / 1e3), "unit": "routes/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (canonical fabric, ranks on seeded random hosts)",
        "config": {"workload": "%s flow entries of %d ranks (%d ordered pairs)" % (
            args.fabric, R, npairs_all), "fabric": args.fabric, "ranks": R,
            "pairs": npairs_all, "entries": total * world, "sources": S,
            "parallelism": "pairs sharded over %d GPU(s)" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": ctx.last_kernel(), "kernel_ms": kern_ms,
                     "bytes_per_launch": bytes_launch, **_measured(traffic, kern_ms)},
        "entries_per_s": float(total) * world / (ms / 1e3),
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main_ecmp(args, world, rank, local, dev):
    """ECMP-set sizes: the number of shortest routes of
    every host-switch pair, the count find_route(..., multiple=True) returns
    (reference topology_db.py:86-122, exponential there), by a level DP over
    the shortest-path DAG per destination.  Distances resident in HBM; one
    step = the counts of all destinations; value = switch pairs per second."""
    fabric = T.by_name(args.fabric)
    csr = fabric.csr()
    V = csr.V
    dsts = np.unique(fabric.host_table()[0]).astype(np.int32)
    lo, hi, per = D.shard_bounds(len(dsts), world, rank)
    my = D.padded_shard(dsts, world, rank)
    ctx = _native.Context(local)
    ctx.upload(csr)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    t_dst = my.to(dev)
    dist_t = torch.empty((per, V), dtype=torch.int16, device=dev)
    ctx.shortest_tables_device(t_dst.data_ptr(), per, dist_t.data_ptr())
    paths = torch.empty((per, V), dtype=torch.int64, device=dev)
    for _ in range(args.warmup):
        ctx.ecmp_counts_device(dist_t.data_ptr(), per, paths.data_ptr())
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.ecmp_counts_device(dist_t.data_ptr(), per, paths.data_ptr(), timing=True)
        kms.append(ctx.last_kernel_ms())
    torch.cuda.synchronize(dev)
    ctx.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    kern_ms = float(np.mean(kms))
    # per destination: dist row read (2V), CSR read (4(V+1) + 4E), counts written (8V)
    bytes_launch = (hi - lo) * (2 * V + 4 * (V + 1) + 4 * csr.E + 8 * V)
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    pairs = float(len(dsts)) * V
    out = {
        "metric": "ECMP-set sizes of all switch->host-switch pairs (find_route multiple=True), pairs/sec",
        "value": pairs / (ms / 1e3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "uint64", "data": "synthetic (canonical fabric)",
        "config": {"workload": "%s shortest-route counts for %d destinations" % (
            args.fabric, len(dsts)), "fabric": args.fabric, "V": V, "destinations": len(dsts),
            "max_routes_per_pair": int(paths.max().item()),
            "parallelism": "destinations sharded over %d GPU(s)" % world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": _traffic("%s/ecmp/N%d" % (
                         args.fabric, world)),
                     "kernel": ctx.last_kernel(), "kernel_ms": kern_ms,
                     "bytes_per_launch": bytes_launch,
                     **_measured(_traffic("%s/ecmp/N%d" % (args.fabric, world)), kern_ms)},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def main_apsp(args, world, rank, local, dev):
    """All-pairs hop distances by the blocked min-plus closure (apsp.hip) --
    the north star's small-dense-fabric kernel; every switch pair's hop count
    of find_route(..., multiple=True).  One step = the full V x V matrix;
    value = switch pairs per second; bound: the VALU min/add rate (min-plus is
    not a multiply-accumulate, so MFMA does not apply), reported against the
    packed-u16 VALU peak."""
    fabric = T.by_name(args.fabric)
    csr = fabric.csr()
    V = csr.V
    ctx = _native.Context(local)
    ctx.upload(csr)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    d = torch.empty((V, V), dtype=torch.int16, device=dev)
    for _ in range(args.warmup):
        ctx.apsp_device(d.data_ptr())
    torch.cuda.synchronize(dev)
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.apsp_device(d.data_ptr(), timing=True)
        kms.append(ctx.last_kernel_ms())
    torch.cuda.synchronize(dev)
    ctx.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    kern_ms = float(np.mean(kms))
    passes = ctx.last_launches()            # squaring passes of one APSP call
    sweeps = ctx.last_sweeps()              # Bellman-Ford sweeps (apsp_relax8_kernel)
    # algorithmic: one add + one min per (i, j, k) per squaring pass over the
    # V x V matrix (the kernels pad V to their tile: 64, or 128 for sq128),
    # and per (i, edge k -> j) per sweep
    tile = 128 if ctx.last_kernel() == "minplus_square_kernel" else 64
    Vp = (V + tile - 1) // tile * tile
    ops = passes * 2.0 * float(V) ** 3 + sweeps * 2.0 * float(V) * csr.E
    achieved = ops / (kern_ms / 1e3) / 1e12
    # VALU peak: 256 CUs x 4 SIMDs x 32 lanes x 2 (packed u16) ops/clk x 2.4 GHz
    peak = 256 * 4 * 32 * 2 * 2.4e9 / 1e12
    out = {
        "metric": "all-pairs hop distances (blocked min-plus APSP), switch pairs/sec",
        "value": float(V) * V / (ms / 1e3), "unit": "pairs/s", "n_gpus": 1,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u16",
        "data": "synthetic (canonical fabric)",
        "config": {"workload": "%s APSP (V=%d)" % (args.fabric, V), "fabric": args.fabric, "V": V},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "Tops/s",
                     "frac": achieved / peak, "traffic": _traffic("%s/apsp/N1" % args.fabric),
                     "kernel": ctx.last_kernel(),
                     "kernel_ms": kern_ms, "ops_per_launch": ops, "passes": passes,
                     "sweeps": sweeps,
                     "padded_ops_per_launch": passes * 2.0 * float(Vp) ** 3,
                     **_measured(_traffic("%s/apsp/N1" % args.fabric), kern_ms)},
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()


def _max_min(x, dev):
    """(max, min) of a float over the ranks."""
    on = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    a = torch.tensor([x], dtype=torch.float64, device=on)
    b = torch.tensor([-x], dtype=torch.float64, device=on)
    dist.all_reduce(a, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.MAX)
    return float(a.item()), -float(b.item())


def multi_gpu_extras(args, world, rank, local, dev, csr, srcs, per, packed, slots, kern_ms,
                     ms_per_step, routes, step, drain, bufs, gathered, assemble, check=None):
    """N > 1: what the step time is made of, and the other assembly forms.

    kernel_ms_max / _min  the route kernel per rank (HIP events);
    gather_ms             the table assembly alone (same tensors, no kernel);
    overlap               share of the shorter of the two hidden under the
                          other in the double-buffered step;
    assemble_{all,root}   ms per step with the tables assembled on every rank
                          (RCCL all-gather) / on rank 0 only (point-to-point);
    single_process        ms per step of ONE process driving all N devices
                          (sdnr_create_multi: shards on every device, rows
                          peer-copied to device 0), measured by rank 0 while
                          the other ranks wait."""
    reps = max(2, args.steps)

    def timed(fn):
        drain()
        torch.cuda.synchronize(dev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        drain()
        torch.cuda.synchronize(dev)
        dist.barrier()
        return _max_min((time.perf_counter() - t0) / reps * 1e3, dev)[0]

    def gather_only():
        for t, g in zip(bufs[0], gathered[0]):
            (D.all_gather_rows_async(t, g) if assemble[0] == "all"
             else D.gather_rows_to_root(t, g)).wait()

    kmax, kmin = _max_min(kern_ms, dev)
    gather_ms = timed(gather_only) if args.assemble != "none" else 0.0
    other = "root" if args.assemble == "all" else "all"
    # the secondary form is reported, never fatal for the headline (a form
    # that failed its preflight is not run at all)
    try:
        if args.assemble == "none":
            raise RuntimeError("no assembly: the shards stay on their ranks")
        if check and check.get(other) != "ok":
            raise RuntimeError("preflight: %s" % check.get(other))
        assemble[0] = other
        other_ms = timed(step)
        other_res = {"ms_per_step": other_ms, "value": routes / (other_ms / 1e3)}
    except Exception as e:   # noqa: BLE001
        other_res = {"error": repr(e)[:200]}
    finally:
        assemble[0] = args.assemble
    hidden = kmax + gather_ms - ms_per_step
    res = {
        "kernel_ms_max": kmax, "kernel_ms_min": kmin, "gather_ms": gather_ms,
        "overlap": max(0.0, min(1.0, hidden / max(1e-9, min(kmax, gather_ms)))),
        "assemble_" + args.assemble: {"ms_per_step": ms_per_step,
                                      "value": routes / (ms_per_step / 1e3)},
        "assemble_" + other: other_res,
    }
    # one process over all devices (the controller's own process, TopologyDB(
    # devices=[...])): rank 0 alone, the others wait at the barrier
    devices = [local] * world if os.environ.get("BENCH_DEVICE") else list(range(world))
    sp = None
    if rank == 0:
        try:
            mctx = _native.Context(devices)
            mctx.upload(csr)
            S = len(srcs)
            ts = torch.from_numpy(np.ascontiguousarray(srcs, np.int32)).to(dev)
            tab = torch.empty((S, csr.V), dtype=torch.int32, device=dev)
            tab2 = None if packed else torch.empty_like(tab)
            dist16 = torch.empty((S, csr.V), dtype=torch.int16, device=dev) \
                if args.mode == "shortest" else None

            def one():
                if dist16 is not None:
                    mctx.shortest_tables_device(ts.data_ptr(), S, dist16.data_ptr(),
                                                tab.data_ptr(), tab2.data_ptr())
                elif slots:
                    mctx.dfs_tables_slots_device(ts.data_ptr(), S, tab.data_ptr())
                elif packed:
                    mctx.dfs_tables_packed_device(ts.data_ptr(), S, tab.data_ptr())
                else:
                    mctx.dfs_tables_device(ts.data_ptr(), S, tab.data_ptr(), tab2.data_ptr())
            one()
            mctx.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                one()
            mctx.synchronize()
            ms = (time.perf_counter() - t0) / reps * 1e3
            sp = {"ms_per_step": ms, "value": routes / (ms / 1e3), "devices": devices,
                  "kernel": mctx.last_kernel()}
            mctx.close()
        except Exception as e:   # noqa: BLE001 -- reported, not fatal for the headline
            sp = {"error": repr(e)[:200], "devices": devices}
    dist.barrier()
    if sp is not None:
        res["single_process"] = sp
    return res


def pick_assembly(requested, check):
    """The assembly form an N > 1 line runs, from the preflight's verdicts
    (distributed.check_assembly): the requested form if it passed, else the
    other RCCL form if that passed, else none (each rank keeps its shard).
    Returns (form, "requested -> form" or None)."""
    if requested == "none" or check.get(requested) == "ok":
        return requested, None
    other = "all" if requested == "root" else "root"
    form = other if check.get(other) == "ok" else "none"
    return form, "%s -> %s" % (requested, form)


# why the line's default assembly is what it is (printed in config)
ASSEMBLE_REASON = {
    "root": "tables assembled on rank 0, the controller's GPU (the one process that serves "
            "find_route, reference sdnmpi/topology.py:138-142): each peer's rows go straight "
            "into its slice of the root's table over its own xGMI link (RCCL point-to-point, "
            "SURVEY.md 8(e) 'or on GPU 0 only'); the north_star's all-gather delivers 7/8 of "
            "the tables into EVERY GPU, ~7x the xGMI bytes of what the controller consumes, "
            "and is timed beside it (multi_gpu.assemble_all)",
    "all": "tables assembled on every rank by one RCCL all-gather per table over xGMI (the "
           "north_star's form); the root-only point-to-point form is timed beside it "
           "(multi_gpu.assemble_root)",
    "none": "each rank keeps its shard of the tables (sources partitioned, no data-path "
            "collective): chosen by --assemble none, or by the line itself when neither "
            "RCCL assembly form passed the preflight (multi_gpu.assembly_check)",
}


def n1_base(args, rank, local, dev, csr, srcs, tables, slots, packed, routes, est_ms):
    """The N = 1 base of an N > 1 line, measured in the same run: rank 0's GPU
    alone computes the WHOLE workload (all sources), one step at a time and
    -- where the table sets are small -- with 3 steps in flight, exactly as
    the N = 1 line's value / 'pipelined' do.  The other ranks wait at a
    barrier.  Returns None on the other ranks."""
    res = None
    if rank == 0:
        S = len(srcs)
        t_all = torch.from_numpy(np.ascontiguousarray(srcs, np.int32)).to(dev)
        set_bytes = sum(t.numel() * t.element_size() for t in tables(1)) * S
        res = {"measured_on": "rank 0's GPU alone, all %d sources per step" % S}
        try:
            if set_bytes <= (48 << 30):
                reps = int(max(2, min(max(args.steps, 30), 3000.0 / max(est_ms, 1e-3))))
                res["inflight_1"] = pipelined_rate(local, dev, csr, t_all, S, lambda: tables(S),
                                                   slots, packed, args.mode, routes, reps, k=1)
            if 3 * set_bytes <= (4 << 30) and est_ms <= 10.0:
                res["inflight_3"] = pipelined_rate(local, dev, csr, t_all, S, lambda: tables(S),
                                                   slots, packed, args.mode, routes,
                                                   max(args.steps, 30), k=3)
        except Exception as e:   # noqa: BLE001 -- reported, not fatal for the headline
            res["error"] = repr(e)[:200]
        torch.cuda.synchronize(dev)
    dist.barrier()
    return res


def scaling_keys(value, by_inflight, base, world):
    """Scaling efficiency of an N > 1 line against its own run's N = 1 base:
    like-for-like (same steps in flight as the headline when the base has
    them) and one step at a time on both sides."""
    if not base:
        return {}
    out = {}
    head = next(v for v in by_inflight.values() if v.get("headline"))
    k = head["steps_in_flight"]
    b = base.get("inflight_%d" % k) or base.get("inflight_1")
    if b:
        out["scaling_efficiency"] = value / (world * b["value"])
        out["scaling_efficiency_base"] = "n1_base.inflight_%d" % b["steps_in_flight"]
    b1, h1 = base.get("inflight_1"), by_inflight.get("1")
    if b1 and h1:
        out["scaling_efficiency_one_at_a_time"] = h1["value"] / (world * b1["value"])
    best = max([v["value"] for k_, v in base.items() if k_.startswith("inflight_")] or [0.0])
    if best:
        out["speedup_vs_n1_best"] = value / best
    return out


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """``--gpus N`` (N > 1) run without a launcher: start the N rank
    processes under torch.distributed.run (one process per GPU, RCCL over
    xGMI; rendezvous on 127.0.0.1) and return their exit status.  This
    process makes no GPU call at all -- the ranks are children, nothing is
    exec'd -- and each rank checks that the process group it forms has
    exactly N members on N distinct devices."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def rank_devices(dev, local):
    """Every rank's (rank, local device index, device uuid) in rank order --
    the multi-GPU line names the devices it ran on."""
    props = torch.cuda.get_device_properties(dev)
    mine = (dist.get_rank(), local, "pci %04x:%02x:%02x" % (
        props.pci_domain_id, props.pci_bus_id, props.pci_device_id))
    every = [None] * dist.get_world_size()
    dist.all_gather_object(every, mine)
    return every


def main_rehearse(args, world, rank):
    """The N-rank launch path without a GPU (CPU tests): the ranks form a
    gloo group, take their contiguous source shards exactly as the bench
    does, assemble them with the bench's all-gather helper, and rank 0
    prints the multi-rank keys of the line.  No kernel runs: the timing is
    the assembly of the source ids only."""
    dist.init_process_group("gloo")
    fabric = T.by_name(args.fabric)
    hv, _ = fabric.host_table()
    srcs, counts = np.unique(hv, return_counts=True)
    srcs = srcs.astype(np.int32)
    lo, hi, per = D.shard_bounds(len(srcs), world, rank)
    check = D.check_assembly()              # the line's preflight, on CPU
    mine = D.padded_shard(srcs, world, rank).view(per, 1)
    out = torch.empty((world * per, 1), dtype=torch.int32)
    routes = float(len(srcs)) * fabric.n_hosts

    args.assemble, fb = pick_assembly(args.assemble, check)
    if fb:
        check["fallback"] = fb

    def step():                             # the "step": this rank's ids assembled
        if args.assemble == "none":         # each rank keeps its shard
            out[rank * per:(rank + 1) * per].copy_(mine)
            return
        (D.all_gather_rows_async(mine, out) if args.assemble == "all"
         else D.gather_rows_to_root(mine, out)).wait()

    def timed(reps):
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        dist.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()) / reps * 1e3

    ms = timed(max(1, args.steps))
    single = timed(1)
    by_inflight = {"1": {"steps_in_flight": 1, "ms_per_step": ms, "value": routes / (ms / 1e3),
                         "steps": args.steps, "headline": True}}
    base = None
    if rank == 0:                           # rank 0 alone, all ids (meaningless rate)
        t0 = time.perf_counter()
        torch.from_numpy(srcs).clone()
        b = max(1e-6, (time.perf_counter() - t0) * 1e3)
        base = {"measured_on": "rank 0 alone (rehearsal)",
                "inflight_1": {"steps_in_flight": 1, "ms_per_step": b,
                               "value": routes / (b / 1e3)}}
    shards = [None] * world
    dist.all_gather_object(shards, (rank, lo, hi, os.getpid()))
    if args.assemble == "none":             # this rank's own slice holds its shard
        ok = bool(np.array_equal(out[rank * per:(rank + 1) * per].view(-1).numpy(),
                                 mine.view(-1).numpy()))
    elif args.assemble == "root":
        ok = rank != 0 or bool(np.array_equal(D.unpad(out.view(-1), len(srcs)).numpy(), srcs))
    else:
        ok = bool(np.array_equal(D.unpad(out.view(-1), len(srcs)).numpy(), srcs))
    cpu = None
    if rank == 0 and not args.no_cpu_baseline:   # as the N > 1 line: rank 0, after the steps
        cpu = cpu_baseline(fabric, fabric.csr(), srcs, counts, fabric.n_hosts,
                           args.cpu_budget_s)[0]
    dist.barrier()
    if rank == 0:
        multi = {"single_step_ms": single, "by_inflight": by_inflight,
                 "assembly_check": check, "n1_base": base}
        multi.update(scaling_keys(routes / (ms / 1e3), by_inflight, base, world))
        print(json.dumps({
            "metric": METRIC, "rehearsal": True, "value": None, "n_gpus": world,
            "steps": args.steps, "ms_per_step": ms, "single_step_ms": single,
            "process_group": {"backend": dist.get_backend(), "world_size": dist.get_world_size()},
            "config": {"fabric": args.fabric, "sources": len(srcs), "assemble": args.assemble,
                       "assemble_reason": ASSEMBLE_REASON[args.assemble],
                       "parallelism": "sources sharded over %d rank(s)" % world},
            "multi_gpu": multi, "cpu_baseline": cpu,
            "shards": [{"rank": r, "lo": a, "hi": b, "pid": p} for r, a, b, p in shards],
            "sources_assembled_exactly": ok}), flush=True)
    dist.destroy_process_group()
    return 0 if ok else 1


def pipelined_rate(local, dev, csr, t_src, per, tables, slots, packed, mode, routes, steps,
                   k=3):
    """The same step with k consecutive steps in flight on their own streams
    and library contexts (what an N > 1 rank runs), one GPU: every step
    still computes every table of the step.  k = 1: one step at a time,
    back to back on one stream (the N = 1 line's own schedule)."""
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    ctxs = []
    for st in streams:
        c = _native.Context(local)
        c.upload(csr)
        c.set_stream(st.cuda_stream)
        ctxs.append(c)
    bufs = [tables() for _ in range(k)]

    def launch(i):
        c, tb = ctxs[i % k], bufs[i % k]
        with torch.cuda.stream(streams[i % k]):
            if slots:
                c.dfs_tables_slots_device(t_src.data_ptr(), per, tb[0].data_ptr())
            elif packed:
                c.dfs_tables_packed_device(t_src.data_ptr(), per, tb[0].data_ptr())
            elif mode == "dfs":
                c.dfs_tables_device(t_src.data_ptr(), per, tb[0].data_ptr(), tb[1].data_ptr())
            else:
                c.shortest_tables_device(t_src.data_ptr(), per, tb[0].data_ptr(),
                                         tb[1].data_ptr(), tb[2].data_ptr())
    for i in range(2 * k):
        launch(i)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(steps):
        launch(i)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    for c in ctxs:
        c.synchronize()
        c.close()
    return {"steps_in_flight": k, "ms_per_step": ms, "value": routes / (ms / 1e3),
            "steps": steps,
            "note": "same workload, %d consecutive steps in flight on their own streams (as "
                    "an N > 1 rank runs them); every step computes every table" % k}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher around us: become the launcher (before any GPU call)
        sys.exit(launch_ranks(args))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: %d ranks were launched (WORLD_SIZE) but --gpus is %d"
                         % (world, args.gpus))
    if args.rehearse:
        sys.exit(main_rehearse(args, world, rank) if world > 1 else 0)
    ref_mp = None
    if world == 1 and args.mode == "dfs" and not args.no_cpu_baseline:
        # forks: must run before the first GPU call of this process (and so
        # before the device count below, which may initialise HIP when
        # torch cannot count through amdsmi)
        ref_mp = cpu_reference_path_mp(T.by_name(args.fabric),
                                       secs=min(5.0, args.cpu_budget_s / 4))
    # BENCH_DEVICE pins every rank to one device (rehearsing the N > 1 code
    # path on a one-GPU box); the driver never sets it
    if os.environ.get("BENCH_DEVICE"):
        local = int(os.environ["BENCH_DEVICE"])
    elif torch.cuda.device_count() < world:
        raise SystemExit("bench.py: --gpus %d but only %d GPU(s) are visible"
                         % (world, torch.cuda.device_count()))
    torch.cuda.set_device(local)              # before the process group: its communicator
    if world > 1:                             # and every context live on this rank's GPU
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")   # gloo: rehearsal only
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    devices = None
    if world > 1:
        devices = rank_devices(dev, local)
        uuids = {d[2] for d in devices}
        if len(uuids) != world and not os.environ.get("BENCH_DEVICE"):
            raise SystemExit("bench.py: %d ranks share %d device(s): %r"
                             % (world, len(uuids), devices))
    assembly_check = None
    if world > 1 and args.mode in ("dfs", "shortest"):
        # both assembly forms on a small table before anything is timed: a
        # form that raises or assembles wrong rows is reported, and the
        # headline falls back to the other one instead of losing the line
        assembly_check = D.check_assembly(dev)
        args.assemble, fb = pick_assembly(args.assemble, assembly_check)
        if fb:                              # the line is kept either way
            assembly_check["fallback"] = fb
    if args.mode == "flows":
        return main_flows(args, world, rank, local, dev)
    if args.mode == "ecmp":
        return main_ecmp(args, world, rank, local, dev)
    if args.mode == "apsp":
        return main_apsp(args, world, rank, local, dev)
    if args.mode == "matflows":
        return main_matflows(args, world, rank, local, dev)

    fabric = T.by_name(args.fabric)
    csr = fabric.csr()
    V, E = csr.V, csr.E
    hv, _ = fabric.host_table()
    srcs, counts = np.unique(hv, return_counts=True)
    srcs = srcs.astype(np.int32)
    H = fabric.n_hosts
    if args.all_vertices:                   # switch pairs: one endpoint per switch
        srcs, counts, H = np.arange(V, dtype=np.int32), np.ones(V, np.int64), V
    if args.max_sources and args.max_sources < len(srcs):
        pick = np.linspace(0, len(srcs) - 1, args.max_sources).astype(np.int64)
        srcs, counts = srcs[pick], counts[pick]
    S = len(srcs)
    lo, hi, per = D.shard_bounds(S, world, rank)
    my = D.padded_shard(srcs, world, rank)   # pad: id -1 -> empty row

    ctx = _native.Context(local)
    ctx.upload(csr)
    stream = torch.cuda.Stream(dev)       # the kernels' stream (events go here)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    t_src = my.to(dev)
    port16 = args.mode == "dfs" and args.layout in ("auto", "packed") and V <= 0xFFFF and \
        csr.E > 0 and int(csr.port.min()) >= 0 and int(csr.port.max()) < 0xFFFF
    if args.layout == "packed" and not port16:
        raise SystemExit("--layout packed: fabric has V > 65535 or ports >= 0xFFFF")
    slots = args.mode == "dfs" and not port16 and args.layout in ("auto", "slots") and \
        V < (1 << 26) and csr.max_degree() <= 63
    if args.layout == "slots" and not slots:
        raise SystemExit("--layout slots: fabric has a switch with more than 63 links")
    packed = port16 or slots                  # one u32 per tree entry
    def tables(rows=per):
        if packed:
            return (torch.empty((rows, V), dtype=torch.int32, device=dev),)   # parent | port << 16
        if args.mode == "dfs":
            return (torch.empty((rows, V), dtype=torch.int32, device=dev),    # parent
                    torch.empty((rows, V), dtype=torch.int32, device=dev))    # port
        return (torch.empty((rows, V), dtype=torch.int16, device=dev),        # dist (u16)
                torch.empty((rows, V), dtype=torch.int32, device=dev),        # nh
                torch.empty((rows, V), dtype=torch.int32, device=dev))        # nh_port

    # N > 1: one rank's share of the k=48 sources (144 at N = 8) fills an
    # eighth of the GPU, and a source's search is a serial chain (DESIGN.md
    # 4.1b): consecutive steps -- independent recomputations of the same
    # tables -- run on their own streams so that a rank keeps about as many
    # sources resident as one GPU holds at N = 1 (4 per CU); two table sets
    # per stream, so a step's kernel overlaps the previous step's gather
    # (3 in flight is the most that pays: HIP gives a process 4 hardware
    # queues, and RCCL's stream takes one; one GPU, k=48 shares of 144 / 288 /
    # 576 sources: 47.5 -> 20.9 / 26.5 / 39.2 us per step at 3, 28.4 / 34.0
    # at 4, profiles/r05_inflight_sweep.jsonl).  N = 1 keeps one step at a
    # time -- the line's per-launch roofline -- and reports the same GPU's
    # rate with 3 in flight beside it ("pipelined"), the like-for-like base
    # of an N > 1 line
    # (a share of >= 4 sources per CU -- the torus, Jellyfish -- fills the GPU
    # with one step, and its table sets are large: one step at a time)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    inflight = args.inflight if args.inflight > 0 else \
        (3 if world > 1 and per < 4 * cus else 1)
    infl = [inflight]                        # steps in flight right now (the single-step
                                             # and one-at-a-time measurements set 1)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(inflight - 1)]
    # one library context per stream in flight: a context's scratch (the split
    # kernel's spill rings and chunk cursors, the watchdog word) serves one
    # stream at a time
    ctxs = [ctx]
    for st in streams[1:]:
        c = _native.Context(local)
        c.upload(csr)
        c.set_stream(st.cuda_stream)
        ctxs.append(c)
    nbuf = (2 if world > 1 else 1) * inflight
    bufs = [tables() for _ in range(nbuf)]
    gathered = [tuple(torch.empty((world * per, V), dtype=t.dtype, device=dev) for t in b)
                for b in bufs]
    pending = [[] for _ in range(nbuf)]
    counter = [0]
    assemble = [args.assemble]

    def step(ev=None):
        k = counter[0] % nbuf
        st = streams[counter[0] % infl[0]]    # table set k runs on stream k % inflight
        cx = ctxs[counter[0] % infl[0]]       # ... through that stream's context
        counter[0] += 1
        with torch.cuda.stream(st):
            for w in pending[k]:            # this set's previous gather is done
                w.wait()
            pending[k] = []
            tb = bufs[k]
            if ev is not None:
                ev[0].record(st)
            if slots:
                cx.dfs_tables_slots_device(t_src.data_ptr(), per, tb[0].data_ptr())
            elif packed:
                cx.dfs_tables_packed_device(t_src.data_ptr(), per, tb[0].data_ptr())
            elif args.mode == "dfs":
                cx.dfs_tables_device(t_src.data_ptr(), per, tb[0].data_ptr(), tb[1].data_ptr())
            else:
                cx.shortest_tables_device(t_src.data_ptr(), per, tb[0].data_ptr(),
                                          tb[1].data_ptr(), tb[2].data_ptr())
            if ev is not None:
                ev[1].record(st)
            if world > 1 and assemble[0] != "none":   # [sources][V] on every rank / rank 0
                for t, g in zip(tb, gathered[k]):
                    pending[k].append(D.all_gather_rows_async(t, g) if assemble[0] == "all"
                                      else D.gather_rows_to_root(t, g))

    def drain():
        for k in range(nbuf):
            with torch.cuda.stream(streams[k % infl[0]]):
                for w in pending[k]:
                    w.wait()
            pending[k] = []

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    every = max(1, args.event_every)
    for i in range(args.steps):
        step(evs[i] if i % every == 0 else None)
    drain()
    torch.cuda.synchronize(dev)
    for c in ctxs:
        c.synchronize()        # raises if a kernel's bounded wait tripped: tables invalid
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([e0.elapsed_time(e1) for i, (e0, e1) in enumerate(evs)
                             if i % every == 0]))

    ms_per_step = elapsed / args.steps * 1e3
    routes = float(counts.sum()) * float(H)      # every host pair of these sources
    value = routes / (ms_per_step / 1e3)

    def single_step_ms():
        """ONE step alone -- launched, assembled (N > 1) and synchronized: the
        latency a controller waits for one fresh table set.  Median over a
        few repetitions, max over the ranks."""
        reps = max(3, min(20, args.steps))
        drain()
        torch.cuda.synchronize(dev)
        infl[0] = 1
        ts = []
        for _ in range(reps):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            step()
            drain()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        infl[0] = inflight
        ms = float(np.median(ts)) * 1e3
        return _max_min(ms, dev)[0] if world > 1 else ms

    def rate_at(k, reps):
        """Back-to-back steps with k in flight (same assembly), ms per step
        over the ranks' max."""
        drain()
        torch.cuda.synchronize(dev)
        infl[0] = k
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        drain()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        infl[0] = inflight
        ms = (time.perf_counter() - t0) / reps * 1e3
        ms = _max_min(ms, dev)[0] if world > 1 else ms
        return {"steps_in_flight": k, "ms_per_step": ms, "value": routes / (ms / 1e3),
                "steps": reps}

    single_ms = None if args.profile else single_step_ms()
    by_inflight = {str(inflight): {"steps_in_flight": inflight, "ms_per_step": ms_per_step,
                                   "value": value, "steps": args.steps, "headline": True}}
    if inflight > 1 and not args.profile:     # the same ranks, one step at a time
        by_inflight["1"] = rate_at(1, max(args.steps // 2, 10))
    pipelined = None
    set_bytes = sum(t.numel() * t.element_size() for t in bufs[0])
    if world == 1 and inflight == 1 and args.inflight == 0 and 3 * set_bytes <= (4 << 30) \
            and ms_per_step <= 10.0:      # small steps only: 3 more table sets, 30+ steps
        pipelined = pipelined_rate(local, dev, csr, t_src, per, tables, slots, packed,
                                   args.mode, routes, max(args.steps, 30))
        by_inflight["3"] = {k: pipelined[k] for k in ("steps_in_flight", "ms_per_step",
                                                      "value", "steps")}
    multi = None
    if world > 1:
        multi = multi_gpu_extras(args, world, rank, local, dev, csr, srcs, per, packed, slots,
                                 kern_ms, ms_per_step, routes, step, drain, bufs, gathered,
                                 assemble, assembly_check)
        multi["single_step_ms"] = single_ms
        multi["by_inflight"] = by_inflight
        multi["assembly_check"] = assembly_check
        multi["n1_base"] = n1_base(args, rank, local, dev, csr, srcs, tables, slots, packed,
                                   routes, kern_ms * world)
        multi.update(scaling_keys(value, by_inflight, multi["n1_base"], world))
    for c in ctxs[1:]:
        c.close()
    bytes_launch = algorithmic_bytes_per_source(V, E, args.mode, packed) * (hi - lo)
    achieved = bytes_launch / (kern_ms / 1e3) / 1e9
    per_entry = (4 if packed else 8) if args.mode == "dfs" else 10
    compulsory = 4 * (V + 1) + 8 * E + per_entry * V * (hi - lo)
    traffic = None
    layout = "slots" if slots else ("packed" if packed else
                                    ("int32" if args.mode == "dfs" else "u16+int32"))
    if os.path.exists(TRAFFIC_FILE):
        try:
            tf = json.load(open(TRAFFIC_FILE))
            traffic = tf.get("%s/%s%s/N%d" % (args.fabric, args.mode,
                                               "-" + layout if packed else "", world))
        except Exception:   # noqa: BLE001
            traffic = None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "routes/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic (canonical fat-tree, SURVEY.md 8(d))",
        "config": {
            "workload": "%s all-pairs %s route tables (find_route%s)" % (
                args.fabric, args.mode,
                "" if args.mode == "dfs" else "(multiple=True)[0] + dist"),
            "fabric": args.fabric, "V": V, "E": E, "hosts": H, "sources": S,
            "host_pairs_per_step": int(routes), "table_layout": layout,
            "endpoints": "every switch (V x V switch pairs)" if args.all_vertices
                         else "host-bearing switches (host pairs)",
            "source_subset": bool(args.max_sources and S < (V if args.all_vertices
                                                             else len(np.unique(hv)))),
            "parallelism": "sources sharded over %d GPU(s)%s" % (
                world, (" + tables assembled %s over RCCL (double-buffered: step i+1's "
                        "kernel overlaps step i's assembly)" % (
                            "on every rank by all-gather" if args.assemble == "all"
                            else "on rank 0 by point-to-point receives"))
                       if world > 1 and args.assemble != "none" else
                       (" (each rank keeps its shard: no assembly)" if world > 1 else "")),
            "steps_in_flight": inflight,
        },
        "roofline": {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "kernel": ctx.last_kernel(),
            "kernel_ms": kern_ms, "bytes_per_launch": bytes_launch,
            # the compulsory bytes -- CSR (row_ptr, col,
            # port) read once + this launch's tables written once
            "compulsory_bytes": compulsory,
            "compulsory_gbs": compulsory / (kern_ms / 1e3) / 1e9,
            **_measured(traffic, kern_ms),
            **({"note": "bytes_per_launch counts SURVEY.md 8(d)'s algorithmic bytes (the CSR "
                        "once per destination); the plane BFS reads it once per 64 "
                        "destinations (one bit each), so frac is an effective rate and can "
                        "pass 1; hbm_frac is the PMC-measured HBM fraction"}
               if args.mode == "shortest" and ctx.last_kernel().startswith("msbfs_plane")
               else {}),
        },
        "switch_pair_routes_per_s": float(S) * V / (ms_per_step / 1e3),
        "teps": float(hi - lo) * E / (kern_ms / 1e3),
    }
    out["single_step_ms"] = single_ms
    out["by_inflight"] = by_inflight
    if pipelined is not None:
        out["pipelined"] = pipelined
    if multi is not None:
        multi["process_group"] = {"backend": dist.get_backend(),
                                  "world_size": dist.get_world_size()}
        if dist.get_backend() == "nccl":
            multi["rccl_world_size"] = dist.get_world_size()
        multi["devices"] = [{"rank": r, "local": l, "device": d} for r, l, d in devices]
        out["multi_gpu"] = multi
        out["config"]["assemble"] = args.assemble
        out["config"]["assemble_reason"] = ASSEMBLE_REASON[args.assemble]
    if rank == 0 and world == 1 and args.mode == "dfs" and not args.profile and \
            float(S) * V * (4 if packed else 8) <= 4e9:
        # the drop-in's host-buffer boundary: sources in, tables out over PCIe
        # (skipped where the host copy of the tables would exceed 4 GB)
        ctx.set_stream(None)
        reps = max(1, min(5, args.steps))
        t0 = time.perf_counter()
        for _ in range(reps):
            if slots:
                ctx.dfs_tables_slots(srcs)
            elif packed:
                ctx.dfs_tables_packed(srcs)
            else:
                ctx.dfs_tables(srcs, with_hops=False)
        dt = (time.perf_counter() - t0) / reps
        out["host_boundary"] = {
            "value": routes / dt, "unit": "routes/s", "ms_per_call": dt * 1e3,
            "note": "sdnr_dfs_tables%s with host buffers (sources H2D, tables D2H, "
                    "synchronous), not the HBM-resident bench value" % (
                        "_" + layout if packed else "")}
    # fat-trees only: their default routes are ~70 entries; a torus or
    # Jellyfish all-pairs fdb set (~2,400-5,600 entries per pair) is TBs
    if rank == 0 and world == 1 and args.mode == "dfs" and not args.max_sources and \
            not args.no_flows and not args.profile and not args.all_vertices and \
            args.fabric.startswith("fat_tree"):
        # the form the drop-in uses: one u32 word (switch | port << 16) per
        # entry, 4 B; the two int32 arrays (8 B per entry) beside it
        out["materialised_flows"] = materialised_flows(ctx, dev, stream, csr, fabric, srcs,
                                                       packed=True)
        out["materialised_flows_int32"] = materialised_flows(ctx, dev, stream, csr, fabric, srcs)
    if rank == 0 and world == 1 and args.mode == "dfs" and not args.max_sources and \
            not args.no_flows and not args.profile and not args.all_vertices and \
            args.fabric.startswith("fat_tree"):
        out["dropin"] = dropin_block(fabric)
    if world > 1 and not args.no_cpu_baseline and args.mode == "dfs":
        dist.barrier()         # the GPU work of every rank is done: rank 0 alone on the host
    if rank == 0 and not args.no_cpu_baseline and args.mode == "dfs":
        # N > 1 too (north_star: the host-CPU baseline "in the same run"):
        # pthreads and plain loops, no fork, after every rank's timed work
        base, ref, ref_pred = cpu_baseline(fabric, csr, srcs, counts, H, args.cpu_budget_s)
        if "dropin" in out:   # the reference's own cost per query, beside the drop-in's
            out["dropin"]["cpu_reference_ms_per_route"] = 1e3 / ref["value"]
        out["cpu_baseline"] = base
        out["cpu_reference_path"] = ref
        out["cpu_reference_path_pred"] = ref_pred
        if ref_mp is not None:
            out["cpu_reference_path_all_cores"] = ref_mp
        out["gpu_over_cpu"] = value / base["value"]
    if world > 1 and not args.no_cpu_baseline and args.mode == "dfs":
        dist.barrier()
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
