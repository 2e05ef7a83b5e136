#!/usr/bin/env python3
"""Generate the golden route fixtures by running the REFERENCE itself.

Run in the development container only (needs /root/reference, read-only):

    python tests/golden/make_golden.py            # all fixtures
    python tests/golden/make_golden.py --small    # skip the full-size samples

The reference ``sdnmpi/util/topology_db.py`` needs only
``ryu.ofproto.ofproto_v1_0.OFPP_LOCAL`` from Ryu (not installed, no network):
a three-file stub package is written to a temporary directory OUTSIDE the
repository and put on ``sys.path`` together with ``/root/reference``.  The
stub's only value, 0xfffe, is OpenFlow 1.0's OFPP_LOCAL.

Outputs (data only -- inputs and the reference's outputs):

* ``<name>.npz``  per fabric: the fabric arrays (small fabrics) or the CSR
  digest (full-size fabrics), the host pairs queried, and the fdb lists
  ``find_route`` returned, flattened with offsets; ``multiple=True`` route
  sets where the reference can enumerate them.
* ``scenarios.json``  mutation/edge-case scenarios (deleted switches, deleted
  links, parallel links, switch-local MACs, unknown MACs, directly assigned
  dicts as in the reference tests) with every query's expected result.
"""
import argparse
import json
import os
import random
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "sdn-mpi-router_amd"))

import numpy as np  # noqa: E402

from sdnmpi_amd import topologies as T  # noqa: E402
from sdnmpi_amd.objects import Host, Link, Port, Switch  # noqa: E402

REFERENCE = "/root/reference"


def import_reference():
    stub = tempfile.mkdtemp(prefix="ryu_stub_")
    os.makedirs(os.path.join(stub, "ryu", "ofproto"))
    open(os.path.join(stub, "ryu", "__init__.py"), "w").close()
    open(os.path.join(stub, "ryu", "ofproto", "__init__.py"), "w").close()
    with open(os.path.join(stub, "ryu", "ofproto", "ofproto_v1_0.py"), "w") as f:
        f.write("OFPP_LOCAL = 0xfffe\n")
    sys.path[:0] = [stub, REFERENCE]
    from sdnmpi.util.topology_db import TopologyDB
    return TopologyDB


def flatten(results):
    """list of fdb lists -> (off int64[n+1], dpid int64[m], port int64[m])"""
    off = np.zeros(len(results) + 1, np.int64)
    dp, pt = [], []
    for i, r in enumerate(results):
        for (a, b) in r:
            dp.append(a)
            pt.append(b)
        off[i + 1] = len(dp)
    return off, np.asarray(dp, np.int64), np.asarray(pt, np.int64)


def flatten_multi(results):
    """list (per pair) of list of fdbs -> pair_off, route_off, dpid, port"""
    pair_off = np.zeros(len(results) + 1, np.int64)
    routes = []
    for i, rs in enumerate(results):
        routes.extend(rs)
        pair_off[i + 1] = len(routes)
    route_off, dp, pt = flatten(routes)
    return pair_off, route_off, dp, pt


def fabric_arrays(f):
    return dict(link_src=f.link_src, link_sport=f.link_sport,
                link_dst=f.link_dst, link_dport=f.link_dport,
                host_mac=f.host_mac, host_dpid=f.host_dpid,
                host_port=f.host_port, switches=f.switches)


def run_fabric(TopologyDB, name, fabric, pairs=None, multiple=False,
               store_fabric=True, n_sample=None, seed=0):
    t0 = time.time()
    db = fabric.populate(TopologyDB())
    macs = fabric.host_macs()
    H = len(macs)
    if pairs is None:
        if n_sample is None:
            pairs = [(a, b) for a in range(H) for b in range(H)]
        else:
            rng = random.Random(seed)
            pairs = [(rng.randrange(H), rng.randrange(H)) for _ in range(n_sample)]
    res = [db.find_route(macs[a], macs[b]) for a, b in pairs]
    out = dict(pair_src=np.asarray([a for a, _ in pairs], np.int32),
               pair_dst=np.asarray([b for _, b in pairs], np.int32))
    out["fdb_off"], out["fdb_dpid"], out["fdb_port"] = flatten(res)
    if multiple:
        mres = [db.find_route(macs[a], macs[b], True) for a, b in pairs]
        (out["m_pair_off"], out["m_route_off"], out["m_dpid"],
         out["m_port"]) = flatten_multi(mres)
    csr = fabric.csr()
    out["csr_digest"] = np.array(csr.digest())
    out["V"], out["E"] = np.int64(csr.V), np.int64(csr.E)
    out["name"] = np.array(fabric.name)
    if store_fabric:
        out.update(fabric_arrays(fabric))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print("%-28s pairs=%-6d multiple=%s  %.1fs" % (name, len(pairs), multiple,
                                                   time.time() - t0))


def random_directed(V, E, hosts, seed, dpid_spread=True):
    """Asymmetric links, random ports, sparse dpids, some isolated switches,
    and a parallel link overwritten last-write-wins."""
    rng = random.Random(seed)
    dpids = sorted(rng.sample(range(1, 40 * V), V)) if dpid_spread else \
        list(range(1, V + 1))
    src, sp, dst, dp = [], [], [], []
    for _ in range(E):
        u, v = rng.choice(dpids), rng.choice(dpids)
        if u == v:
            continue
        src.append(u); sp.append(rng.randrange(1, 60))
        dst.append(v); dp.append(rng.randrange(1, 60))
    # parallel link (same ordered pair) added again with another port
    if src:
        src.append(src[0]); sp.append(sp[0] + 100)
        dst.append(dst[0]); dp.append(dp[0])
    macs, hd, hp = [], [], []
    for i in range(hosts):
        macs.append(0x0A0000000000 + i)
        hd.append(rng.choice(dpids))
        hp.append(rng.randrange(1, 60))
    # a host on a switch that has no links at all
    lone = max(dpids) + 7
    macs.append(0x0A0000000000 + hosts)
    hd.append(lone)
    hp.append(3)
    switches = dpids[: max(1, V - 2)]          # two dpids not in switches
    return T.Fabric("random_V%d_E%d_s%d" % (V, E, seed), src, sp, dst, dp,
                    macs, hd, hp, switches, {"V": V, "E": E, "seed": seed})


# --------------------------------------------------------------------------
# scenarios: sequences of mutations + queries on a reference TopologyDB
# --------------------------------------------------------------------------

def apply_op(db, op):
    kind = op[0]
    if kind == "add_switch":
        db.add_switch(Switch(op[1]))
    elif kind == "delete_switch":
        db.delete_switch(Switch(op[1]))
    elif kind == "add_link":
        _, u, pu, v, pv = op
        db.add_link(Link(Port(u, pu), Port(v, pv)))
    elif kind == "delete_link":
        _, u, pu, v, pv = op
        db.delete_link(Link(Port(u, pu), Port(v, pv)))
    elif kind == "add_host":
        _, mac, d, p = op
        db.add_host(Host(mac, Port(d, p)))
    elif kind == "del_links_key":          # `del self.topology.links[k]`
        del db.links[op[1]]
    elif kind == "del_inner_link":         # `del db.links[u][v]`
        del db.links[op[1]][op[2]]
    elif kind == "set_links":              # `db.links = {...}` (test setUp)
        db.links = {int(u): {int(v): Link(Port(int(u), pu), Port(int(v), pv))
                             for v, (pu, pv) in nb.items()}
                    for u, nb in op[1].items()}
    elif kind == "set_hosts":
        db.hosts = {m: Host(m, Port(d, p)) for m, (d, p) in op[1].items()}
    elif kind == "set_switches":
        db.switches = {int(d): Switch(int(d)) for d in op[1]}
    else:
        raise ValueError(kind)


def mock_setup_ops():
    M = ["02:00:00:00:00:0%d" % i for i in (1, 2, 3, 4)]
    links = {1: {2: (2, 2), 3: (3, 3)}, 2: {1: (2, 2), 4: (3, 2)},
             3: {1: (3, 3), 4: (2, 3)}, 4: {2: (2, 3), 3: (3, 2)}}
    return M, [["set_links", {str(u): {str(v): list(pp) for v, pp in nb.items()}
                              for u, nb in links.items()}],
               ["set_hosts", {m: [i + 1, 1] for i, m in enumerate(M)}],
               ["set_switches", [1, 2, 3, 4]]]


def scenarios(TopologyDB):
    out = []
    M, setup = mock_setup_ops()
    local4 = "00:00:00:00:00:04"
    local1 = "00:00:00:00:00:01"
    unknown = "02:00:00:00:00:99"
    allq = [[a, b, m] for a in M + [local4, local1, unknown]
            for b in M + [local4, local1, unknown] for m in (False, True)]
    steps = [
        ("setup", setup),
        ("del_links_1", [["del_links_key", 1]]),
        ("re_add_1_2", [["add_link", 1, 2, 2, 2]]),
        ("re_add_1_3_parallel", [["add_link", 1, 3, 3, 3],
                                 ["add_link", 1, 9, 3, 9]]),
        ("delete_link_3_4", [["delete_link", 3, 2, 4, 3]]),
        ("delete_switch_2_links_stay", [["delete_switch", 2]]),
        ("host_moves_and_new", [["add_host", M[0], 4, 7],
                                ["add_host", "02:00:00:00:00:05", 99, 1]]),
        ("switch_without_links", [["add_switch", 42]]),
        ("del_inner_4_2", [["del_inner_link", 4, 2]]),
    ]
    db = TopologyDB()
    for name, ops in steps:
        for op in ops:
            apply_op(db, op)
        qs = list(allq) + [[M[0], "00:00:00:00:00:2a", False],
                           ["00:00:00:00:00:2a", M[3], False],
                           ["00:00:00:00:00:2a", "00:00:00:00:00:2a", False]]
        res = [db.find_route(a, b, m) for a, b, m in qs]
        out.append({"name": name, "ops": ops,
                    "queries": [[a, b, m, r] for (a, b, m), r in zip(qs, res)]})
    # malformed MAC: the reference raises ValueError from int(mac, 16)
    try:
        db.find_route("zz:00:00:00:00:01", M[1])
        raised = None
    except Exception as e:        # noqa: BLE001
        raised = type(e).__name__
    out.append({"name": "malformed_mac", "ops": [],
                "raises": [["zz:00:00:00:00:01", M[1], raised]]})
    with open(os.path.join(HERE, "scenarios.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    print("scenarios.json: %d steps" % len(out))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--large-only", action="store_true",
                    help="regenerate only the full-size samples")
    args = ap.parse_args()
    TopologyDB = import_reference()
    if args.large_only:
        return large(TopologyDB)

    scenarios(TopologyDB)
    run_fabric(TopologyDB, "mock", T.mock_square(), multiple=True)
    run_fabric(TopologyDB, "fat_tree_k4", T.fat_tree(4), multiple=True)
    run_fabric(TopologyDB, "fat_tree_k8", T.fat_tree(8))
    run_fabric(TopologyDB, "torus_4x4x4", T.torus3d(4, 4, 4))
    run_fabric(TopologyDB, "torus_2x2x2", T.torus3d(2, 2, 2), multiple=True)
    run_fabric(TopologyDB, "torus_5x3x2", T.torus3d(5, 3, 2))
    run_fabric(TopologyDB, "dragonfly_a4_h2_p2", T.dragonfly(4, 2, 2))
    run_fabric(TopologyDB, "jellyfish_n60_r5", T.jellyfish(60, 5, seed=3))
    run_fabric(TopologyDB, "random_V40", random_directed(40, 110, 30, seed=11))
    run_fabric(TopologyDB, "random_V60_dense", random_directed(60, 400, 25, seed=5))
    run_fabric(TopologyDB, "random_V9", random_directed(9, 22, 7, seed=2),
               multiple=True)
    run_fabric(TopologyDB, "random_V12", random_directed(12, 30, 9, seed=4,
                                                         dpid_spread=False),
               multiple=True)
    if args.small:
        return
    large(TopologyDB)


def large(TopologyDB):
    # full-size BASELINE configs: sampled host pairs (the reference needs
    # 2.9 ms/pair at k=48 and ~1-4 s/pair on the torus and Jellyfish; the
    # seeded sequences extend the round-1 samples, whose pairs come first)
    run_fabric(TopologyDB, "fat_tree_k48_sample", T.fat_tree(48),
               store_fabric=False, n_sample=400, seed=48)
    run_fabric(TopologyDB, "dragonfly_a16_h8_p8_sample", T.dragonfly(16, 8, 8),
               store_fabric=False, n_sample=200, seed=16)
    run_fabric(TopologyDB, "torus_32x32x32_sample", T.torus3d(32, 32, 32),
               store_fabric=False, n_sample=72, seed=32)
    run_fabric(TopologyDB, "jellyfish_n100000_r16_sample",
               T.jellyfish(100000, 16, seed=1), store_fabric=False, n_sample=40,
               seed=100)


if __name__ == "__main__":
    main()
