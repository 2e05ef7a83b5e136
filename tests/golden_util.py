"""Loading the golden fixtures written by tests/golden/make_golden.py."""
import json
import os

import numpy as np

from sdnmpi_amd import topologies as T
from sdnmpi_amd.objects import Host, Link, Port, Switch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SMALL = ["mock", "fat_tree_k4", "fat_tree_k8", "torus_4x4x4", "torus_2x2x2",
         "torus_5x3x2", "dragonfly_a4_h2_p2", "jellyfish_n60_r5", "random_V40",
         "random_V60_dense", "random_V9", "random_V12"]
MULTI = ["mock", "fat_tree_k4", "torus_2x2x2", "random_V9", "random_V12"]
# full-size BASELINE configs (sampled pairs) and their canonical generators
LARGE = {
    "fat_tree_k48_sample": lambda: T.fat_tree(48),
    "dragonfly_a16_h8_p8_sample": lambda: T.dragonfly(16, 8, 8),
    "torus_32x32x32_sample": lambda: T.torus3d(32, 32, 32),
    "jellyfish_n100000_r16_sample": lambda: T.jellyfish(100000, 16, seed=1),
}


class Golden(object):
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        self.pair_src = self.z["pair_src"]
        self.pair_dst = self.z["pair_dst"]

    def fabric(self):
        z = self.z
        if "link_src" in z:
            return T.Fabric(str(z["name"]), z["link_src"], z["link_sport"], z["link_dst"],
                            z["link_dport"], z["host_mac"], z["host_dpid"], z["host_port"],
                            z["switches"])
        f = LARGE[self.name]()
        assert f.csr().digest() == str(z["csr_digest"]), "generator drifted"
        return f

    def fdb(self, i):
        o, d, p = self.z["fdb_off"], self.z["fdb_dpid"], self.z["fdb_port"]
        return [(int(a), int(b)) for a, b in zip(d[o[i]:o[i + 1]], p[o[i]:o[i + 1]])]

    def has_multi(self):
        return "m_pair_off" in self.z

    def multi(self, i):
        po, ro = self.z["m_pair_off"], self.z["m_route_off"]
        d, p = self.z["m_dpid"], self.z["m_port"]
        out = []
        for r in range(po[i], po[i + 1]):
            out.append([(int(a), int(b)) for a, b in zip(d[ro[r]:ro[r + 1]],
                                                         p[ro[r]:ro[r + 1]])])
        return out

    def __len__(self):
        return int(self.pair_src.shape[0])


def scenarios():
    with open(os.path.join(GOLDEN, "scenarios.json")) as f:
        return json.load(f)


def as_tuples(x):
    """JSON lists -> the reference's tuple shapes."""
    if not x:
        return []
    if isinstance(x[0][0], list):
        return [[tuple(t) for t in r] for r in x]
    return [tuple(t) for t in x]


def apply_op(db, op):
    """Replay one scenario mutation (same vocabulary as make_golden.py)."""
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
    elif kind == "del_links_key":
        del db.links[op[1]]
    elif kind == "del_inner_link":
        del db.links[op[1]][op[2]]
    elif kind == "set_links":
        db.links = {int(u): {int(v): Link(Port(int(u), pu), Port(int(v), pv))
                             for v, (pu, pv) in nb.items()}
                    for u, nb in op[1].items()}
    elif kind == "set_hosts":
        db.hosts = {m: Host(m, Port(d, p)) for m, (d, p) in op[1].items()}
    elif kind == "set_switches":
        db.switches = {int(d): Switch(int(d)) for d in op[1]}
    else:
        raise ValueError(kind)


def host_vertex_rows(fabric):
    """Distinct source vertices of a fabric's hosts and each host's vertex."""
    hv, hp = fabric.host_table()
    srcs = np.unique(hv)
    return srcs, hv, hp
