"""TopologyDB dict state -> dense CSR, with change tracking.

The reference keeps the switch graph as dicts (``sdnmpi/util/topology_db.py``
:14-18): ``switches`` dpid -> Switch, ``links`` src dpid -> dst dpid -> Link,
``hosts`` MAC -> Host.  Its callers mutate them through the methods
(:20-42) AND directly -- the reference tests assign whole dicts and ``del``
entries (``tests/test_topologydb.py:30-61``, :74, :103).  Device tables are
only valid for the graph they were computed on, so the drop-in stores the
three dicts as :class:`TrackedDict` objects (plain ``dict`` subclasses) whose
every mutation, including on the nested ``links[src]`` dicts, bumps a
version counter the route cache compares against.

Limits of the tracking (documented in DESIGN.md): mutating an attribute of a
Link/Host object in place (``link.src.port_no = ...``), or mutating a plain
dict after handing it to the TopologyDB (it is copied on insertion), is not
seen; the reference itself never does either.
"""

import numpy as np

from .topologies import CSR, build_csr

__all__ = ["Versions", "TrackedDict", "export_graph", "GraphExport"]


class Versions(object):
    """Mutation counters of one TopologyDB's three dicts."""

    __slots__ = ("links", "switches", "hosts")

    def __init__(self):
        self.links = 0
        self.switches = 0
        self.hosts = 0

    def key(self):
        return (self.links, self.switches, self.hosts)


class TrackedDict(dict):
    """dict that bumps ``versions.<field>`` on every mutation.

    With ``nested=True`` (the outer ``links`` dict) dict values are stored as
    TrackedDicts reporting to the same counter.
    """

    __slots__ = ("_versions", "_field", "_nested")

    def __init__(self, versions, field, data=None, nested=False):
        dict.__init__(self)
        self._versions = versions
        self._field = field
        self._nested = nested
        if data:
            for k, v in dict(data).items():
                dict.__setitem__(self, k, self._wrap(v))
        self._bump()

    def _bump(self):
        setattr(self._versions, self._field, getattr(self._versions, self._field) + 1)

    def _wrap(self, v):
        if self._nested and isinstance(v, dict) and not (
                isinstance(v, TrackedDict) and v._versions is self._versions):
            return TrackedDict(self._versions, self._field, v)
        return v

    def __setitem__(self, k, v):
        dict.__setitem__(self, k, self._wrap(v))
        self._bump()

    def __delitem__(self, k):
        dict.__delitem__(self, k)
        self._bump()

    def pop(self, *a):
        r = dict.pop(self, *a)
        self._bump()
        return r

    def popitem(self):
        r = dict.popitem(self)
        self._bump()
        return r

    def clear(self):
        dict.clear(self)
        self._bump()

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = default
        return dict.__getitem__(self, k)

    def update(self, *a, **kw):
        for k, v in dict(*a, **kw).items():
            dict.__setitem__(self, k, self._wrap(v))
        self._bump()

    def __ior__(self, other):
        self.update(other)
        return self

    def __reduce__(self):
        return (dict, (dict(self),))


class GraphExport(object):
    """CSR of the switch graph plus the version key it was built from."""

    __slots__ = ("csr", "key", "index")

    def __init__(self, csr, key):
        self.csr = csr
        self.key = key
        self.index = {int(d): i for i, d in enumerate(csr.dpids.tolist())}


def export_graph(links, switches, hosts, key=None):
    """Dense CSR of ``links`` (vertex set = link endpoints, switches and host
    dpids, ascending dpid order; row order = ``sorted(links[u])``, the
    reference's neighbour order, topology_db.py:76; port = ``link.src.port_no``,
    :130)."""
    src, dst, sport = [], [], []
    for u, nbrs in links.items():
        for v, link in nbrs.items():
            src.append(u)
            dst.append(v)
            sport.append(int(link.src.port_no))
    extra = list(switches.keys())
    extra.extend(h.port.dpid for h in hosts.values())
    csr = build_csr(src, dst, np.asarray(sport, np.int64), extra_vertices=extra)
    return GraphExport(csr, key)


def empty_csr():
    return CSR(np.zeros(0, np.uint64), np.zeros(1, np.int32), np.zeros(0, np.int32),
               np.zeros(0, np.int32))
