"""Ryu-shaped topology objects (duck types).

The route path reads exactly these attributes of the objects Ryu hands to
``TopologyDB`` (reference ``sdnmpi/util/topology_db.py:20-42``, ``:127-166``):

* ``switch.dp.id``                       (``add_switch`` / ``delete_switch``)
* ``link.src.dpid``, ``link.dst.dpid``,   (``add_link`` / ``delete_link``)
  ``link.src.port_no``                    (``_route_to_fdb`` :130)
* ``host.mac``, ``host.port.dpid``,       (``add_host`` / ``find_route`` :161,:166)
  ``host.port.port_no``                   (``_route_to_fdb`` :136)

The synthetic topology generators (``sdnmpi_amd.topologies``) build fabrics
out of these, and real Ryu objects can be passed instead: nothing else is
required of them.  ``to_dict`` mirrors Ryu's JSON shape loosely so that the
RPC snapshot path (``TopologyDB.to_dict``) works on synthetic fabrics too.
"""

__all__ = ["Datapath", "Switch", "Port", "Host", "Link"]


def _dpid_str(dpid):
    return "%016x" % dpid


class Datapath(object):
    __slots__ = ("id",)

    def __init__(self, id):
        self.id = id


class Port(object):
    __slots__ = ("dpid", "port_no", "name")

    def __init__(self, dpid, port_no, name=None):
        self.dpid = dpid
        self.port_no = port_no
        self.name = name

    def is_reserved(self):
        return self.port_no > 0xff00

    def to_dict(self):
        return {"dpid": _dpid_str(self.dpid), "port_no": "%08x" % self.port_no,
                "name": self.name or ""}

    def __eq__(self, other):
        return (isinstance(other, Port) and self.dpid == other.dpid
                and self.port_no == other.port_no)

    def __hash__(self):
        return hash((self.dpid, self.port_no))

    def __repr__(self):
        return "Port<dpid=%d, port_no=%d>" % (self.dpid, self.port_no)


class Switch(object):
    __slots__ = ("dp", "ports")

    def __init__(self, dpid, ports=None):
        self.dp = Datapath(dpid)
        self.ports = list(ports) if ports else []

    def to_dict(self):
        return {"dpid": _dpid_str(self.dp.id),
                "ports": [p.to_dict() for p in self.ports]}


class Host(object):
    __slots__ = ("mac", "port", "ipv4", "ipv6")

    def __init__(self, mac, port):
        self.mac = mac
        self.port = port
        self.ipv4 = []
        self.ipv6 = []

    def to_dict(self):
        return {"mac": self.mac, "ipv4": self.ipv4, "ipv6": self.ipv6,
                "port": self.port.to_dict()}


class Link(object):
    __slots__ = ("src", "dst")

    def __init__(self, src, dst):
        self.src = src
        self.dst = dst

    def to_dict(self):
        return {"src": self.src.to_dict(), "dst": self.dst.to_dict()}
