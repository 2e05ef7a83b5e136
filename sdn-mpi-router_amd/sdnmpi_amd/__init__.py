"""sdnmpi_amd -- MI355X-native route computation for SDN-MPI Router.

Drop-in replacement for the route hot path of keichi/sdn-mpi-router
(``sdnmpi/util/topology_db.py``): ``sdnmpi_amd.util.topology_db.TopologyDB``
keeps the reference API and computes per-source route tables with
hand-written HIP kernels for gfx950 behind a C ABI (``include/sdnroute.h``).
"""

__version__ = "0.1.0"
