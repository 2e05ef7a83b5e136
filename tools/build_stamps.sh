#!/bin/bash
# Diagnostic library with s_memtime phase stamps (tools/stamps*.py); never
# used for timing claims.  Run after any csrc change before a stamps run.
cd "$(dirname "$0")/../sdn-mpi-router_amd" && \
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSDNR_STAMPS \
  -Wno-unused-function -o sdnmpi_amd/libsdnroute_stamps.so csrc/*.hip -Wl,-rpath,/opt/rocm/lib
