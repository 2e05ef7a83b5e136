#!/bin/bash
# Diagnostic library with s_memtime phase stamps (tools/stamps*.py); never
# used for timing claims.  Run after any csrc change before a stamps run.
# It holds the diagnostic DFS variants too (tools/diag/).
cd "$(dirname "$0")/../sdn-mpi-router_amd" && \
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSDNR_STAMPS \
  -DSDNR_DIAG_VARIANTS -Wno-unused-function -Icsrc -o sdnmpi_amd/libsdnroute_stamps.so \
  csrc/*.hip ../tools/diag/*.hip -Wl,-rpath,/opt/rocm/lib
