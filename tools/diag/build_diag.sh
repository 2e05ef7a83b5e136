#!/bin/bash
# Diagnostic library: the product sources plus the two losing DFS variants
# (dfs_runs.hip, dfs_bits.hip), compiled with
# -DSDNR_DIAG_VARIANTS.  Loaded only through SDNROUTE_LIB (never by the
# product or the driver's tests); tools/diag/test_diag_variants.py checks it.
set -e
cd "$(dirname "$0")/../../sdn-mpi-router_amd"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DSDNR_DIAG_VARIANTS \
  -Wno-unused-function -Icsrc -o sdnmpi_amd/libsdnroute_diag.so csrc/*.hip ../tools/diag/*.hip \
  -Wl,-rpath,/opt/rocm/lib
