#!/bin/bash
# round-3 A/B of the LDS-row DFS search anatomy (stamps builds)
OUT=gpurun_out/r3e; mkdir -p $OUT
L32=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_stamps32.so
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/stamps_runs.py fat_tree:48 $N 2>&1 | grep -v amdgpu.ids; r=$?; }
for N in 1 1152; do
  run X=1
  run SDNROUTE_DFS_RUNS_S=1
  run SDNROUTE_DFS_RUNS_S=2
  run SDNROUTE_DFS_FLAGS=$((1 + (4 << 8)))
  run SDNROUTE_DFS_FLAGS=$((1 + (8 << 8)))
  run SDNROUTE_DFS_FLAGS=0
  run SDNROUTE_LIB=$L32
  run SDNROUTE_LIB=$L32 SDNROUTE_DFS_FLAGS=$((1 + (4 << 8)))
done > $OUT/stamps.log 2>&1
cat $OUT/stamps.log
