#!/bin/bash
# round-3: LDS-row DFS workers per slot / children per worker step (stamps)
OUT=gpurun_out/r3h; mkdir -p $OUT
run() { echo "== N=$N $*"; env "$@" timeout -k 10 120 python tools/stamps_runs.py fat_tree:48 $N 2>&1 | grep -v amdgpu.ids; }
{
for N in 1 144; do
  for S in 3 5 7; do run SDNROUTE_DFS_RUNS_S=$S; run SDNROUTE_DFS_RUNS_S=$S SDNROUTE_DFS_FLAGS=$((1 + (32 << 8))); done
done
N=1152; run X=1; run SDNROUTE_DFS_FLAGS=$((1 + (32 << 8)))
run SDNROUTE_DFS_RUNS_SLOTS=3 SDNROUTE_DFS_RUNS_S=3
run SDNROUTE_DFS_RUNS_SLOTS=3 SDNROUTE_DFS_RUNS_S=3 SDNROUTE_DFS_FLAGS=$((1 + (32 << 8)))
} > $OUT/stamps.log 2>&1
cat $OUT/stamps.log
