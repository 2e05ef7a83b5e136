#!/bin/bash
# round-3: Jellyfish split-kernel occupancy variants (search waves per workgroup x stack ring)
OUT=gpurun_out/r4g; mkdir -p $OUT
J="--fabric jellyfish:100000,16,1 --steps 2 --warmup 1"
bash tools/sweep_gpu.sh $OUT "|$J" "SDNROUTE_DFS_SPLIT_RING=256|$J" "SDNROUTE_DFS_SPLIT_NS=11 SDNROUTE_DFS_SPLIT_RING=256|$J" \
  "SDNROUTE_DFS_SPLIT_NS=11|$J" "SDNROUTE_DFS_SPLIT_NS=3|$J"
