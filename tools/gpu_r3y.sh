#!/bin/bash
# round-3: async DFS decrement-worker count vs resident sources (k=48, dragonfly)
OUT=gpurun_out/r3y; mkdir -p $OUT
A=SDNROUTE_DFS_ASYNC_WAVES
bash tools/sweep_gpu.sh $OUT "$A=4|--max-sources 1" "$A=6|--max-sources 1" "$A=4|--max-sources 256" "$A=6|--max-sources 256" \
  "$A=4|--max-sources 288" "$A=6|--max-sources 288" "$A=4|--max-sources 576" "$A=6|--max-sources 576" \
  "$A=5|--max-sources 576" "$A=4|--max-sources 144" "$A=6|--max-sources 144" "$A=8|--max-sources 144" "$A=8|--max-sources 1" "$A=8|--max-sources 256" \
  "$A=3|--fabric dragonfly:16,8,8 --max-sources 258" "$A=4|--fabric dragonfly:16,8,8 --max-sources 258" \
  "$A=6|--fabric dragonfly:16,8,8 --max-sources 258" "$A=3|--fabric dragonfly:16,8,8" "$A=4|--fabric dragonfly:16,8,8"
