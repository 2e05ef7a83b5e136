#!/bin/bash
# round-3 A/B: async DFS with the prefetched rows kept u16 across the back-edge (libsdnroute_xp16)
# vs the committed kernel (libsdnroute_base), alternating, same box
OUT=gpurun_out/r3w; mkdir -p $OUT
L=sdn-mpi-router_amd/sdnmpi_amd
B="SDNROUTE_LIB=$L/libsdnroute_base.so"; X="SDNROUTE_LIB=$L/libsdnroute_xp16.so"
bash tools/sweep_gpu.sh $OUT "$B|" "$X|" "$B|" "$X|" "$B|--max-sources 144" "$X|--max-sources 144" \
  "$B|--max-sources 1" "$X|--max-sources 1" "$B|--fabric dragonfly:16,8,8" "$X|--fabric dragonfly:16,8,8" \
  "$B|--fabric dragonfly:16,8,8" "$X|--fabric dragonfly:16,8,8"
