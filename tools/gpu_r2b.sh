#!/bin/bash
# round-2 profiles of the large-fabric kernels (kernel trace + PMC passes)
set -u
for spec in "torus_dfs|--fabric torus:32,32,32 --mode dfs --steps 3 --warmup 1" \
            "jf_dfs|--fabric jellyfish:100000,16,1 --mode dfs --steps 2 --warmup 1" \
            "df_dfs|--fabric dragonfly:16,8,8 --mode dfs"; do
  tag=${spec%%|*}; args=${spec#*|}
  bash tools/profile_gpu.sh r02_$tag $args || exit $?
done
exit 0
