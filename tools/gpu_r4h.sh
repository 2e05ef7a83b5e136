#!/bin/bash
# round-3 final profiles: headline k=48 default route (1,152 sources) and one GPU's N=8 share (144)
mkdir -p gpurun_out/sum
prof() {  # tag key kernel-prefix bench-args...
  local tag=$1 key=$2 kp=$3; shift 3
  bash tools/profile_gpu.sh $tag "$@" > gpurun_out/sum/$tag.profile.log 2>&1 || { cat gpurun_out/sum/$tag.profile.log; exit 1; }
  python3 tools/summarize_profile.py gpurun_out/prof_$tag gpurun_out/sum/$tag $key "$kp" > gpurun_out/sum/$tag.sum.log 2>&1 || exit 1
  tail -1 gpurun_out/sum/$tag.sum.log
  rm -rf gpurun_out/prof_$tag
}
prof r03_dfs48p fat_tree:48/dfs-packed/N1 dfs_async_kernel --no-flows
prof r03_dfs48p_144 fat_tree:48/dfs-packed-144/N1 dfs_async_kernel --no-flows --max-sources 144
