#!/bin/bash
# round-3 profiles: dragonfly default route (compact-LDS async kernel), torus shortest (padded
# plane stride), torus and Jellyfish default route (split kernel) -> gpurun_out/sum/r03_*
mkdir -p gpurun_out/sum
prof() {  # tag key kernel-prefix bench-args... (STEPS: steps the run executed, multi-kernel steps)
  local tag=$1 key=$2 kp=$3; shift 3
  bash tools/profile_gpu.sh $tag "$@" > gpurun_out/sum/$tag.profile.log 2>&1 || { cat gpurun_out/sum/$tag.profile.log; exit 1; }
  python3 tools/summarize_profile.py gpurun_out/prof_$tag gpurun_out/sum/$tag $key "$kp" $STEPS > gpurun_out/sum/$tag.sum.log 2>&1 || exit 1
  tail -1 gpurun_out/sum/$tag.sum.log
  rm -rf gpurun_out/prof_$tag
}
prof r03_df_dfs dragonfly:16,8,8/dfs-packed/N1 dfs_async_kernel --fabric dragonfly:16,8,8 --no-flows
STEPS=5 prof r03_torus_sp torus:32,32,32/shortest/N1 "msbfs_plane_level_kernel+msbfs_plane_tables_kernel+msbfs_plane_seed_kernel" --fabric torus:32,32,32 --mode shortest --steps 4 --warmup 1
prof r03_torus_dfs torus:32,32,32/dfs-packed/N1 dfs_split_kernel --fabric torus:32,32,32 --steps 3 --warmup 1
prof r03_jf_dfs jellyfish:100000,16,1/dfs-slots/N1 dfs_split_kernel --fabric jellyfish:100000,16,1 --steps 2 --warmup 1
