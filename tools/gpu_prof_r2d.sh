#!/bin/bash
# round-2 re-profiles of the kernels changed late in the round (async DFS,
# Jellyfish split DFS at raised priority, plane BFS chunking / level loops);
# each run is summarized on the box (tools/summarize_profile.py) and its raw
# rocprofv3 output removed, so gpurun_out stays small enough to copy back
set -u
mkdir -p gpurun_out/sum
P() {
  local tag=$1; shift
  bash tools/profile_gpu.sh "$tag" "$@" || exit $?
  python3 tools/summarize_profile.py "gpurun_out/prof_$tag" "gpurun_out/sum/$tag" > /dev/null || exit 1
  rm -rf "gpurun_out/prof_$tag"
}
P r02_dfs48p --no-flows
P r02_df_dfs --fabric dragonfly:16,8,8 --no-flows
P r02_jf_dfs --fabric jellyfish:100000,16,1 --steps 2 --warmup 1 --no-flows
P r02_torus_sp --fabric torus:32,32,32 --mode shortest --steps 2 --warmup 1
P r02_jf_sp --fabric jellyfish:100000,16,1 --mode shortest --steps 2 --warmup 1
P r02_df_sp --fabric dragonfly:16,8,8 --mode shortest
exit 0
