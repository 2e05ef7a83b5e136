#!/bin/bash
# re-profile the async DFS lines (k=48 headline, dragonfly) on the final kernel
set -u
mkdir -p gpurun_out/sum
P() {
  local tag=$1; shift
  bash tools/profile_gpu.sh "$tag" "$@" > /dev/null || exit $?
  python3 tools/summarize_profile.py "gpurun_out/prof_$tag" "gpurun_out/sum/$tag" > /dev/null || exit 1
  rm -rf "gpurun_out/prof_$tag"
  echo "profiled $tag"
}
P r02_dfs48p --no-flows
P r02_df_dfs --fabric dragonfly:16,8,8 --no-flows
