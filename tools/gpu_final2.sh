#!/bin/bash
# round-end check plus the dragonfly async-DFS re-profile (priority default)
bash tools/gpu_final.sh || exit $?
mkdir -p gpurun_out/sum
bash tools/profile_gpu.sh r02_df_dfs --fabric dragonfly:16,8,8 --no-flows > /dev/null || exit $?
python3 tools/summarize_profile.py gpurun_out/prof_r02_df_dfs gpurun_out/sum/r02_df_dfs > /dev/null || exit 1
rm -rf gpurun_out/prof_r02_df_dfs
echo "profiled r02_df_dfs"
