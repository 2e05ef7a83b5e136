#!/bin/bash
# round-3 end-state validation (after the paired worker rows): full GPU suite, smoke, bench lines,
# dragonfly default-route profile
bash tools/gpu_round.sh r3final2 || exit $?
bash tools/bench_all.sh gpurun_out/r3final2/bench_all.jsonl || exit $?
mkdir -p gpurun_out/sum
bash tools/profile_gpu.sh r03_df_dfs --fabric dragonfly:16,8,8 --no-flows > gpurun_out/sum/r03_df_dfs.profile.log 2>&1 || exit 1
python3 tools/summarize_profile.py gpurun_out/prof_r03_df_dfs gpurun_out/sum/r03_df_dfs dragonfly:16,8,8/dfs-packed/N1 dfs_async_kernel > gpurun_out/sum/r03_df_dfs.sum.log 2>&1 || exit 1
rm -rf gpurun_out/prof_r03_df_dfs
tail -1 gpurun_out/sum/r03_df_dfs.sum.log
