#!/bin/bash
# dragonfly default-route bench line + profile after the worker-count rule
set -u
mkdir -p gpurun_out/dff gpurun_out/sum
timeout -k 10 300 python bench.py --fabric dragonfly:16,8,8 --steps 10 --warmup 2 > gpurun_out/dff/line.json 2> gpurun_out/dff/line.err || exit 1
bash tools/profile_gpu.sh r02_df_dfs --fabric dragonfly:16,8,8 --no-flows > /dev/null || exit $?
python3 tools/summarize_profile.py gpurun_out/prof_r02_df_dfs gpurun_out/sum/r02_df_dfs > /dev/null || exit 1
rm -rf gpurun_out/prof_r02_df_dfs
echo ok
