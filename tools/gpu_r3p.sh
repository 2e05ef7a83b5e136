#!/bin/bash
# round-3 re-entry: full parity + smoke + default bench lines, then the headline k=48 profile
bash tools/gpu_round.sh r3p || exit $?
mkdir -p gpurun_out/sum
bash tools/profile_gpu.sh r03_dfs48p --no-flows > /dev/null || exit $?
python3 tools/summarize_profile.py gpurun_out/prof_r03_dfs48p gpurun_out/sum/r03_dfs48p > /dev/null || exit 1
rm -rf gpurun_out/prof_r03_dfs48p
echo "profiled r03_dfs48p"
