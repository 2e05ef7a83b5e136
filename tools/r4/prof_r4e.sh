#!/bin/bash
# round 4, last: one GPU's N=8 share with the 7-worker low-load regime
set -u
bash tools/profile_gpu.sh r04_dfs48p_144 --no-flows --max-sources 144 > gpurun_out/prof_r04_dfs48p_144.log 2>&1
rc=$?; tail -1 gpurun_out/prof_r04_dfs48p_144.log
case $rc in 124|134|137|139) exit $rc;; esac
STAMPS_WAVES=8 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 1 > gpurun_out/r4_stamps_final_1.log 2>&1 || exit $?
exit 0
