#!/bin/bash
# round 4, late: re-profile the kernels changed after tools/r4/prof_r4.sh
# (plane table pass with 4 threads per vertex; dword-paired worker rows at
# <= 2 sources per CU), plus the dragonfly shortest step
set -u
run() { bash tools/profile_gpu.sh "$@" > gpurun_out/prof_$1.log 2>&1; rc=$?; tail -1 gpurun_out/prof_$1.log
        case $rc in 124|134|137|139) exit $rc;; esac; }
run r04_sp48 --mode shortest
run r04_dfs48p_144 --no-flows --max-sources 144
run r04_df_sp --mode shortest --fabric dragonfly:16,8,8
exit 0
