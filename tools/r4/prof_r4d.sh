#!/bin/bash
# round 4, final: shortest steps after the compact level planes
set -u
run() { bash tools/profile_gpu.sh "$@" > gpurun_out/prof_$1.log 2>&1; rc=$?; tail -1 gpurun_out/prof_$1.log
        case $rc in 124|134|137|139) exit $rc;; esac; }
run r04_sp48 --mode shortest
run r04_df_sp --mode shortest --fabric dragonfly:16,8,8
exit 0
