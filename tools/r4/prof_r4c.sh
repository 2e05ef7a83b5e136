#!/bin/bash
# round 4, final: the headline kernel after the next-candidate change
set -u
run() { bash tools/profile_gpu.sh "$@" > gpurun_out/prof_$1.log 2>&1; rc=$?; tail -1 gpurun_out/prof_$1.log
        case $rc in 124|134|137|139) exit $rc;; esac; }
run r04_dfs48p --no-flows
run r04_dfs48p_144 --no-flows --max-sources 144
exit 0
