#!/bin/bash
# round 5: rocprofv3 kernel-trace + PMC passes of the round's benched kernels
# (tools/profile_gpu.sh per workload; summaries via tools/summarize_profile.py)
set -u
run() { bash tools/profile_gpu.sh "$@" > gpurun_out/prof_$1.log 2>&1; rc=$?; tail -1 gpurun_out/prof_$1.log
        case $rc in 124|134|137|139) exit $rc;; esac; }
run r05_dfs48p --no-flows
run r05_dfs48p_144 --no-flows --max-sources 144
run r05_torus_dfs --fabric torus:32,32,32 --steps 3 --warmup 1
run r05_flows48 --mode matflows --steps 1
exit 0
