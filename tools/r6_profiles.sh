#!/bin/bash
# round 6: rocprofv3 kernel-trace + PMC passes (tools/profile_gpu.sh, which
# now carries the read-coalescing group) of the benched kernels named in the
# arguments.  Usage: bash tools/r6_profiles.sh NAME... (see the case below)
set -u
run() { bash tools/profile_gpu.sh "$@" > gpurun_out/prof_$1.log 2>&1; rc=$?; tail -1 gpurun_out/prof_$1.log
        case $rc in 124|134|137|139) exit $rc;; esac; }
for n in "$@"; do
  case $n in
    dfs48p)      run r06_dfs48p --no-flows ;;
    dfs48p_144)  run r06_dfs48p_144 --no-flows --max-sources 144 ;;
    dfs48p_1)    run r06_dfs48p_1 --no-flows --max-sources 1 ;;
    sp48)        run r06_sp48 --mode shortest ;;
    df_dfs)      run r06_df_dfs --fabric dragonfly:16,8,8 ;;
    torus_dfs)   run r06_torus_dfs --fabric torus:32,32,32 --steps 2 --warmup 1 ;;
    jf_dfs)      run r06_jf_dfs --fabric jellyfish:100000,16,1 --steps 1 --warmup 1 ;;
    flows48)     run r06_flows48 --mode matflows --steps 1 ;;
    apsp48)      run r06_apsp48 --mode apsp ;;
    dfs48)       run r06_dfs48 --no-flows --layout int32 ;;
    ecmp48)      run r06_ecmp48 --mode ecmp ;;
    rflows48)    run r06_rflows48 --mode flows ;;
    df_sp)       run r06_df_sp --fabric dragonfly:16,8,8 --mode shortest ;;
    torus_sp)    run r06_torus_sp --fabric torus:32,32,32 --mode shortest --steps 2 --warmup 1 ;;
    jf_sp)       run r06_jf_sp --fabric jellyfish:100000,16,1 --mode shortest --steps 1 --warmup 1 ;;
    *) echo "unknown profile $n"; exit 2 ;;
  esac
done
exit 0
