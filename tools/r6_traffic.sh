#!/bin/bash
# round 6: profiles/r06_* summaries + profiles/traffic.json (the bench lines'
# roofline.traffic) from the gpurun_out/prof_r06_* runs that exist.
# Steps per profiled process: warmup + steps of tools/r6_profiles.sh (bench
# --profile runs nothing else).
S=python3; P=tools/summarize_profile.py
PL="msbfs_plane_init1_kernel+msbfs_plane_level_kernel+msbfs_plane_tables_kernel"
rec() {  # name key prefix [steps]
  d=gpurun_out/prof_r06_$1
  [ -d "$d" ] || { echo "skip $1"; return; }
  $S $P "$d" profiles/r06_$1 "$2" "$3" ${4:-} > /dev/null && echo "ok $1 -> $2"
}
rec dfs48p     "fat_tree:48/dfs-packed/N1"            "dfs_async_kernel"
rec dfs48p_144 "fat_tree:48/dfs-packed/N1/144src"     "dfs_async_kernel"
rec dfs48      "fat_tree:48/dfs/N1"                   "dfs_async_kernel"
rec df_dfs     "dragonfly:16,8,8/dfs-packed/N1"       "dfs_async_kernel"
rec torus_dfs  "torus:32,32,32/dfs-packed/N1"         "dfs_split_kernel"
rec jf_dfs     "jellyfish:100000,16,1/dfs-slots/N1"   "dfs_split_kernel"
rec sp48       "fat_tree:48/shortest/N1"              "$PL" 12
rec df_sp      "dragonfly:16,8,8/shortest/N1"         "$PL" 12
rec torus_sp   "torus:32,32,32/shortest/N1"           "$PL" 3
rec jf_sp      "jellyfish:100000,16,1/shortest/N1"    "$PL" 2
rec ecmp48     "fat_tree:48/ecmp/N1"                  "ecmp_count"
rec apsp48     "fat_tree:48/apsp/N1"                  "apsp_relax8_kernel"
rec rflows48   "fat_tree:48/flows/N1"                 "route_seg"
