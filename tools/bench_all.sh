#!/bin/bash
# One bench.py line per BASELINE config/mode (N=1).  Usage: bash tools/bench_all.sh OUTFILE
OUT=${1:-gpurun_out/bench_all.jsonl}
mkdir -p "$(dirname "$OUT")"; : > "$OUT"
run() {  # fabric mode steps warmup extra...
  timeout -k 10 ${TMO:-300} python bench.py --fabric "$1" --mode "$2" --steps "$3" --warmup "$4" "${@:5}" >> "$OUT" 2> "$OUT.$1.$2.err"
  rc=$?; echo "$1 $2 rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
}
run mock dfs 50 5
run fat_tree:8 dfs 50 5
run fat_tree:8 shortest 50 5 --no-cpu-baseline
run fat_tree:48 dfs 100 3
run fat_tree:48 dfs 100 3 --layout int32 --no-cpu-baseline
run fat_tree:48 shortest 50 2 --no-cpu-baseline
run fat_tree:48 flows 10 2 --ranks 1024
run fat_tree:48 ecmp 10 2
run fat_tree:48 apsp 5 1
run dragonfly:16,8,8 dfs 50 2
run dragonfly:16,8,8 shortest 20 1 --no-cpu-baseline
TMO=600 run torus:32,32,32 dfs 2 1 --cpu-budget-s 8
TMO=600 run torus:32,32,32 shortest 2 1 --no-cpu-baseline
TMO=900 run jellyfish:100000,16,1 dfs 2 1 --cpu-budget-s 8
TMO=900 run jellyfish:100000,16,1 shortest 3 1 --no-cpu-baseline
exit 0
