#!/bin/bash
# late sweep: async-DFS waves per workgroup (priority default) on k=48 and
# dragonfly; torus split kernel search waves per workgroup x priority
OUT=gpurun_out/sw
mkdir -p "$OUT"
b() { # tag fabric steps env...
  local tag=$1 fab=$2 st=$3; shift 3
  env "$@" timeout -k 10 150 python bench.py --fabric $fab --steps $st --warmup 2 --no-cpu-baseline --no-flows \
    > "$OUT/$tag.json" 2> "$OUT/$tag.err" || { tail -3 "$OUT/$tag.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$tag.json'));print('$tag', 'kernel %.4f ms'%d['roofline']['kernel_ms'], d['roofline']['kernel'])"
}
for w in 4 3 5 6 4; do
  b k48_w$w fat_tree:48 30 SDNROUTE_DFS_ASYNC_WAVES=$w
  b df_w$w dragonfly:16,8,8 30 SDNROUTE_DFS_ASYNC_WAVES=$w
done
b torus_ns7 torus:32,32,32 2 SDNROUTE_DFS_SPLIT_NS=7
b torus_ns3 torus:32,32,32 2 SDNROUTE_DFS_SPLIT_NS=3
b torus_ns3p torus:32,32,32 2 SDNROUTE_DFS_SPLIT_NS=3 SDNROUTE_DFS_FLAGS=1
