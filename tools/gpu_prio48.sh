#!/bin/bash
# k=48 / dragonfly async DFS: search wave at raised issue priority (flags 1) vs not
OUT=gpurun_out/prio
mkdir -p "$OUT"
for rep in 1 2; do
 for fab in fat_tree:48 dragonfly:16,8,8; do
  for fl in 0 1; do
   for ms in 576 0; do
    SDNROUTE_DFS_FLAGS=$fl timeout -k 10 120 python bench.py --fabric $fab --steps 30 --warmup 5 --no-cpu-baseline \
      --no-flows --max-sources $ms > "$OUT/b.json" 2> "$OUT/b.err" || { tail -3 "$OUT/b.err"; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$fab flags=$fl', 'S=%d'%d['config']['sources'], 'kernel %.4f ms'%d['roofline']['kernel_ms'])"
   done
  done
 done
done
