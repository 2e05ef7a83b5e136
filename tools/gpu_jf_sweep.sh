#!/bin/bash
# Jellyfish 100k DFS: split-kernel knob sweep (sources per workgroup, stack ring).
OUT=${1:-gpurun_out/jf}
mkdir -p "$OUT"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --fabric jellyfish:100000,16,1 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-flows > "$OUT/b_$tag.json" 2> "$OUT/b_$tag.err"
  rc=$?; [ $rc -ne 0 ] && { echo "bench $tag rc=$rc"; tail -5 "$OUT/b_$tag.err"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/b_$tag.json'));print('$tag', 'step %.1f ms'%d['ms_per_step'], 'kernel %.1f ms'%d['roofline']['kernel_ms'], d['roofline']['kernel'], d['config'].get('table_layout'))"
}
run default X=1
run prio_nt SDNROUTE_DFS_FLAGS=3
run noprio SDNROUTE_DFS_FLAGS=0
