#!/bin/bash
# round-end check of the committed tree: GPU parity, smoke, the default bench
# line, then every bench line (tools/bench_all.sh)
OUT=gpurun_out/final
mkdir -p "$OUT"
bash tools/gpu_round.sh final > "$OUT/round.log" 2>&1
rc=$?; cat "$OUT/round.log" | grep -v "^{" ; [ $rc -ne 0 ] && exit $rc
bash tools/bench_all.sh "$OUT/bench_all.jsonl"
