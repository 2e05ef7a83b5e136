#!/bin/bash
# Async DFS kernel time at 1, 144 (one GPU's share at N=8) and all sources,
# k=48 and dragonfly, twice per SDNROUTE_DFS_FLAGS value (first used for the
# L2 warm-up A/B, flag 32, since removed; the flags are diagnostics).
OUT=${1:-gpurun_out/warm}
mkdir -p "$OUT"
for fl in 32 0 32 0; do
  for fab in fat_tree:48 dragonfly:16,8,8; do
    for ms in 1 144 0; do
      SDNROUTE_DFS_FLAGS=$fl timeout -k 10 120 python bench.py --fabric $fab --steps 30 --warmup 5 \
        --no-cpu-baseline --no-flows --max-sources $ms > "$OUT/b_${fl}_${fab}_${ms}.json" 2> "$OUT/b_${fl}_${fab}_${ms}.err"
      rc=$?; case $rc in 0) ;; *) echo "rc=$rc flags=$fl $fab $ms"; tail -3 "$OUT/b_${fl}_${fab}_${ms}.err"; exit $rc;; esac
      python -c "import json;d=json.load(open('$OUT/b_${fl}_${fab}_${ms}.json'));print('flags=$fl', '$fab', 'S=%d'%d['config']['sources'], 'step %.4f ms'%d['ms_per_step'], 'kernel %.4f ms'%d['roofline']['kernel_ms'], d['roofline']['kernel'])"
    done
  done
done
