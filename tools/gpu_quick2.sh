#!/bin/bash
# quick check: DFS parity subset + k=48 / dragonfly bench lines (no CPU legs)
OUT=gpurun_out/q2; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${KEXPR:-dfs or multi}" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head -20; exit $rc; }
for f in "fat_tree:48" "dragonfly:16,8,8"; do
  for w in ${WAVES:-4}; do
    SDNROUTE_DFS_ASYNC_WAVES=$w timeout -k 10 120 python bench.py --fabric $f --steps 30 --warmup 5 \
      --no-cpu-baseline --no-flows > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/b.json'));print('$f waves=$w', round(d['ms_per_step'],4), 'ms kernel', round(d['roofline']['kernel_ms'],4), d['roofline']['kernel'], 'frac', round(d['roofline']['frac'],3))"
  done
done
