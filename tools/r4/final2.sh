#!/bin/bash
# round 4 end (after the 7-worker low-load regime): whole GPU suite, smoke, default line, N=8-share lines
OUT=gpurun_out/r4_final2; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/default.json 2> $OUT/default.err || exit $?
for ms in 1 144; do
  timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_$ms.json 2>> $OUT/err.log || exit $?
done
timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --max-sources 258 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/df_258.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
