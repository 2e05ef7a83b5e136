#!/bin/bash
# round 4: workers in the low-load regime with dword-paired rows: 5 (default) vs 4 / 7
OUT=gpurun_out/r4_c30; mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-flows --steps 50 --warmup 5"
for rep in 1 2; do
  for ms in 1 144; do
    timeout -k 10 200 $B --max-sources $ms > $OUT/w6_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_DFS_ASYNC_WAVES=8 SDNROUTE_DFS_DW=1 timeout -k 10 200 $B --max-sources $ms > $OUT/w8_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_DFS_ASYNC_WAVES=5 SDNROUTE_DFS_DW=1 timeout -k 10 200 $B --max-sources $ms > $OUT/w5_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
SDNROUTE_DFS_ASYNC_WAVES=8 SDNROUTE_DFS_DW=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "dfs or async" > $OUT/pytest_w8.log 2>&1
rc=$?; tail -1 $OUT/pytest_w8.log
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
exit $rc
