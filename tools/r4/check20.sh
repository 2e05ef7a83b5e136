#!/bin/bash
# round 4: worker count x dword-paired rows at the 1,152-source headline
OUT=gpurun_out/r4_c20; mkdir -p $OUT
B="python bench.py --no-cpu-baseline --no-flows --steps 50 --warmup 5"
for cfg in "4 0" "4 1" "3 0" "3 1" "5 0" "5 1"; do
  set -- $cfg
  SDNROUTE_DFS_ASYNC_WAVES=$1 SDNROUTE_DFS_DW=$2 timeout -k 10 200 $B > $OUT/w$1_dw$2.json 2>> $OUT/err.log || exit $?
done
SDNROUTE_DFS_ASYNC_WAVES=3 SDNROUTE_DFS_DW=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_fullsize_parity.py -m gpu -k "dfs and 48" > $OUT/pytest_w3dw.log 2>&1
rc=$?; tail -3 $OUT/pytest_w3dw.log
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
exit $rc
