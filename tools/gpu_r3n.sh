#!/bin/bash
# round-3: pre-swizzle dummies inside the count padding (5 workgroups per CU at k=48) A/B + async parity subset
OUT=gpurun_out/r3n; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact_lds or one_residency or async_waves or packed_fullsize or async" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|' 'SDNROUTE_DFS_PRESWZ=0|' '|' 'SDNROUTE_DFS_PRESWZ=0|' '|--max-sources 144' 'SDNROUTE_DFS_PRESWZ=0|--max-sources 144' \
  '|--max-sources 1' 'SDNROUTE_DFS_PRESWZ=0|--max-sources 1' '|--fabric dragonfly:16,8,8' 'SDNROUTE_DFS_C16=0|--fabric dragonfly:16,8,8' \
  'SDNROUTE_DFS_ASYNC_WAVES=3|' 'SDNROUTE_DFS_ASYNC_WAVES=5|' || exit $?
