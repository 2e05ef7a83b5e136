#!/bin/bash
# round-3: plane-pad parity test; async DFS worker count / compact-LDS sweep at k=48 (1,152 and 144 sources)
OUT=gpurun_out/r3x; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "plane_stride_pad or shortest_small or shortest_fullsize" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|' 'SDNROUTE_DFS_ASYNC_WAVES=3|' 'SDNROUTE_DFS_ASYNC_WAVES=5|' 'SDNROUTE_DFS_C16=1|' '|' \
  '|--max-sources 144' 'SDNROUTE_DFS_ASYNC_WAVES=3|--max-sources 144' 'SDNROUTE_DFS_ASYNC_WAVES=5|--max-sources 144' \
  'SDNROUTE_DFS_ASYNC_WAVES=6|--max-sources 144' 'SDNROUTE_DFS_C16=1|--max-sources 144'
