#!/bin/bash
# round-3: async DFS table entries written by the decrement workers: async parity subset + A/B
OUT=gpurun_out/r4b; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "small_all_sources and async" > $OUT/pytest0.log 2>&1
rc=$?; tail -3 $OUT/pytest0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async or k48 or packed or dropin or fullsize_all_host or compact or residency" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
W=SDNROUTE_DFS_WTAB=0
bash tools/sweep_gpu.sh $OUT/sw "$W|" "|" "$W|" "|" "$W|--max-sources 144" "|--max-sources 144" "$W|--layout int32" "|--layout int32" \
  "$W|--fabric dragonfly:16,8,8" "|--fabric dragonfly:16,8,8" "$W|--fabric dragonfly:16,8,8" "|--fabric dragonfly:16,8,8"
