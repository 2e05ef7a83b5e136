#!/bin/bash
# round-3: pre-swizzled worker rows (per-slot dummies) A/B, parity, upload cost, torus bimodality
OUT=gpurun_out/r3m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact_lds or one_residency or async_waves or fullsize_all_host or packed_fullsize" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|' 'SDNROUTE_DFS_PRESWZ=0|' '|--max-sources 144' 'SDNROUTE_DFS_PRESWZ=0|--max-sources 144' \
  '|--max-sources 1' 'SDNROUTE_DFS_PRESWZ=0|--max-sources 1' '|--fabric dragonfly:16,8,8' 'SDNROUTE_DFS_C16=0|--fabric dragonfly:16,8,8' \
  'SDNROUTE_DFS_C16=0 SDNROUTE_DFS_PRESWZ=0|--fabric dragonfly:16,8,8' || exit $?
timeout -k 10 300 python tools/upload_cost.py > $OUT/upload.log 2>&1; cat $OUT/upload.log
bash tools/gpu_bimodal.sh 4
