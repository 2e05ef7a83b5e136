#!/bin/bash
# round-3: compact-LDS pre-swizzled rows (dragonfly) A/B + parity subset, torus bimodality probes
OUT=gpurun_out/r3o; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact_lds or one_residency or async_waves or packed_fullsize or async" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|' '|--fabric dragonfly:16,8,8' 'SDNROUTE_DFS_PRESWZ=0|--fabric dragonfly:16,8,8' \
  'SDNROUTE_DFS_C16=0|--fabric dragonfly:16,8,8' '|--fabric dragonfly:16,8,8' 'SDNROUTE_DFS_ASYNC_WAVES=4|--fabric dragonfly:16,8,8' \
  'SDNROUTE_DFS_ASYNC_WAVES=2|--fabric dragonfly:16,8,8' || exit $?
timeout -k 10 300 python tools/bimodal_probe.py 8 > $OUT/probe.log 2>&1; rc=$?; cat $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bimodal2.sh 4
