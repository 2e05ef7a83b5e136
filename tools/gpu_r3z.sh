#!/bin/bash
# round-3: occupancy-aware decrement-worker count: async parity subset + k=48 / dragonfly lines
OUT=gpurun_out/r3z; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async or k48 or packed or dropin" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|' '|--max-sources 144' '|--max-sources 1' '|--fabric dragonfly:16,8,8' '|--fabric dragonfly:16,8,8 --max-sources 258'
