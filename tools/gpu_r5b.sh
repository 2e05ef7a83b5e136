#!/bin/bash
# round-3: where the async kernel's search waves land (tools/simd_probe) and
# the role-rotation knob (SDNROUTE_DFS_ROTATE) A/B
OUT=gpurun_out/r5b; mkdir -p $OUT
timeout -k 10 60 tools/simd_probe 1152 4 31792 > $OUT/probe.log 2>&1 || exit $?
timeout -k 10 60 tools/simd_probe 144 6 31792 >> $OUT/probe.log 2>&1 || exit $?
timeout -k 10 60 tools/simd_probe 2064 3 17000 >> $OUT/probe.log 2>&1 || exit $?
cat $OUT/probe.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "|" "SDNROUTE_DFS_ROTATE=1|" "SDNROUTE_DFS_ROTATE=4|" "SDNROUTE_DFS_ROTATE=9|" "SDNROUTE_DFS_ROTATE=6|" \
  "|" "SDNROUTE_DFS_ROTATE=1|" "SDNROUTE_DFS_ROTATE=4|" "SDNROUTE_DFS_ROTATE=9|" \
  "|--max-sources 144" "SDNROUTE_DFS_ROTATE=1|--max-sources 144" "SDNROUTE_DFS_ROTATE=4|--max-sources 144" \
  "|$D" "SDNROUTE_DFS_ROTATE=1|$D" "SDNROUTE_DFS_ROTATE=4|$D"
