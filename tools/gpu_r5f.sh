#!/bin/bash
# round-3: plane BFS level pass -- speculative row loads (opt bit 0) and
# return-less atomic-OR plane updates (bit 1), SDNROUTE_PLANE_OPT A/B
OUT=gpurun_out/r5f; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
S="--mode shortest"; D="--fabric dragonfly:16,8,8"
T="--fabric torus:32,32,32 --steps 3 --warmup 1"; J="--fabric jellyfish:100000,16,1 --steps 3 --warmup 1"
O=SDNROUTE_PLANE_OPT
bash tools/sweep_gpu.sh $OUT/sw "$O=0|$S" "$O=1|$S" "$O=2|$S" "$O=3|$S" "$O=0|$S" "$O=3|$S" \
  "$O=0|$S $D" "$O=1|$S $D" "$O=2|$S $D" "$O=3|$S $D" \
  "$O=0|$S $T" "$O=1|$S $T" "$O=2|$S $T" "$O=3|$S $T" "$O=0|$S $J" "$O=2|$S $J" "$O=3|$S $J"
