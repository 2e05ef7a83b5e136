#!/bin/bash
# round-3: bit-plane BFS with 4 lanes per vertex + split table pass on small
# graphs (SDNROUTE_PLANE_SPLIT) -- parity, A/B, kernel trace of k=48 shortest
OUT=gpurun_out/r5c; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
S="--mode shortest"; D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "SDNROUTE_PLANE_SPLIT=0|$S" "|$S" "SDNROUTE_PLANE_SPLIT=0|$S" "|$S" \
  "SDNROUTE_PLANE_SPLIT=0|$S $D" "|$S $D" "|$S --fabric torus:32,32,32 --steps 3 --warmup 1" || exit $?
bash tools/profile_gpu.sh sp48_split --mode shortest > $OUT/prof.log 2>&1; tail -3 $OUT/prof.log
