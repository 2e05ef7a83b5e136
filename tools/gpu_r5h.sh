#!/bin/bash
# round-3: plane BFS queues the levels the previous call on the graph needed
# (ctx->plane_depth) before its first host check; parity + A/B
OUT=gpurun_out/r5h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest or ecmp or dropin" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
G="SDNROUTE_PLANE_GUESS=0"
S="--mode shortest"; D="--fabric dragonfly:16,8,8"
T="--fabric torus:32,32,32 --steps 3 --warmup 1"; J="--fabric jellyfish:100000,16,1 --steps 3 --warmup 1"
bash tools/sweep_gpu.sh $OUT/sw "$G|$S" "|$S" "$G|$S" "|$S" "$G|$S $D" "|$S $D" \
  "$G|$S $T" "|$S $T" "$G|$S $J" "|$S $J" || exit $?
bash tools/profile_gpu.sh sp48_r5h --mode shortest > $OUT/prof.log 2>&1; tail -1 $OUT/prof.log
