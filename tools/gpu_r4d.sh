#!/bin/bash
# round-3: plane BFS level kernel with 1/2/4 vertices per thread: parity + A/B on every fabric
OUT=gpurun_out/r4d; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "plane_stride or shortest_fullsize_torus or shortest_small" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
V=SDNROUTE_PLANE_VPT
T="--fabric torus:32,32,32 --mode shortest --steps 5 --warmup 1"
J="--fabric jellyfish:100000,16,1 --mode shortest --steps 3 --warmup 1"
bash tools/sweep_gpu.sh $OUT/sw "$V=1|$T" "$V=2|$T" "$V=4|$T" "$V=1|$T" "$V=2|$T" "$V=4|$T" \
  "$V=1|--mode shortest" "$V=2|--mode shortest" "$V=4|--mode shortest" \
  "$V=1|--fabric dragonfly:16,8,8 --mode shortest" "$V=2|--fabric dragonfly:16,8,8 --mode shortest" "$V=4|--fabric dragonfly:16,8,8 --mode shortest" \
  "$V=1|$J" "$V=2|$J" "$V=4|$J"
