#!/bin/bash
# round-3: bit-plane BFS group-frontier pruning: shortest parity (small fabrics, torus all
# destinations, Jellyfish sample) + A/B on every fabric (SDNROUTE_PLANE_PRUNE=0 = before)
OUT=gpurun_out/r4a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "shortest_small or plane_stride" > $OUT/pytest0.log 2>&1
rc=$?; tail -3 $OUT/pytest0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest and not jellyfish_shortest_all" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
P=SDNROUTE_PLANE_PRUNE=0
bash tools/sweep_gpu.sh $OUT/sw "$P|--fabric torus:32,32,32 --mode shortest --steps 5 --warmup 1" "|--fabric torus:32,32,32 --mode shortest --steps 5 --warmup 1" \
  "$P|--fabric torus:32,32,32 --mode shortest --steps 5 --warmup 1" "|--fabric torus:32,32,32 --mode shortest --steps 5 --warmup 1" \
  "$P|--mode shortest" "|--mode shortest" "$P|--fabric dragonfly:16,8,8 --mode shortest" "|--fabric dragonfly:16,8,8 --mode shortest" \
  "$P|--fabric jellyfish:100000,16,1 --mode shortest --steps 3 --warmup 1" "|--fabric jellyfish:100000,16,1 --mode shortest --steps 3 --warmup 1"
