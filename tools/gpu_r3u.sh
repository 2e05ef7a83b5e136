#!/bin/bash
# round-3: split-writer refactor parity subset + timing; torus plane-stride padding vs the allocation dependence
OUT=gpurun_out/r3u; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "(small_all_sources and global) or fullsize_sampled" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/bimodal_settings.py 8 SDNROUTE_PLANE_PAD=0 SDNROUTE_PLANE_PAD=32 SDNROUTE_PLANE_PAD=64 \
  SDNROUTE_PLANE_PAD=320 SDNROUTE_PLANE_PAD=1000 > $OUT/pad.log 2>&1; rc=$?; cat $OUT/pad.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT/sw '|--fabric torus:32,32,32 --steps 3 --warmup 1' '|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1'
