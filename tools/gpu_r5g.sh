#!/bin/bash
# round-3: plane BFS table pass -- 8 destinations per group (lookups issued
# together), padded LDS stride; parity + A/B against the build before
OUT=gpurun_out/r5g; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="SDNROUTE_LIB=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_base.so"
S="--mode shortest"; D="--fabric dragonfly:16,8,8"
T="--fabric torus:32,32,32 --steps 3 --warmup 1"; J="--fabric jellyfish:100000,16,1 --steps 3 --warmup 1"
bash tools/sweep_gpu.sh $OUT/sw "$B|$S" "|$S" "$B|$S" "|$S" "$B|$S $D" "|$S $D" \
  "$B|$S $T" "|$S $T" "$B|$S $J" "|$S $J" || exit $?
bash tools/profile_gpu.sh sp48_r5g --mode shortest > $OUT/prof.log 2>&1; tail -1 $OUT/prof.log
