#!/bin/bash
# round-3: bit-plane BFS, one workgroup per 64-destination batch running
# every level (msbfs_plane_batch_kernel, SDNROUTE_PLANE_FUSED) -- parity,
# A/B against the per-level launches and the build before, k=48 trace
OUT=gpurun_out/r5e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "shortest" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="SDNROUTE_LIB=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_base.so"; G="SDNROUTE_PLANE_FUSED=0"
S="--mode shortest"; D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "$B|$S" "|$S" "$G|$S" "$B|$S" "|$S" "$G|$S" \
  "$B|$S $D" "|$S $D" "$G|$S $D" "$B|$S --fabric fat_tree:8" "|$S --fabric fat_tree:8" || exit $?
bash tools/profile_gpu.sh sp48_r5e --mode shortest > $OUT/prof.log 2>&1; tail -3 $OUT/prof.log
