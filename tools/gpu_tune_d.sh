#!/bin/bash
# Tuning pass: shortest-mode parity, kernel-variant sweep, async-DFS anatomy
# with one source per CU.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k shortest > gpurun_out/d_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/d_pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep_gpu.sh gpurun_out/sweep_d \
  "SDNROUTE_SP_VARIANT=0|--mode shortest" "SDNROUTE_SP_VARIANT=1|--mode shortest" \
  "SDNROUTE_SP_VARIANT=2|--mode shortest" "SDNROUTE_SP_STRATEGY=msbfs|--mode shortest" \
  "SDNROUTE_SP_VARIANT=0|--mode shortest --fabric dragonfly:16,8,8" \
  "SDNROUTE_SP_VARIANT=2|--mode shortest --fabric dragonfly:16,8,8" "X=1|" || exit $?
timeout -k 10 200 python tools/stamps_async.py fat_tree:48 256 > gpurun_out/d_stamps256.log 2>&1
rc=$?; cat gpurun_out/d_stamps256.log; exit $rc
