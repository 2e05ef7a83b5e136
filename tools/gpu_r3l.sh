#!/bin/bash
# round-3: dragonfly compact-LDS A/B + its parity, JF split-kernel store
# diagnostics, traffic calibration, multi-GPU rehearsal (gloo, 2 ranks on 1 GPU)
OUT=gpurun_out/r3l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "compact_lds or one_residency or async_waves" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT '|--fabric dragonfly:16,8,8' 'SDNROUTE_DFS_C16=0|--fabric dragonfly:16,8,8' \
  '|' 'SDNROUTE_DFS_C16=1|' 'SDNROUTE_DFS_PRESWZ=0|' '|--max-sources 144' 'SDNROUTE_DFS_PRESWZ=0|--max-sources 144' || exit $?
TMO=400 bash tools/sweep_gpu.sh $OUT/jf '|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_FLAGS=3|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_FLAGS=5|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_FLAGS=9|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' || exit $?
bash tools/gpu_calib.sh || exit $?
bash tools/rehearse_multi.sh || exit $?
exit 0
