#!/bin/bash
# round-3: row-prefetch split kernel (dfs_pf_kernel): parity subset, A/B, stamps
# (dfs_pf_kernel and tools/stamps_pf.py were removed after this measurement: DESIGN.md 4.2)
OUT=gpurun_out/r3s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "(small_all_sources and global) or fullsize_sampled" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT/sw '|--fabric torus:32,32,32 --steps 3 --warmup 1' 'SDNROUTE_DFS_PF=1|--fabric torus:32,32,32 --steps 3 --warmup 1' \
  '|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' 'SDNROUTE_DFS_PF=1|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_PF=1 SDNROUTE_DFS_SPLIT_NS=3|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' || exit $?
timeout -k 10 300 python tools/stamps_pf.py torus:32,32,32 256 7168 32768 > $OUT/stamps_torus.log 2>&1; rc=$?; cat $OUT/stamps_torus.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamps_pf.py jellyfish:100000,16,1 512 3840 > $OUT/stamps_jf.log 2>&1; rc=$?; cat $OUT/stamps_jf.log; exit $rc
