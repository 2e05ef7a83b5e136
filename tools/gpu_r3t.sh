#!/bin/bash
# round-3: row-prefetch split kernel with J-slot windows: parity subset, A/B, stamps of both split
# (dfs_pf_kernel and tools/stamps_pf.py were removed after this measurement: DESIGN.md 4.2)
# kernels; Jellyfish / torus store-flag sweep; plane-chunk placement probe
OUT=gpurun_out/r3t; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "(small_all_sources and global) or fullsize_sampled" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT/sw '|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' 'SDNROUTE_DFS_PF=1|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_PF=1 SDNROUTE_DFS_SPLIT_NS=3|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  'SDNROUTE_DFS_FLAGS=3|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' 'SDNROUTE_DFS_FLAGS=5|--fabric jellyfish:100000,16,1 --steps 2 --warmup 1' \
  '|--fabric torus:32,32,32 --steps 3 --warmup 1' 'SDNROUTE_DFS_FLAGS=2|--fabric torus:32,32,32 --steps 3 --warmup 1' \
  'SDNROUTE_DFS_FLAGS=4|--fabric torus:32,32,32 --steps 3 --warmup 1' || exit $?
timeout -k 10 300 python tools/stamps_pf.py jellyfish:100000,16,1 512 3840 > $OUT/stamps_pf_jf.log 2>&1; rc=$?; cat $OUT/stamps_pf_jf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamps_split.py jellyfish:100000,16,1 512 3840 > $OUT/stamps_jf.log 2>&1; rc=$?; cat $OUT/stamps_jf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stamps_split.py torus:32,32,32 256 7168 32768 > $OUT/stamps_torus.log 2>&1; rc=$?; cat $OUT/stamps_torus.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bimodal_chunk.py 8 64 56 48 40 32 > $OUT/chunk.log 2>&1; rc=$?; cat $OUT/chunk.log; exit $rc
