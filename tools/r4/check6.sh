#!/bin/bash
# round 4: bits kernel v2 (batch candidate tests, per-child worker split): parity, anatomy, A/B
OUT=gpurun_out/r4_c6; mkdir -p $OUT
timeout -k 10 60 tools/r4/chain_probe > $OUT/chain.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "dfs_bits" > $OUT/pytest_bits.log 2>&1
rc=$?; tail -3 $OUT/pytest_bits.log; [ $rc -eq 0 ] || exit $rc
BITS_WAVES=4,6,8 timeout -k 10 200 python tools/r4/stamps_bits.py fat_tree:48 1,144,1152 > $OUT/stamps_bits.log 2>&1 || exit $?
for ms in 1 144 0; do
  SDNROUTE_DFS_STRATEGY=bits timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_bits_$ms.json 2>> $OUT/err.log || exit $?
done
for ms in 1 144 0; do
  timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_cur_$ms.json 2>> $OUT/err.log || exit $?
done
timeout -k 10 120 python bench.py --mode shortest --steps 20 --warmup 3 > $OUT/sp48.json 2>> $OUT/err.log || exit $?
timeout -k 10 120 python bench.py --mode shortest --fabric dragonfly:16,8,8 --steps 20 --warmup 3 > $OUT/spdf.json 2>> $OUT/err.log || exit $?
SDNROUTE_PLANE_GUESS=0 timeout -k 10 120 python bench.py --mode shortest --steps 20 --warmup 3 > $OUT/sp48_noguess.json 2>> $OUT/err.log || exit $?
timeout -k 10 300 python bench.py --mode matflows --steps 2 > $OUT/matflows.json 2>> $OUT/err.log || exit $?
SDNROUTE_ROUTE_NT=1 timeout -k 10 300 python bench.py --mode matflows --steps 2 > $OUT/matflows_nt.json 2>> $OUT/err.log || exit $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "shortest or plane or ecmp" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
