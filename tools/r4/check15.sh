#!/bin/bash
# round 4: (a) table pass with Q = 4 threads per vertex on small graphs
# (SDNROUTE_PLANE_BLOCK=256: the old blocks); (b) dword-paired worker rows in
# the async DFS (SDNROUTE_DFS_DW=0: one u16 row per child)
OUT=gpurun_out/r4_c15; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "shortest or plane or ecmp or multiple or dfs or async or tree" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_q4_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_BLOCK=256 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_b256_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_dw_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_DFS_DW=0 timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_u16_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
