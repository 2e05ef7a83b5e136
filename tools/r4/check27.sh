#!/bin/bash
# round 4: compact level planes (3 when the previous call ended by level 7;
# SDNROUTE_PLANE_DP=8: always 8)
OUT=gpurun_out/r4_c27; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py tests/test_topologydb_dropin.py -m gpu -k "shortest or plane or ecmp or multiple" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_dp3_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_DP=8 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_dp8_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
for f in torus:32,32,32 jellyfish:100000,16,1; do
  t=${f%%:*}
  timeout -k 10 300 python bench.py --mode shortest --fabric $f --steps 3 --warmup 1 > $OUT/sp_dp3_${t}.json 2>> $OUT/err.log || exit $?
  SDNROUTE_PLANE_DP=8 timeout -k 10 300 python bench.py --mode shortest --fabric $f --steps 3 --warmup 1 > $OUT/sp_dp8_${t}.json 2>> $OUT/err.log || exit $?
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
