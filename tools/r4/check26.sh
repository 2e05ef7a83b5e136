#!/bin/bash
# round 4: table pass with 8 threads per vertex (SDNROUTE_PLANE_Q=8) vs 4
OUT=gpurun_out/r4_c26; mkdir -p $OUT
SDNROUTE_PLANE_Q=8 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "shortest or plane" > $OUT/pytest_q8.log 2>&1
rc=$?; tail -3 $OUT/pytest_q8.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_q4_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_Q=8 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_q8_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
