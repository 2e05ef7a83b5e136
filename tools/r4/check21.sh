#!/bin/bash
# round 4: children's counts read with the visited words (default) vs in the
# push (tools/r4/ab/libsdnroute_late.so, -DSDNR_CNT_LATE)
OUT=gpurun_out/r4_c21; mkdir -p $OUT
LATE=$PWD/tools/r4/ab/libsdnroute_late.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "dfs or async or tree" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/early_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$LATE timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/late_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/early_df.json 2>> $OUT/err.log || exit $?
SDNROUTE_LIB=$LATE timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/late_df.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
