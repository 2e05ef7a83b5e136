#!/bin/bash
# round 4: tight explore loop A/B (HEAD dfs.hip = tools/r4/ab/libsdnroute_old.so),
# u32 flow-entry output parity + matflows, then the round's profiles
OUT=gpurun_out/r4_c7; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "dfs or async or tree" > $OUT/pytest_dfs.log 2>&1
rc=$?; tail -3 $OUT/pytest_dfs.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/new_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$PWD/tools/r4/ab/libsdnroute_old.so timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/old_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
for f in dragonfly:16,8,8; do
  timeout -k 10 200 python bench.py --fabric $f --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/new_df.json 2>> $OUT/err.log || exit $?
  SDNROUTE_LIB=$PWD/tools/r4/ab/libsdnroute_old.so timeout -k 10 200 python bench.py --fabric $f --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/old_df.json 2>> $OUT/err.log || exit $?
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_topologydb_dropin.py -m gpu > $OUT/pytest_dropin.log 2>&1
rc=$?; tail -3 $OUT/pytest_dropin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode matflows --steps 3 > $OUT/matflows.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
