#!/bin/bash
# round 4: the next candidate chosen in the row step (its row prefetched, one
# ballot -> readlane chain per candidate) vs the previous commit's search
# (tools/r4/ab/libsdnroute_prev.so)
OUT=gpurun_out/${CHK_OUT:-r4_c23}; mkdir -p $OUT
PREV=$PWD/tools/r4/ab/libsdnroute_prev.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py tests/test_events.py tests/test_topologydb_dropin.py -m gpu -k "dfs or async or tree or event or slot or route or pool" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/new_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$PREV timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/prev_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/new_df.json 2>> $OUT/err.log || exit $?
SDNROUTE_LIB=$PREV timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/prev_df.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
STAMPS_WAVES=6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 1 > $OUT/stamps_1.log 2>&1 || exit $?
STAMPS_WAVES=4 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 > $OUT/stamps_all.log 2>&1 || exit $?
