#!/bin/bash
# round 4: worker step size in the 5-worker regime -- dword-paired rows 16
# (default) vs 32 children; dragonfly's paired rows 8 (default) vs 16
OUT=gpurun_out/r4_c29; mkdir -p $OUT
G32=$PWD/tools/r4/ab/libsdnroute_g32.so
P16=$PWD/tools/r4/ab/libsdnroute_p16.so
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "dfs or async or tree" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for L in P16 G32; do
  eval lib=\$$L
  SDNROUTE_LIB=$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu -k "dfs or async" > $OUT/pytest_$L.log 2>&1
  rc=$?; tail -1 $OUT/pytest_$L.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/g16_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
  for ms in 1 144; do
    SDNROUTE_LIB=$G32 timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/g32_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
  for ms in 258 0; do
    timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --max-sources $ms --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/df_p8_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$P16 timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --max-sources $ms --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/df_p16_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
