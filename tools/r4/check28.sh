#!/bin/bash
# round 4: 16 children per worker step with dword-paired rows (tools/r4/ab/libsdnroute_g16.so) vs 8
OUT=gpurun_out/r4_c28; mkdir -p $OUT
G16=$PWD/tools/r4/ab/libsdnroute_g16.so
SDNROUTE_LIB=$G16 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "dfs or async" > $OUT/pytest_g16.log 2>&1
rc=$?; tail -3 $OUT/pytest_g16.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ms in 1 144 288; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/g8_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$G16 timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/g16_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
