#!/bin/bash
# round 4: 16-B stores of the u32 flow entries (SDNROUTE_ROUTE_V4=0: 4-B stores)
OUT=gpurun_out/r4_c17; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_topologydb_dropin.py -m gpu > $OUT/pytest_dropin.log 2>&1
rc=$?; tail -3 $OUT/pytest_dropin.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode matflows --steps 3 > $OUT/matflows_v4.json 2>> $OUT/err.log || exit $?
SDNROUTE_ROUTE_V4=0 timeout -k 10 400 python bench.py --mode matflows --steps 3 > $OUT/matflows_v1.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
