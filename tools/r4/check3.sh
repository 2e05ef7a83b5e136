#!/bin/bash
# round 4: APSP sweeps parity + bench; seg-kernel flat stores parity + matflows; latency probe
OUT=gpurun_out/r4_c3; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -k "apsp or route_entries or expand" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --mode apsp --steps 10 --warmup 2 > $OUT/apsp.json 2> $OUT/err.log || exit $?
timeout -k 10 300 python bench.py --mode matflows --steps 3 > $OUT/matflows.json 2>> $OUT/err.log || exit $?
timeout -k 10 60 tools/r4/latency_probe > $OUT/latency.log 2>> $OUT/err.log || exit $?
