#!/bin/bash
# round 4: parity of the new kernels (seg expansion, APSP relax, slot re-slot), then bench lines
OUT=gpurun_out/r4_c1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_topologydb_dropin.py tests/test_events.py tests/test_gpu_parity.py -m gpu \
  -k "route_entries or apsp or slot_layout or expand" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit $?
SDNROUTE_ROUTE_SEG=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_noseg.json 2>> $OUT/bench.err || exit $?
timeout -k 10 120 python bench.py --mode apsp --steps 5 --warmup 1 > $OUT/apsp.json 2>> $OUT/bench.err || exit $?
SDNROUTE_APSP_RELAX=0 timeout -k 10 120 python bench.py --mode apsp --steps 5 --warmup 1 > $OUT/apsp_norelax.json 2>> $OUT/bench.err || exit $?
timeout -k 10 120 python bench.py --mode flows --steps 10 --warmup 2 > $OUT/flows.json 2>> $OUT/bench.err || exit $?
SDNROUTE_ROUTE_SEG=0 timeout -k 10 120 python bench.py --mode flows --steps 10 --warmup 2 > $OUT/flows_noseg.json 2>> $OUT/bench.err || exit $?
