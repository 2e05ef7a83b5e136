#!/bin/bash
# round-3: flow-entry expansion with 1/2/4/8 walks per thread: parity + A/B (flows mode, materialised flows)
OUT=gpurun_out/r4e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "route_entries" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
I=SDNROUTE_ROUTE_IL
bash tools/sweep_gpu.sh $OUT/sw "$I=1|--mode flows --steps 10" "$I=2|--mode flows --steps 10" "$I=4|--mode flows --steps 10" "$I=8|--mode flows --steps 10" \
  "$I=1|--mode flows --steps 10" "$I=4|--mode flows --steps 10"
for il in 1 4 8; do
  SDNROUTE_ROUTE_IL=$il timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/mf$il.json 2> $OUT/mf$il.err || exit $?
  python -c "import json,sys; d=json.load(open('$OUT/mf$il.json'))['materialised_flows']; print('IL=$il materialised flows %.1f ms %.3e pairs/s' % (d['ms'], d['value']))"
done
