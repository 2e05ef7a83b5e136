#!/bin/bash
# round 4: 16-B stores for both flow-entry forms; parity + matflows
OUT=gpurun_out/${CHK_OUT:-r4_c18}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_topologydb_dropin.py tests/test_gpu_parity.py -m gpu -k "route or flow or fdb or expand" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode matflows --steps 3 > $OUT/matflows_v4.json 2>> $OUT/err.log || exit $?
timeout -k 10 200 python bench.py --mode flows --steps 10 --warmup 2 > $OUT/flows1024.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
