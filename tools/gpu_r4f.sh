#!/bin/bash
# round-3: N>1 rehearsal (2 ranks on one device, gloo) of the bench path + the new route-entries test
OUT=gpurun_out/r4f; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "route_entries_k48" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/rehearse_multi.sh
