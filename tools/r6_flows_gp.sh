#!/bin/bash
# round 6: line-owned slots by group size -- parity on the product library,
# then matflows timing per diagnostic library (0 = normal, 1 = no walks,
# 3 = neither walks nor stores)
set -u
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -x -q \
  --timeout 200 --timeout-method thread -k "pipe_edges or line_owned or k48_large_batch or route_entries_runs" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
for lib in base g62 g56 base g62 g56; do
  for d in 0 1 3; do
    SDNROUTE_LIB=tools/ab/libdiag_$lib.so SDNROUTE_ROUTE_PIPE=2,2,4 SDNROUTE_ROUTE_DIAG=$d \
      timeout -k 10 200 python bench.py --mode matflows --steps 2 > $O/d.tmp 2>> $O/err.log
    rc=$?; case $rc in 0) ;; *) echo "$lib diag=$d rc=$rc"; exit $rc;; esac
    python -c "import json; d=json.loads(open('$O/d.tmp').read().strip().splitlines()[-1]); print('$lib', 'diag=$d', [round(x,1) for x in d['all_ms']])" | tee -a $O/diag.txt
  done
done
