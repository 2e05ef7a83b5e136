#!/bin/bash
# round 6: walker-only / storer-only timing of the pipelined expansion, base
# vs line-owned slots (diagnostic libraries; SDNROUTE_ROUTE_DIAG 1 = no route
# walks, 2 = no entry stores -- the entries are then wrong)
set -u
O=gpurun_out/$1; mkdir -p $O
for lib in base new; do
  for d in 0 1 2 3; do
    SDNROUTE_LIB=tools/ab/libdiag_$lib.so SDNROUTE_ROUTE_PIPE=2,2,4 SDNROUTE_ROUTE_DIAG=$d \
      timeout -k 10 200 python bench.py --mode matflows --steps 2 > $O/d.tmp 2>> $O/err.log
    rc=$?; case $rc in 0) ;; *) echo "$lib diag=$d rc=$rc"; exit $rc;; esac
    python -c "import json; d=json.loads(open('$O/d.tmp').read().strip().splitlines()[-1]); print('$lib', 'diag=$d', [round(x,1) for x in d['all_ms']])" | tee -a $O/diag.txt
  done
done
