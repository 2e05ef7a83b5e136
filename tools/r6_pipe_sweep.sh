#!/bin/bash
# round 6: walker / storer shapes of the pipelined expansion on the final
# library (all-pairs u32 flow entries, bench --mode matflows)
set -u
O=gpurun_out/$1; mkdir -p $O
for rep in 1 2; do
  for sh in 2,2,4 2,2,3 4,4,2 8,4,2 3,3,2 4,2,2 2,2,2; do
    SDNROUTE_ROUTE_PIPE=$sh timeout -k 10 200 python bench.py --mode matflows --steps 2 > $O/t.tmp 2>> $O/err.log
    rc=$?; case $rc in 0) ;; *) echo "$sh rc=$rc"; exit $rc;; esac
    python -c "import json; d=json.loads(open('$O/t.tmp').read().strip().splitlines()[-1]); print('$sh', [round(x,1) for x in d['all_ms']])" | tee -a $O/sweep.txt
  done
done
