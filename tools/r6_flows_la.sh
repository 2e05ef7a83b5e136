#!/bin/bash
# round 6: line-aligned store heads in the flow-entry expansion -- store
# probe, route parity, then matflows A/B against the saved base library
set -u
O=gpurun_out/$1; mkdir -p $O
if [ "${PROBE:-0}" = 1 ]; then
  timeout -k 10 60 ./tools/probes/store_pattern > $O/probe.log 2>&1
  rc=$?; echo "probe rc=$rc"; cat $O/probe.log; case $rc in 0) ;; *) exit $rc;; esac
fi
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py tests/test_topologydb_dropin.py -x -q \
  --timeout 200 --timeout-method thread -k "route or flow or fdb or line_owned" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
for lib in base new base new; do
  if [ $lib = base ]; then export SDNROUTE_LIB=tools/ab/libsdnroute_base.so; else unset SDNROUTE_LIB; fi
  timeout -k 10 200 python bench.py --mode matflows --steps 3 > $O/mf_$lib.tmp 2>> $O/ab.err
  rc=$?; echo "$lib rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  python -c "import json,sys; d=json.loads(open('$O/mf_$lib.tmp').read().strip().splitlines()[-1]); d['lib']='$lib'; print(json.dumps(d))" >> $O/ab.jsonl
  python -c "import json; d=json.loads(open('$O/ab.jsonl').read().splitlines()[-1]); print(d['lib'], d['all_ms'], d['int32_all_ms'])"
done
