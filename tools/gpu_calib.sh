#!/bin/bash
# Known-byte calibration of FETCH_SIZE / WRITE_SIZE (tools/calib_traffic.hip):
# one PMC pass per counter, then tools/calib_traffic.py.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/calib; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $ROOT/tools/calib_traffic > $OUT/run.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c -f csv -d $OUT/$tag -o run -- $ROOT/tools/calib_traffic > $OUT/$tag.log 2>&1
  echo "$c rc=$?"
done
cd $ROOT && python tools/calib_traffic.py $OUT
