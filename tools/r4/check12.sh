#!/bin/bash
# round 4: torus shortest, round-3 library vs current -- kernel traces
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4_c12; mkdir -p $OUT
R3=$GRAFT_REPO_ROOT/tools/r4/ab/libsdnroute_r3.so
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/cur -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --fabric torus:32,32,32 --steps 3 --warmup 1 > $OUT/cur.log 2>&1 || exit $?
SDNROUTE_LIB=$R3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/r3 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --fabric torus:32,32,32 --steps 3 --warmup 1 > $OUT/r3.log 2>&1 || exit $?
