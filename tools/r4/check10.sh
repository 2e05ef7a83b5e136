#!/bin/bash
# round 4: torus shortest regression hunt (round-3 library vs current, knobs),
# contention probe, stamps anatomy of the async DFS kernel
OUT=gpurun_out/r4_c10; mkdir -p $OUT
R3=$PWD/tools/r4/ab/libsdnroute_r3.so
B="python bench.py --mode shortest --fabric torus:32,32,32 --steps 5 --warmup 2"
SDNROUTE_LIB=$R3 timeout -k 10 200 $B > $OUT/torus_r3.json 2>> $OUT/err.log || exit $?
timeout -k 10 200 $B > $OUT/torus_cur.json 2>> $OUT/err.log || exit $?
SDNROUTE_PLANE_INIT=0 SDNROUTE_PLANE_PUB=0 timeout -k 10 200 $B > $OUT/torus_cur_oldinit_copy.json 2>> $OUT/err.log || exit $?
SDNROUTE_PLANE_GUESS=0 timeout -k 10 200 $B > $OUT/torus_cur_noguess.json 2>> $OUT/err.log || exit $?
SDNROUTE_LIB=$R3 timeout -k 10 200 python bench.py --mode shortest --steps 20 --warmup 3 > $OUT/k48_r3.json 2>> $OUT/err.log || exit $?
timeout -k 10 60 tools/r4/contention_probe > $OUT/contention.log 2>&1 || exit $?
STAMPS_WAVES=4 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 > $OUT/stamps_all.log 2>&1 || exit $?
STAMPS_WAVES=6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 144 > $OUT/stamps_144.log 2>&1 || exit $?
STAMPS_WAVES=6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 1 > $OUT/stamps_1.log 2>&1 || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$OUT/torus_tl -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --fabric torus:32,32,32 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$OUT/torus_tl.log 2>&1 || exit $?
