#!/bin/bash
# round 4: plane BFS -- merged init kernel (SDNROUTE_PLANE_INIT=0: fills + seed)
# and transposed u16 ELL rows in the level pass (SDNROUTE_PLANE_T16=0: int32 rows)
OUT=gpurun_out/r4_c9; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "shortest or plane or ecmp or multiple" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
SDNROUTE_PLANE_INIT=0 SDNROUTE_PLANE_T16=0 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "plane" > $OUT/pytest_sp_old.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp_old.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_new_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_INIT=0 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_noinit_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_T16=0 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_not16_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 200 python bench.py --mode shortest --fabric torus:32,32,32 --steps 5 --warmup 2 > $OUT/sp_new_torus.json 2>> $OUT/err.log || exit $?
SDNROUTE_PLANE_T16=0 timeout -k 10 200 python bench.py --mode shortest --fabric torus:32,32,32 --steps 5 --warmup 2 > $OUT/sp_not16_torus.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$OUT/sp_tl -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/sp_tl.log 2>&1 || exit $?
