#!/bin/bash
# round 4: plane BFS 64-vertex blocks on small launches (SDNROUTE_PLANE_BLOCK=256: the old blocks)
OUT=gpurun_out/r4_c14; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "shortest or plane or ecmp or multiple" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
SDNROUTE_PLANE_BLOCK=64 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "plane" > $OUT/pytest_sp64.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp64.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_b64_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_BLOCK=256 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_b256_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/$OUT/sp_tl -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/sp_tl.log 2>&1 || exit $?
