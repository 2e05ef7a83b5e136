#!/bin/bash
# round 4: speculative visited gather of the top child (SDNR_ASYNC_SPEC,
# tools/r4/ab/libsdnroute_spec.so) vs the default build: parity, then A/B
OUT=gpurun_out/r4_c8; mkdir -p $OUT
SPEC=$PWD/tools/r4/ab/libsdnroute_spec.so
SDNROUTE_LIB=$SPEC timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_fullsize_parity.py -m gpu -k "dfs or async or tree" > $OUT/pytest_spec.log 2>&1
rc=$?; tail -3 $OUT/pytest_spec.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for ms in 1 144 0; do
    timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/new_${ms}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_LIB=$SPEC timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/spec_${ms}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/new_df.json 2>> $OUT/err.log || exit $?
SDNROUTE_LIB=$SPEC timeout -k 10 200 python bench.py --fabric dragonfly:16,8,8 --no-cpu-baseline --no-flows --steps 20 --warmup 3 > $OUT/spec_df.json 2>> $OUT/err.log || exit $?
# plane BFS: status published by the table kernel into coherent host memory
# (default) vs a D2H copy on the stream (SDNROUTE_PLANE_PUB=0)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "shortest or plane or ecmp" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_pub_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_PUB=0 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_copy_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $GRAFT_REPO_ROOT/$OUT/sp_tl -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/sp_tl.log 2>&1 || exit $?
SDNROUTE_PLANE_PUB=0 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -f csv -d $GRAFT_REPO_ROOT/$OUT/sp_tl0 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --mode shortest --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/sp_tl0.log 2>&1 || exit $?
