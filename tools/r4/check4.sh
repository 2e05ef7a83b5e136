#!/bin/bash
# round 4: parity of the round's kernel changes, then A/B + bench lines
OUT=gpurun_out/r4_c4; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "dfs_bits" > $OUT/pytest_bits.log 2>&1
rc=$?; tail -3 $OUT/pytest_bits.log; [ $rc -eq 0 ] || exit $rc
for ms in 1 144 0; do
  SDNROUTE_DFS_STRATEGY=bits timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_bits_$ms.json 2>> $OUT/err.log || exit $?
done
timeout -k 10 60 tools/r4/latency_probe > $OUT/latency.log 2>> $OUT/err.log || exit $?
for lib in cur wfirst; do
  L=$PWD/sdn-mpi-router_amd/sdnmpi_amd/libsdnroute.so; [ $lib = wfirst ] && L=$PWD/tools/r4/ab/libsdnroute_wfirst.so
  for ms in 1 144 0; do
    SDNROUTE_LIB=$L timeout -k 10 200 python bench.py --max-sources $ms --no-cpu-baseline --no-flows --steps 50 --warmup 5 > $OUT/dfs_${lib}_$ms.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_topologydb_dropin.py tests/test_events.py -m gpu \
  -k "apsp or route_entries or expand or dfs_packed or dfs_tree or dfs_slots or async or switch_fdb or slot_layout or all_host_pairs or scenarios or shortest or plane or ecmp" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread \
  tests/test_fullsize_parity.py -m gpu -k "tree_depth" > $OUT/pytest_large.log 2>&1
rc=$?; tail -3 $OUT/pytest_large.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --mode apsp --steps 10 --warmup 2 > $OUT/apsp.json 2>> $OUT/err.log || exit $?
timeout -k 10 120 python bench.py --mode shortest --steps 20 --warmup 3 > $OUT/sp48.json 2>> $OUT/err.log || exit $?
timeout -k 10 120 python bench.py --mode shortest --fabric dragonfly:16,8,8 --steps 20 --warmup 3 > $OUT/spdf.json 2>> $OUT/err.log || exit $?
timeout -k 10 300 python bench.py --mode matflows --steps 3 > $OUT/matflows.json 2>> $OUT/err.log || exit $?
timeout -k 10 400 python bench.py > $OUT/bench.json 2>> $OUT/err.log || exit $?
