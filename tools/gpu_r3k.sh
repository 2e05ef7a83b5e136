#!/bin/bash
# round-3: full GPU suite + default bench + smoke on the current tree
OUT=gpurun_out/r3k; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || exit $?
tail -c 600 $OUT/bench.json
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; exit $rc
