#!/bin/bash
# round 4: APSP relax8 parity + A/B; write-bandwidth calibration; materialised-flows profile
OUT=gpurun_out/r4_c2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "apsp" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python bench.py --mode apsp --steps 5 --warmup 1 > $OUT/apsp.json 2> $OUT/err.log || exit $?
SDNROUTE_APSP_RELAX=0 timeout -k 10 120 python bench.py --mode apsp --steps 5 --warmup 1 > $OUT/apsp_norelax.json 2>> $OUT/err.log || exit $?
timeout -k 10 120 python tools/r4/probe_write.py > $OUT/write.log 2>> $OUT/err.log || exit $?
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/mf_trace -o run -- python3 $R/bench.py --mode matflows --steps 2 > $R/$OUT/mf_trace.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/$OUT/mf_pmc1 -o run -- python3 $R/bench.py --mode matflows --steps 1 > $R/$OUT/mf_pmc1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/$OUT/mf_pmc2 -o run -- python3 $R/bench.py --mode matflows --steps 1 > $R/$OUT/mf_pmc2.log 2>&1 || exit $?
timeout -k 10 120 python3 $R/bench.py --mode apsp --steps 3 --warmup 1 > /dev/null 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/$OUT/apsp_trace -o run -- python3 $R/bench.py --mode apsp --steps 5 --warmup 1 > $R/$OUT/apsp_trace.log 2>&1 || exit $?
