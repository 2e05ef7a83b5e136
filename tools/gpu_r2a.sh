#!/bin/bash
# round-2 check: full GPU suite (incl. full-size parity), then a Jellyfish
# shortest-mode probe.  Every GPU step has its own limit; stop at the first failure.
OUT=gpurun_out/r2a
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --durations=25 > $OUT/pytest.log 2>&1
rc=$?; tail -40 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --fabric jellyfish:100000,16,1 --mode shortest \
  --max-sources 4096 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/jf_sp.json 2> $OUT/jf_sp.err
rc=$?; cat $OUT/jf_sp.json; tail -5 $OUT/jf_sp.err
exit $rc
