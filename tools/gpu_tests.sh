#!/bin/bash
# A subset of the GPU suite on the box: bash tools/gpu_tests.sh TAG 'pytest args...'
# then (optional) one default bench line when BENCH=1.
TAG=${1:-t}; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --durations=20 --timeout 300 --timeout-method thread "$@" \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"
case $rc in 124|134|137|139) exit $rc;; esac
[ $rc -ne 0 ] && exit $rc
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
  rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
fi
exit $rc
