#!/bin/bash
# Quick GPU check during development: a pytest selection, a bench sweep and
# (optionally) the async-DFS anatomy.
# Usage: bash tools/gpu_quick.sh TAG "PYTEST_K" "STAMPS_ARGS|-" SPEC...
#   SPEC as in tools/sweep_gpu.sh ("ENV=.. ENV=..|bench args")
TAG=$1; KEXPR=$2; STAMPS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "$KEXPR" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"
  if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" "$OUT/pytest.log" | head -20; exit $rc; fi
fi
bash tools/sweep_gpu.sh "$OUT" "$@" || exit $?
if [ "$STAMPS" != "-" ]; then
  timeout -k 10 200 python tools/stamps_async.py $STAMPS > "$OUT/stamps.log" 2>&1
  rc=$?; cat "$OUT/stamps.log"; exit $rc
fi
exit 0
