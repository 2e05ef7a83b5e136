#!/bin/bash
# GPU parity (-m gpu) then the async-kernel A/B of tools/gpu_warm_ab.sh.
OUT=${1:-gpurun_out/ab2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${PYK:+-k "$PYK"} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_warm_ab.sh "$OUT"
