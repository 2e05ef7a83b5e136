#!/bin/bash
# torus DFS: lean vs split search loop (SDNROUTE_DFS_LEAN=0), then GPU parity.
OUT=${1:-gpurun_out/lean}
mkdir -p "$OUT"
for lean in 1 0 1; do
  SDNROUTE_DFS_LEAN=$lean timeout -k 10 200 python bench.py --fabric torus:32,32,32 --steps 2 --warmup 1 \
    --no-cpu-baseline --no-flows > "$OUT/b_$lean.json" 2> "$OUT/b_$lean.err"
  rc=$?; [ $rc -ne 0 ] && { echo "bench lean=$lean rc=$rc"; tail -5 "$OUT/b_$lean.err"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/b_$lean.json'));print('lean=$lean', 'step %.2f ms'%d['ms_per_step'], 'kernel %.2f ms'%d['roofline']['kernel_ms'], d['roofline']['kernel'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${PYK:+-k "$PYK"} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
exit $rc
