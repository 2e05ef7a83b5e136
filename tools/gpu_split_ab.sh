#!/bin/bash
# GPU parity (-m gpu) then torus / Jellyfish DFS bench lines.
OUT=${1:-gpurun_out/split}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  ${PYK:+-k "$PYK"} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
for fab in ${FABS:-torus:32,32,32 jellyfish:100000,16,1}; do
  timeout -k 10 300 python bench.py --fabric $fab --steps 2 --warmup 1 --no-cpu-baseline --no-flows \
    > "$OUT/b_$fab.json" 2> "$OUT/b_$fab.err"
  rc=$?; [ $rc -ne 0 ] && { echo "bench $fab rc=$rc"; tail -3 "$OUT/b_$fab.err"; exit $rc; }
  python -c "import json;d=json.load(open('$OUT/b_$fab.json'));print('$fab', 'step %.2f ms'%d['ms_per_step'], 'kernel %.2f ms'%d['roofline']['kernel_ms'], d['roofline']['kernel'])"
done
