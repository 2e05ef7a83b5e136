#!/bin/bash
# A/B of kernel variants: ENV specs x fabrics, REPS repetitions each (kernel ms)
OUT=gpurun_out/ab; mkdir -p $OUT
if [ -n "$KEXPR" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$KEXPR" > $OUT/pytest.log 2>&1
  rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" $OUT/pytest.log | head; exit $rc; }
fi
for f in $FABRICS; do
  for spec in "$@"; do
    for r in $(seq ${REPS:-3}); do
      env $spec timeout -k 10 120 python bench.py --fabric $f --steps ${STEPS:-30} --warmup 5 \
        --no-cpu-baseline --no-flows $BARGS > $OUT/b.json 2> $OUT/b.err || { tail $OUT/b.err; exit 1; }
      python -c "import json;d=json.load(open('$OUT/b.json'));print('$f [$spec]', round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), d['roofline']['kernel'])"
    done
  done
done
