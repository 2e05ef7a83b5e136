#!/bin/bash
# late round 2: APSP parity (both tilings), APSP tiling A/B, then every bench line
OUT=gpurun_out/r2f
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
  --timeout-method thread -k apsp > "$OUT/pytest_apsp.log" 2>&1
rc=$?; echo "pytest apsp rc=$rc"; tail -3 "$OUT/pytest_apsp.log"; [ $rc -ne 0 ] && exit $rc
for t in sq128 64 sq128 64; do
  SDNROUTE_APSP=$t timeout -k 10 120 python bench.py --mode apsp --steps 5 --warmup 1 > "$OUT/apsp_$t.json" 2>"$OUT/apsp_$t.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/apsp_$t.json'));r=d['roofline'];print('$t', 'step %.3f ms'%d['ms_per_step'], 'kernel %.3f ms'%r['kernel_ms'], r['kernel'], 'passes', r['passes'], 'frac %.3f'%r['frac'])"
done
bash tools/bench_all.sh "$OUT/bench_all.jsonl"
