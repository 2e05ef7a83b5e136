#!/bin/bash
# GPU round trip used during development: DFS/drop-in parity tests, then a
# kernel-variant sweep of bench.py.  Usage: bash tools/gpu_check.sh OUTDIR
OUT=${1:-gpurun_out/check}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -q -x \
  --timeout 300 -k "dfs or dropin or Reference or scenarios or pairs or tables" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
for st in ${SWEEP:-async4 async3 async2 count2 coop}; do
  case $st in
    async*) export SDNROUTE_DFS_STRATEGY=async SDNROUTE_DFS_ASYNC_WAVES=${st#async};;
    count*) export SDNROUTE_DFS_STRATEGY=count SDNROUTE_DFS_COUNT_WAVES=${st#count};;
    *) export SDNROUTE_DFS_STRATEGY=$st;;
  esac
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_$st.json" 2> "$OUT/bench_$st.err" || exit 3
  python -c "import json;d=json.load(open('$OUT/bench_$st.json'));print('$st', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.3g'%d['value'], round(d['roofline']['frac'],3), d['roofline']['kernel'])"
done
