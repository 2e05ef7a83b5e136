#!/bin/bash
# k=48 async DFS: kernel time vs sources (per-CU load) and the LDS counters at
# one source vs all 1,152 (to read SQ_LDS_IDX_ACTIVE against SQ_BUSY_CU_CYCLES)
OUT=gpurun_out/ldsp
mkdir -p "$OUT"
for ms in 144 288 576 864 1152; do
  timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-flows --max-sources $ms \
    > "$OUT/b$ms.json" 2> "$OUT/b$ms.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/b$ms.json'));print('S=$ms', 'kernel %.4f ms'%d['roofline']['kernel_ms'])"
done
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
for ms in 1 1152; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
    -f csv -d "$ROOT/$OUT/pmc$ms" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline \
    --no-flows --max-sources $ms > "$ROOT/$OUT/pmc$ms.log" 2>&1 || exit 1
  python3 - "$ROOT/$OUT/pmc$ms" $ms <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "dfs_async" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print("S=" + sys.argv[2], {k: "%.4g" % (sum(v) / len(v)) for k, v in acc.items()})
PY
done
