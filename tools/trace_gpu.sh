#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench.py invocation.
# Usage (repo root, GPU box): bash tools/trace_gpu.sh TAG [bench args...]
TAG=${1:-run}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline "$@" > "$OUT/bench.log" 2>&1
rc=$?; echo "trace rc=$rc"
python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print("%-70s calls %5s avg %10.1f us total %10.1f us" % (
        r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e3))
PY
exit $rc
