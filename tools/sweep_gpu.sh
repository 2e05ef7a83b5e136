#!/bin/bash
# Kernel-variant sweep of bench.py on the GPU box (tuning only; the numbers
# that count come from the default bench line).
# Usage: bash tools/sweep_gpu.sh OUTDIR "ENV=.. ENV=..|bench args" ...
#   each argument: space-separated env assignments, '|', extra bench.py args
OUT=${1:-gpurun_out/sweep}; shift
mkdir -p "$OUT"
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=${spec%%|*}; args=${spec#*|}
  [ "$args" = "$spec" ] && args=""
  env $envs timeout -k 10 180 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $args \
    > "$OUT/s$i.json" 2> "$OUT/s$i.err"
  rc=$?
  case $rc in 124|134|137|139) echo "fatal rc=$rc in [$spec]"; exit $rc;; esac
  python - "$OUT/s$i.json" "$spec" <<'EOF'
import json, sys
try:
    d = json.load(open(sys.argv[1]))
    r = d["roofline"]
    print("%-60s step %.4f ms kernel %.4f ms frac %.3f %s" % (
        sys.argv[2], d["ms_per_step"], r["kernel_ms"], r["frac"], r["kernel"]))
except Exception as e:  # noqa: BLE001
    print("%-60s FAILED (%s)" % (sys.argv[2], e))
EOF
done
exit 0
