#!/bin/bash
# A/B bench lines on one box: bash tools/gpu_ab.sh TAG "ENV=.. ENV=..|bench args" ...
# (each spec: env assignments, '|', bench.py args; one JSON line each into
# gpurun_out/TAG/ab.jsonl, the spec in a "spec" key)
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; : > "$OUT/ab.jsonl"
for spec in "$@"; do
  envs=${spec%%|*}; args=${spec#*|}
  line=$(env $envs timeout -k 10 ${TMO:-300} python bench.py $args 2> "$OUT/last.err")
  rc=$?
  echo "{\"spec\": \"$spec\", \"rc\": $rc, \"line\": ${line:-null}}" >> "$OUT/ab.jsonl"
  python3 - "$spec" "$rc" "$line" <<'PY'
import json, sys
spec, rc, line = sys.argv[1], sys.argv[2], sys.argv[3]
try:
    d = json.loads(line); r = d.get("roofline", {})
    print("%-60s rc=%s ms=%.4f kernel_ms=%s %s" % (spec, rc, d["ms_per_step"], r.get("kernel_ms"), r.get("kernel")))
except Exception:
    print(spec, "rc", rc, "no line")
PY
  case $rc in 124|134|137|139) tail -5 "$OUT/last.err"; exit $rc;; esac
done
