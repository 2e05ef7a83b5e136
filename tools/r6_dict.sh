#!/bin/bash
# round 6: dictionary rows (split kernel) -- parity, then torus A/B
set -u
O=gpurun_out/r6_dict; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "dict or dfs_small_all_sources or torus_dfs" \
  > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
for d in 1 0 1 0; do
  SDNROUTE_DFS_DICT=$d timeout -k 10 200 python bench.py --fabric torus:32,32,32 --steps 3 --warmup 1 \
    --no-cpu-baseline >> $O/torus_ab.jsonl 2>> $O/torus_ab.err
  rc=$?; echo "dict=$d rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
python - <<'PY'
import json
for l in open("gpurun_out/r6_dict/torus_ab.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(r["kernel"], round(r["kernel_ms"], 2), round(d["ms_per_step"], 2), round(r["frac"], 4))
PY
