#!/bin/bash
# round 6: split kernel (batched writer, dictionary rows) -- parity, then A/B
# lines: torus dict on/off, Jellyfish.  Usage: bash tools/r6_split.sh TAG [pytest -k]
set -u
O=gpurun_out/$1; mkdir -p $O
K=${2:-"dict or dfs_small_all_sources or torus_dfs or jellyfish_dfs or slots_large or depth_large or split_wide or sampled_sources"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -x -q \
  --timeout 400 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
for d in 1 0; do
  SDNROUTE_DFS_DICT=$d timeout -k 10 200 python bench.py --fabric torus:32,32,32 --steps 3 --warmup 1 \
    --no-cpu-baseline >> $O/ab.jsonl 2>> $O/ab.err
  rc=$?; echo "torus dict=$d rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
timeout -k 10 300 python bench.py --fabric jellyfish:100000,16,1 --steps 2 --warmup 1 \
  --no-cpu-baseline >> $O/ab.jsonl 2>> $O/ab.err
rc=$?; echo "jellyfish rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
python - "$O" <<'PY'
import json, sys
for l in open(sys.argv[1] + "/ab.jsonl"):
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["fabric"], r["kernel"], round(r["kernel_ms"], 2), round(d["ms_per_step"], 2), round(r["frac"], 4))
PY
