#!/bin/bash
# round 6: the N > 1 bench path as 2 gloo ranks on one GPU (BENCH_DEVICE=0;
# RCCL refuses two ranks on one device), both assembly forms and the
# shortest mode; every key of the N > 1 line is produced, the values are
# meaningless (gloo moves the tables through host memory).  Usage:
# bash tools/r6_rehearse.sh ["MODE ASSEMBLE" ...]
set -u
O=gpurun_out/r6_multi; mkdir -p $O
[ $# -eq 0 ] && set -- "dfs root" "dfs all" "shortest root"
for spec in "$@"; do
  set -- $spec
  BENCH_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
    --steps 10 --warmup 2 --cpu-budget-s 4 --mode $1 --assemble $2 > $O/$1_$2.json 2> $O/$1_$2.err
  rc=$?; echo "$1 $2 rc=$rc"; case $rc in 0) ;; *) tail -5 $O/$1_$2.err; exit $rc;; esac
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6_multi/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); m = d["multi_gpu"]
    print(f, d["config"]["assemble"], m["assembly_check"], sorted(k for k in m if k not in ("devices",)),
          "cpu" if d.get("cpu_baseline") else "no-cpu")
PY
