#!/bin/bash
# round 6: N>1 bench path rehearsed on one GPU (2 gloo ranks, BENCH_DEVICE=0),
# then the profiles of the benched split/async kernels
set -u
mkdir -p gpurun_out/multi6
BENCH_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
  --steps 20 --warmup 2 --cpu-budget-s 8 > gpurun_out/multi6/dfs.json 2> gpurun_out/multi6/dfs.err
rc=$?; echo "multi dfs rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac
bash tools/r6_profiles.sh "$@"
