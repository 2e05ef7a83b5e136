#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks on device 0, gloo
# instead of RCCL (RCCL refuses two ranks on one device).
mkdir -p gpurun_out/multi
for mode in dfs shortest; do
  BENCH_DEVICE=0 BENCH_DIST_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
    --steps 10 --warmup 2 --mode $mode > gpurun_out/multi/$mode.json 2> gpurun_out/multi/$mode.err
  rc=$?; echo "$mode rc=$rc"; cat gpurun_out/multi/$mode.json; tail -5 gpurun_out/multi/$mode.err
  case $rc in 124|134|137|139) exit $rc;; esac
done
