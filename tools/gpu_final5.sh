#!/bin/bash
# round-3 end-state validation after the plane-BFS and APSP changes: full GPU
# suite, smoke, default bench, APSP relaxation-check A/B, every config's
# bench line, k=48 shortest profile
bash tools/gpu_round.sh r3final3 || exit $?
bash tools/sweep_gpu.sh gpurun_out/r3final3/apsp "SDNROUTE_APSP_RELAX=0|--mode apsp --steps 5 --warmup 1" \
  "|--mode apsp --steps 5 --warmup 1" "SDNROUTE_APSP_RELAX=0|--mode apsp --steps 5 --warmup 1 --fabric dragonfly:16,8,8" \
  "|--mode apsp --steps 5 --warmup 1 --fabric dragonfly:16,8,8" || exit $?
bash tools/bench_all.sh gpurun_out/r3final3/bench_all.jsonl || exit $?
bash tools/profile_gpu.sh sp48_final --mode shortest > gpurun_out/r3final3/prof.log 2>&1; tail -1 gpurun_out/r3final3/prof.log
