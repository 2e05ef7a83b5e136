#!/bin/bash
# round-3 end-state validation after the plane-BFS changes: full GPU suite,
# smoke, default bench, every config's bench line, k=48 shortest profile
bash tools/gpu_round.sh r3final3 || exit $?
bash tools/bench_all.sh gpurun_out/r3final3/bench_all.jsonl || exit $?
bash tools/profile_gpu.sh sp48_final --mode shortest > gpurun_out/r3final3/prof.log 2>&1; tail -1 gpurun_out/r3final3/prof.log
