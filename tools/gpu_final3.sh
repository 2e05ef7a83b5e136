#!/bin/bash
# round-3 end-state validation: full GPU suite, smoke, default bench line, one line per config
bash tools/gpu_round.sh r3final || exit $?
bash tools/bench_all.sh gpurun_out/r3final/bench_all.jsonl
