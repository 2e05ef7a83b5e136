#!/bin/bash
# round-3 last validation: full GPU suite, smoke, default and shortest bench lines
bash tools/gpu_round.sh r3final3
