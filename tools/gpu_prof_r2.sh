#!/bin/bash
# round-2 profiles: one tools/profile_gpu.sh run (kernel trace + 7 PMC passes)
# per bench line; usage: bash tools/gpu_prof_r2.sh TAG:ARGS ...
for spec in "$@"; do
  tag=${spec%%:*}; args=${spec#*:}
  bash tools/profile_gpu.sh r02_$tag $args || exit $?
done
exit 0
