#!/bin/bash
set -u
for spec in "jf_sp|--fabric jellyfish:100000,16,1 --mode shortest --steps 2 --warmup 1" \
            "torus_sp|--fabric torus:32,32,32 --mode shortest --steps 3 --warmup 1"; do
  tag=${spec%%|*}; args=${spec#*|}
  bash tools/profile_gpu.sh r02_$tag $args || exit $?
done
exit 0
