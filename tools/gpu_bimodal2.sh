#!/bin/bash
# Torus 32^3 shortest tables: kernel trace (no counters) of N separate
# processes, to split each process's step into kernel time and dispatch gaps
# (tools/bimodal_gaps.py).  Usage: bash tools/gpu_bimodal2.sh [N]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bimodal2; mkdir -p $OUT
N=${1:-4}
cd /tmp && export TMPDIR=/tmp
for i in $(seq 1 $N); do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t$i -o run -- \
    python3 $ROOT/bench.py --fabric torus:32,32,32 --mode shortest --steps 6 --warmup 2 \
    --no-cpu-baseline > $OUT/t$i.json 2> $OUT/t$i.err || exit $?
done
cd $ROOT && python tools/bimodal_gaps.py $OUT $N
