#!/bin/bash
# Torus 32^3 shortest-table time across processes (DESIGN.md 4.3's 11.4 vs
# 14.5 ms modes): N separate processes, each timing the plane BFS and
# printing its kernel-side counters of interest; then PMC passes over three
# more processes.  Usage: bash tools/gpu_bimodal.sh [N]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bimodal; mkdir -p $OUT
N=${1:-4}
for i in $(seq 1 $N); do
  timeout -k 10 240 python $ROOT/bench.py --fabric torus:32,32,32 --mode shortest --steps 6 \
    --warmup 2 --no-cpu-baseline > $OUT/run$i.json 2> $OUT/run$i.err || exit $?
  python - $OUT/run$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print("process: step %.3f ms kernel %.3f ms" % (d["ms_per_step"], r["kernel_ms"]))
PY
done
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --stats -f csv -d $OUT/p$i/$tag -o run -- \
      python3 $ROOT/bench.py --fabric torus:32,32,32 --mode shortest --steps 6 --warmup 2 \
      --no-cpu-baseline > $OUT/p$i.$tag.log 2>&1
    echo "p$i $tag rc=$?"
  done
done
exit 0
