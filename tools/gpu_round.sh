#!/bin/bash
# One GPU validation pass (run from the repo root on the GPU box):
#   parity tests (-m gpu), smoke(), the default bench line, the shortest-mode
#   bench line and, when the diagnostic library is built, the search-wave
#   anatomy of the async DFS kernel.  Every GPU step has its own time limit
#   and the script stops at the first fatal status.
# Usage: bash tools/gpu_round.sh TAG [pytest -k expression]
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
K=()
[ -n "${2:-}" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --durations=60 --timeout 300 --timeout-method thread \
  "${K[@]}" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; fatal $rc smoke
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; fatal $rc bench
timeout -k 10 300 python bench.py --mode shortest --steps 10 --warmup 2 --no-cpu-baseline \
  > "$OUT/bench_shortest.json" 2> "$OUT/bench_shortest.err"
rc=$?; echo "bench shortest rc=$rc"; cat "$OUT/bench_shortest.json"; fatal $rc bench_shortest
if [ -f sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_stamps.so ]; then
  timeout -k 10 300 python tools/stamps_async.py fat_tree:48 > "$OUT/stamps.log" 2>&1
  rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; fatal $rc stamps
fi
exit 0
