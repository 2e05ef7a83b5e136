#!/bin/bash
# Profile bench.py on the GPU box with rocprofv3: one kernel-trace/stats pass,
# then one PMC pass per counter group (never combined with tracing domains).
# Usage (from the repo root, on the GPU box):  bash tools/profile_gpu.sh TAG [bench args...]
set -u
TAG=${1:-run}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# --inflight 1: no 3-in-flight 'pipelined' launches in the trace (their
# overlapped durations would mix into the kernel's average); --profile: only
# the 2 warmup + 10 timed steps run (dispatches per step = dispatches / 12)
BENCH=("$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --inflight 1 --profile "$@")
stop_if_fatal() { # GPU fault / abort / segfault / timeout -> stop the script
  case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
  python3 "${BENCH[@]}" > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"; stop_if_fatal $rc trace
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_BUSY_CU_CYCLES" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TOTAL_READ_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -f csv -d "$OUT/pmc$i" -o run -- \
    python3 "${BENCH[@]}" > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc$i ($grp) rc=$rc"; stop_if_fatal $rc "pmc$i"
done
exit 0
