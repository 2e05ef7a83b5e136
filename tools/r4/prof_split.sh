#!/bin/bash
# round 4: what do the torus / Jellyfish default-route
# waves queue on?  Per workload, one rocprofv3 PMC pass per counter group
# (never combined with tracing), at low and full source counts.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r4_split; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CGROUPS=("VmemLatency" "LdsLatency"
        "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum"
        "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
        "SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD")
run() {  # tag, bench args...
  local tag=$1; shift
  local i=0
  for g in "${CGROUPS[@]}"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $g -f csv -d $OUT/$tag/p$i -o run -- \
      python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-flows "$@" > $OUT/$tag/p$i.log 2>&1
    rc=$?; echo "$tag p$i ($g) rc=$rc"
    case $rc in 124|134|137|139) exit $rc;; esac
  done
}
mkdir -p $OUT/t256 $OUT/tall $OUT/j512 $OUT/jall
run t256 --fabric torus:32,32,32 --max-sources 256
run tall --fabric torus:32,32,32
run j512 --fabric jellyfish:100000,16,1 --max-sources 512
run jall --fabric jellyfish:100000,16,1
exit 0
