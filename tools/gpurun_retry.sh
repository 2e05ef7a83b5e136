#!/bin/bash
# Run a gpurun call, re-submitting it only when gpurun reports an
# infrastructure-side transient (no box / evicted / busy pod: nothing ran,
# nothing charged).  A command that ran -- whatever its exit status -- is
# never re-submitted.  Usage: tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TMO=$2; CMD=$3
for i in 1 2 3 4 5 6 7 8; do
  timeout $((TMO + 1500)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then sleep 150; continue; fi
  exit 0
done
