#!/bin/bash
# round-3 A/B: async DFS with the ports kept in LDS by the search (default)
# vs the epilogue's ell_port gathers (SDNROUTE_DFS_PORTLDS=0) vs the build before
OUT=gpurun_out/r5a; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async or k48 or packed or dropin or fullsize_all_host or compact or residency" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="SDNROUTE_LIB=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_base.so"
G="SDNROUTE_DFS_PORTLDS=0"
D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "$B|" "|" "$G|" "$B|" "|" "$G|" \
  "$B|--max-sources 144" "|--max-sources 144" "$G|--max-sources 144" \
  "$B|--max-sources 1" "|--max-sources 1" \
  "$B|$D" "|$D" "$B|$D --max-sources 258" "|$D --max-sources 258"
