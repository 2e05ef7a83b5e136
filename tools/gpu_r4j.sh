#!/bin/bash
# round-3 A/B on one box: paired worker rows as a template case (default lib) vs the build before pairing
OUT=gpurun_out/r4j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async or k48 or packed or dropin or fullsize_all_host or compact or residency" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
B="SDNROUTE_LIB=sdn-mpi-router_amd/sdnmpi_amd/libsdnroute_base.so"
D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "$B|" "|" "$B|" "|" "$B|--max-sources 144" "|--max-sources 144" "$B|$D" "|$D" "$B|$D" "|$D"
