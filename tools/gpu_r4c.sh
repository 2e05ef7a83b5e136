#!/bin/bash
# round-3 A/B: async DFS epilogue with 12 vertices per thread in flight (libsdnroute_uf12) vs 4 (base)
OUT=gpurun_out/r4c; mkdir -p $OUT
L=sdn-mpi-router_amd/sdnmpi_amd
B="SDNROUTE_LIB=$L/libsdnroute_base.so"; X="SDNROUTE_LIB=$L/libsdnroute_uf12.so"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "async or k48" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_gpu.sh $OUT "$B|" "$X|" "$B|" "$X|" "$B|--max-sources 144" "$X|--max-sources 144" "$B|--layout int32" "$X|--layout int32" \
  "$B|--fabric dragonfly:16,8,8" "$X|--fabric dragonfly:16,8,8" "$B|--fabric dragonfly:16,8,8" "$X|--fabric dragonfly:16,8,8"
