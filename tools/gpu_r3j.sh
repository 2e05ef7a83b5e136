#!/bin/bash
# round-3: async G A/B, then the full Jellyfish parity tests
OUT=gpurun_out/r3j; mkdir -p $OUT
L=sdn-mpi-router_amd/sdnmpi_amd
bash tools/sweep_gpu.sh $OUT '|' "SDNROUTE_LIB=$L/libsdnroute_g32.so|" '|--max-sources 1' "SDNROUTE_LIB=$L/libsdnroute_g32.so|--max-sources 1" '|--max-sources 144' "SDNROUTE_LIB=$L/libsdnroute_g32.so|--max-sources 144" '|--fabric dragonfly:16,8,8' "SDNROUTE_LIB=$L/libsdnroute_g32.so|--fabric dragonfly:16,8,8" || exit $?
timeout -k 10 900 python -u -m pytest tests/test_fullsize_parity.py -m gpu -x -v --timeout 600 --timeout-method thread -k "jellyfish_dfs_slots_all or jellyfish_shortest_all" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log; exit $rc
