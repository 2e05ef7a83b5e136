#!/bin/bash
# round-3: async DFS workers pairing two children per load / ds_sub (in-degree <= 32): parity + A/B
OUT=gpurun_out/r4i; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "small_all_sources and async" > $OUT/pytest0.log 2>&1
rc=$?; tail -2 $OUT/pytest0.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_topologydb_dropin.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "async or k48 or packed or dropin or fullsize_all_host or compact or residency" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
X=SDNROUTE_DFS_PAIR=0
D="--fabric dragonfly:16,8,8"
bash tools/sweep_gpu.sh $OUT/sw "$X|$D" "|$D" "$X|$D" "|$D" "$X|$D --max-sources 258" "|$D --max-sources 258" "$X|--fabric fat_tree:8" "|--fabric fat_tree:8" "|"
