#!/bin/bash
# round 4: level pass with 4 batches per block on small graphs
# (SDNROUTE_PLANE_BPB=1: one batch per block); default line's flows warm-up fix; N>1 rehearsal
OUT=gpurun_out/r4_c22; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -m gpu -k "shortest or plane or ecmp or multiple" > $OUT/pytest_sp.log 2>&1
rc=$?; tail -3 $OUT/pytest_sp.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for f in fat_tree:48 dragonfly:16,8,8; do
    t=${f%%:*}
    timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_bpb4_${t}_$rep.json 2>> $OUT/err.log || exit $?
    SDNROUTE_PLANE_BPB=1 timeout -k 10 120 python bench.py --mode shortest --fabric $f --steps 20 --warmup 3 > $OUT/sp_bpb1_${t}_$rep.json 2>> $OUT/err.log || exit $?
  done
done
timeout -k 10 600 python bench.py > $OUT/default.json 2>> $OUT/err.log || exit $?
python tools/r4/summ.py $OUT > $OUT/summary.txt 2>&1 || true
bash tools/rehearse_multi.sh > $OUT/multi.log 2>&1 || exit $?
