#!/bin/bash
# round-3: one bench line per config (r03_bench_all) + the torus shortest bimodality probes
OUT=gpurun_out/r3q; mkdir -p $OUT
bash tools/bench_all.sh $OUT/bench_all.jsonl || exit $?
timeout -k 10 300 python tools/bimodal_probe.py 8 > $OUT/probe.log 2>&1; rc=$?; cat $OUT/probe.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bimodal2.sh 4 > $OUT/bimodal2.log 2>&1; rc=$?; cat $OUT/bimodal2.log; exit $rc
