#!/bin/bash
# round 4: box calibration -- default bench line + the N=8 share probe
OUT=gpurun_out/r4_base; mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 200 python bench.py --max-sources 144 --no-cpu-baseline --no-flows > $OUT/b144.json 2>> $OUT/bench.err || exit $?
timeout -k 10 200 python bench.py --max-sources 1 --no-cpu-baseline --no-flows > $OUT/b1.json 2>> $OUT/bench.err || exit $?
