#!/bin/bash
# round 4: bits-kernel anatomy (stamps build)
OUT=gpurun_out/r4_c5; mkdir -p $OUT
timeout -k 10 200 python tools/r4/stamps_bits.py fat_tree:48 1,144,1152 > $OUT/stamps_bits.log 2>&1 || exit $?
