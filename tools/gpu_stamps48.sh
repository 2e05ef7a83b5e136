#!/bin/bash
OUT=gpurun_out/r3st; mkdir -p $OUT
STAMPS_WAVES=4,6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 > $OUT/k48_all.log 2>&1; cat $OUT/k48_all.log
STAMPS_WAVES=4,6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 144 > $OUT/k48_144.log 2>&1; cat $OUT/k48_144.log
STAMPS_WAVES=4,6 timeout -k 10 200 python tools/stamps_async.py fat_tree:48 1 > $OUT/k48_1.log 2>&1; cat $OUT/k48_1.log
