OUT=gpurun_out/st; mkdir -p $OUT
timeout -k 10 120 python tools/stamps_async.py fat_tree:48 > $OUT/k48.log 2>&1; cat $OUT/k48.log
timeout -k 10 120 python tools/stamps_async.py fat_tree:48 32 > $OUT/k48_32.log 2>&1; cat $OUT/k48_32.log
timeout -k 10 120 python tools/stamps_async.py dragonfly:16,8,8 > $OUT/df.log 2>&1; cat $OUT/df.log
