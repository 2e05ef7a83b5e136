#!/bin/bash
# round 6: one-pass async-kernel flush (all port gathers before any table
# store) -- async DFS parity, then library A/B (k=48 and dragonfly)
set -u
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_parity.py -x -q \
  --timeout 300 --timeout-method thread -k "async or fat_tree or k48 or dragonfly or speculative" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
for f in fat_tree:48 dragonfly:16,8,8; do
  timeout -k 10 300 python tools/ab_lib_dfs.py --fabric $f tools/ab/libsdnroute_base.so tools/ab/lib_uf12.so \
    tools/ab/lib_uf6.so > $O/ab_$f.log 2> $O/ab_$f.err
  rc=$?; echo "ab $f rc=$rc"; cat $O/ab_$f.log; case $rc in 0) ;; *) exit $rc;; esac
done
