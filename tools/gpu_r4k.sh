#!/bin/bash
# round-3 diagnostic: is the Jellyfish default route bound by its rows overflowing an XCD's L2?
# Same degree, half / quarter the vertices (rows 1.8 / 0.9 MB instead of 3.6 MB): split-kernel
# anatomy at the same sources per CU, and the TCC hit rate.
OUT=gpurun_out/r4k; mkdir -p $OUT
for n in 100000 50000 25000; do
  timeout -k 10 300 python tools/stamps_split.py jellyfish:$n,16,1 3840 > $OUT/stamps_$n.log 2>&1 || exit $?
  cat $OUT/stamps_$n.log
done
cd /tmp && export TMPDIR=/tmp
for n in 100000 50000 25000; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -f csv -d $GRAFT_REPO_ROOT/$OUT/pmc_$n -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --fabric jellyfish:$n,16,1 --max-sources 3840 --steps 2 --warmup 1 --no-cpu-baseline \
    > $GRAFT_REPO_ROOT/$OUT/pmc_$n.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT && python - <<'PY'
import csv, glob
for n in (100000, 50000, 25000):
    f = glob.glob("gpurun_out/r4k/pmc_%d/**/run_counter_collection.csv" % n, recursive=True)
    if not f: print(n, "no counters"); continue
    hit = miss = 0.0
    for r in csv.DictReader(open(f[0])):
        if "dfs_split" not in r.get("Kernel_Name", ""): continue
        v = float(r["Counter_Value"])
        if r["Counter_Name"].startswith("TCC_HIT"): hit += v
        elif r["Counter_Name"].startswith("TCC_MISS"): miss += v
    print("jellyfish %d: TCC hit %.3g miss %.3g miss rate %.1f %%" % (n, hit, miss, 100 * miss / max(1, hit + miss)))
PY
