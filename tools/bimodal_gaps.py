#!/usr/bin/env python3
"""Per process of tools/gpu_bimodal2.sh: the bench step time, the summed
kernel time per step, the idle time between consecutive dispatches (gaps)
and the per-kernel mean durations -- whether a slow process runs slower
kernels or leaves the queue idle between them.
    python tools/bimodal_gaps.py gpurun_out/bimodal2 N"""
import collections
import csv
import glob
import json
import sys


def main(src, n):
    for i in range(1, n + 1):
        try:
            d = json.loads(open("%s/t%d.json" % (src, i)).read().strip().splitlines()[-1])
        except Exception:   # noqa: BLE001
            d = {}
        f = glob.glob("%s/t%d/**/run_kernel_trace.csv" % (src, i), recursive=True)
        if not f:
            print("t%d: no trace" % i)
            continue
        rows = sorted(csv.DictReader(open(f[0])), key=lambda r: int(r["Start_Timestamp"]))
        rows = [r for r in rows if "msbfs" in r["Kernel_Name"]]
        steps = 8.0    # warmup 2 + steps 6
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
        gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(rows, rows[1:])]
        small = [g for g in gaps if g < 200000]      # within a step (< 0.2 ms)
        per = collections.defaultdict(list)
        for r in rows:
            per[r["Kernel_Name"][:48]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print("t%d: bench step %.3f ms | kernels %.3f ms/step, in-step gaps %.3f ms/step "
              "(%d gaps, median %.1f us) | %s" % (
                  i, d.get("ms_per_step", float("nan")), busy / steps / 1e6,
                  sum(small) / steps / 1e6, len(small),
                  sorted(small)[len(small) // 2] / 1e3 if small else 0,
                  ", ".join("%s %d x %.1f us" % (k.split("::")[-1][:26], len(v), sum(v) / len(v) / 1e3)
                            for k, v in per.items())))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
