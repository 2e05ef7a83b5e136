#!/usr/bin/env python3
"""Turn the calibration run (tools/gpu_calib.sh) into per-shape factors:
bytes moved / counter value, for FETCH_SIZE (reads) and WRITE_SIZE (writes),
where "bytes moved" counts whole 128-B lines (what the memory side serves;
a 4-B gather still moves a line).  Writes profiles/r03_traffic_calibration.json
    python tools/calib_traffic.py gpurun_out/calib"""
import csv
import glob
import json
import os
import sys


def main(src):
    known = {}
    for line in open(os.path.join(src, "run.log")):
        if line.startswith("calib_"):
            name, u, l = line.split()
            known[name] = (int(u.split("=")[1]), int(l.split("=")[1]))
    cnt = {}
    for f in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            cnt.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
            cnt[k][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for name, (useful, lines) in known.items():
        c = cnt.get(name, {})
        row = {"useful_bytes": useful, "line_bytes": lines}
        for k, v in c.items():
            row[k] = v
        if "FETCH_SIZE" in c and c["FETCH_SIZE"] > 0:
            row["fetch_factor"] = lines / (c["FETCH_SIZE"] * 1024.0)
        if "WRITE_SIZE" in c and c["WRITE_SIZE"] > 0:
            row["write_factor"] = lines / (c["WRITE_SIZE"] * 1024.0)
        out[name] = row
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                       "r03_traffic_calibration.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in sorted(out.items()):
        print(k, {x: (round(y, 3) if isinstance(y, float) else y) for x, y in v.items()})


if __name__ == "__main__":
    main(sys.argv[1])
