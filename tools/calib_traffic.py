#!/usr/bin/env python3
"""Turn the calibration run (tools/gpu_calib.sh) into per-shape factors.

    python tools/calib_traffic.py gpurun_out/calib [profiles/r03_traffic_calibration.json]

For every calib_* kernel of tools/calib_traffic.hip the run log states the
useful bytes it moved and the bytes of the 128-B lines it touched.  The PMC
passes give FETCH_SIZE / WRITE_SIZE (KiB) and the memory-side request counts
TCC_EA0_RDREQ (+ _32B) and TCC_EA0_WRREQ (+ _64B).  Per shape this records

  fetch_factor   = line bytes / FETCH_SIZE bytes        (read shapes)
  read_req_bytes = RDREQ_32B x 32 + (RDREQ - RDREQ_32B) x 128
  write_req_bytes= WRREQ_64B x 64 + (WRREQ - WRREQ_64B) x 32
  write_factor   = write_req_bytes / WRITE_SIZE bytes   (write shapes)
  write_amplification = write_req_bytes / useful bytes

so tools/summarize_profile.py multiplies FETCH_SIZE by the measured read factor
and WRITE_SIZE by the measured write factor instead of a blanket constant."""
import csv
import glob
import json
import os
import sys

READS = ("calib_read16", "calib_rows_u16", "calib_read_u32", "calib_gather_u32")
WRITES = ("calib_write16", "calib_write_u32", "calib_scatter_u32")


def main(src, dst=None):
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
        row.update(c)
        rd, rd32 = c.get("TCC_EA0_RDREQ_sum"), c.get("TCC_EA0_RDREQ_32B_sum", 0.0)
        wr, wr64 = c.get("TCC_EA0_WRREQ_sum"), c.get("TCC_EA0_WRREQ_64B_sum", 0.0)
        if name in READS:
            row["kind"] = "read"
            if c.get("FETCH_SIZE", 0) > 0:
                row["fetch_factor"] = lines / (c["FETCH_SIZE"] * 1024.0)
            if rd is not None:
                row["read_req_bytes"] = rd32 * 32 + (rd - rd32) * 128
        if name in WRITES:
            row["kind"] = "write"
            if wr is not None:
                row["write_req_bytes"] = wr64 * 64 + (wr - wr64) * 32
                row["write_amplification"] = row["write_req_bytes"] / useful
                if c.get("WRITE_SIZE", 0) > 0:
                    row["write_factor"] = row["write_req_bytes"] / (c["WRITE_SIZE"] * 1024.0)
        out[name] = row
    dst = dst or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                              "r03_traffic_calibration.json")
    json.dump(out, open(dst, "w"), indent=1, sort_keys=True)
    for k, v in sorted(out.items()):
        print(k, {x: (round(y, 3) if isinstance(y, float) else y) for x, y in v.items()})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
