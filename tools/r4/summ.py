"""Summarise the bench JSON lines of a gpurun_out directory (round-4 helper)."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.loads(open(f).read().strip().split("\n")[-1])
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    r = j.get("roofline", {})
    extra = ""
    if "materialised_flows" in j:
        m = j["materialised_flows"]
        extra += " matflows %.1f ms" % m["ms"]
    if "materialised_flows_packed" in j:
        extra += " packed %.1f ms" % j["materialised_flows_packed"]["ms"]
    if "packed_all_ms" in j:
        extra += " packed_all_ms %s" % ["%.1f" % x for x in j["packed_all_ms"]]
    if "materialised_flows_int32" in j:
        extra += " int32 %.1f ms" % j["materialised_flows_int32"]["ms"]
    if "int32_all_ms" in j:
        extra += " int32_all_ms %s" % ["%.1f" % x for x in j["int32_all_ms"]]
    if "all_ms" in j:
        extra += " all_ms %s" % ["%.1f" % x for x in j["all_ms"]]
    print("%-24s ms/step %8.4f kern %8.4f frac %.3f %s%s" % (
        os.path.basename(f), j.get("ms_per_step", 0), r.get("kernel_ms", 0) or 0,
        r.get("frac", 0) or 0, r.get("kernel", ""), extra))
