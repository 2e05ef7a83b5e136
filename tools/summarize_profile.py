#!/usr/bin/env python3
"""Summarize a tools/profile_gpu.sh output directory into profiles/.

    python tools/summarize_profile.py gpurun_out/prof_TAG profiles/r01_TAG

Writes <out>_kernel_stats.csv (rocprofv3 --kernel-trace --stats, verbatim),
<out>_pmc.json (per-dispatch means of every PMC counter, per kernel) and
<out>_summary.md (human-readable, with the HBM traffic derived from
FETCH_SIZE / WRITE_SIZE (KiB per dispatch) with the factors measured by the
known-byte calibration of tools/calib_traffic.hip, profiles/
r03_traffic_calibration.json: every read shape the route kernels use -- 16-B
and 4-B coalesced reads, u16 128-B rows, 4-B random gathers -- is fetched as
128-B requests that FETCH_SIZE tallies at 64 B (factor 2.0); WRITE_SIZE equals
the bytes of the memory-side write requests for both coalesced stores (64-B
requests) and scattered 4-B stores (32-B masked requests, 8x the useful bytes),
factor 1.0).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


CALIBRATION = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles",
                           "r03_traffic_calibration.json")


def factors(path=CALIBRATION):
    """(fetch, write) multipliers from the calibration file: the median over
    the read shapes of line bytes / FETCH_SIZE bytes, and over the write
    shapes of request bytes / WRITE_SIZE bytes.  A shape whose counter
    disagrees with its request count by more than 2x (a kernel the compiler
    thinned) is left out."""
    try:
        cal = json.load(open(path))
    except (OSError, ValueError):
        return 2.0, 1.0     # MI355X_MICROARCH.md's gfx950 correction
    def med(xs, default):
        xs = sorted(xs)
        return xs[len(xs) // 2] if xs else default
    rd = [r["fetch_factor"] for r in cal.values() if r.get("kind") == "read" and
          "fetch_factor" in r and r.get("read_req_bytes") and
          0.5 < r["read_req_bytes"] / r["line_bytes"] < 2.0]
    wr = [r["write_factor"] for r in cal.values() if r.get("kind") == "write" and "write_factor" in r]
    return med(rd, 2.0), med(wr, 1.0)


FETCH_FACTOR, WRITE_FACTOR = factors()


def hbm_bytes(c):
    """Corrected HBM bytes per dispatch from a counter dict (KiB values)."""
    return (FETCH_FACTOR * c.get("FETCH_SIZE", 0.0) + WRITE_FACTOR * c.get("WRITE_SIZE", 0.0)) * 1024.0


def coalescing(c):
    """Read-coalescing figures of one kernel (north_star: "rocprof counters
    must show coalesced CSR reads"), from the per-dispatch counter means:
    * tag_lookups_per_vmem: L1 (TCP) cache-line tag lookups per wavefront
      memory instruction, TCP_TOTAL_CACHE_ACCESSES / (SQ_INSTS_VMEM_RD +
      SQ_INSTS_VMEM_WR).  The TCP looks a 64-lane instruction up one
      quarter-wave at a time, so 4 is the floor: every quarter-wave in ONE
      128-B line (a u16 row of 64 lanes, or 4-B words of 32 consecutive
      lanes); a 16-B-per-lane copy is 8; a gather with every lane in its own
      line is 64 (measured: rocclr's copy kernel 9.3, dfs_async 4.3);
    * l2_req_per_vmem_rd: TCP->L2 read requests per wavefront load
      (TCP_TCC_READ_REQ / SQ_INSTS_VMEM_RD): what leaves the CU's L1;
    * l1_read_hit: 1 - TCP_TCC_READ_REQ / TCP_TOTAL_READ (TCP_TOTAL_READ
      counts read accesses, hits included)."""
    out = collections.OrderedDict()
    req = c.get("TCP_TCC_READ_REQ_sum")
    vm = c.get("SQ_INSTS_VMEM_RD")
    tags = c.get("TCP_TOTAL_CACHE_ACCESSES_sum")
    if tags is not None and vm:
        out["tag_lookups_per_vmem"] = tags / (vm + c.get("SQ_INSTS_VMEM_WR", 0.0))
    if req is not None and vm:
        out["l2_req_per_vmem_rd"] = req / vm
    rd = c.get("TCP_TOTAL_READ_sum")
    if rd and req is not None:
        out["l1_read_hit"] = 1.0 - req / rd
    return out


def main(src, out):
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, out + "_kernel_stats.csv")
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {x: r[x] for x in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                        "VGPR_Count", "SGPR_Count", "Scratch_Size")}
    # dispatches: the fewest values of any counter (a counter listed in two
    # passes -- SQ_INSTS_LDS -- has one value per dispatch per pass)
    pmc = {k: {"meta": meta[k], "counters": {c: sum(v) / len(v) for c, v in cs.items()},
               "dispatches": min(len(v) for v in cs.values())}
           for k, cs in per.items()}
    json.dump(pmc, open(out + "_pmc.json", "w"), indent=1, sort_keys=True)
    lines = ["# rocprofv3 summary: %s" % os.path.basename(out), ""]
    if os.path.exists(stats):
        lines += ["## kernel trace (--kernel-trace --stats)", "", "| kernel | calls | avg us | min us | max us |",
                  "|---|---|---|---|---|"]
        for r in csv.DictReader(open(stats)):
            lines.append("| %s | %s | %.1f | %.1f | %.1f |" % (
                r["Name"][:90], r["Calls"], float(r["AverageNs"]) / 1e3,
                float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3))
    for k, d in pmc.items():
        if "rocclr" in k:
            continue
        c = d["counters"]
        lines += ["", "## %s" % k[:120], "", "launch: %s" % d["meta"], ""]
        for name in sorted(c):
            lines.append("- %s: %.4g per dispatch" % (name, c[name]))
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            lines.append("- HBM traffic per dispatch (FETCH_SIZE x %.3g + WRITE_SIZE x %.3g, "
                         "factors measured by tools/calib_traffic.hip): %.1f MB"
                         % (FETCH_FACTOR, WRITE_FACTOR, hbm_bytes(c) / 1e6))
        co = coalescing(c)
        if co:
            lines.append("- coalescing: " + ", ".join("%s %.3g" % kv for kv in co.items()))
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            lines.append("- wave-cycle split: wait %.0f%%, issue-stall %.0f%%, active %.0f%%" % (
                100 * c.get("SQ_WAIT_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc))
    open(out + "_summary.md", "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))
    return pmc


def record_traffic(pmc, key, kernel_prefix, path, steps=None):
    """Store the corrected HBM bytes per dispatch of the dominant kernel in
    profiles/traffic.json under `key` ("fabric/mode/N<n>"); bench.py reports
    it as roofline.traffic.  With several "+"-separated kernel prefixes
    (a step made of several kernels, e.g. the bit-plane BFS's level launches
    + its table pass) and `steps` = steps the profiled run executed, the
    value is their summed traffic per step."""
    prefixes = kernel_prefix.split("+")
    tb = 0.0
    for pre in prefixes:
        hits = [d for k, d in pmc.items() if pre in k]
        if not hits:
            raise SystemExit("no PMC rows for kernel %r" % pre)
        if len(prefixes) == 1:
            hits = hits[:1]
        # a step of several kernels: every instantiation matching the prefix
        # (e.g. the plane BFS's 8- and 3-level-plane variants) counts
        for h in hits:
            c = h["counters"]
            if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
                raise SystemExit("FETCH_SIZE / WRITE_SIZE missing for %r" % pre)
            tb += hbm_bytes(c) * (h["dispatches"] / float(steps) if len(prefixes) > 1 else 1.0)
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[key] = tb
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print("traffic %s = %.4g bytes per dispatch -> %s" % (key, tb, path))


if __name__ == "__main__":
    res = main(sys.argv[1], sys.argv[2])
    if len(sys.argv) > 4:      # ... KEY KERNEL_PREFIX[+PREFIX...] [STEPS] -> profiles/traffic.json
        record_traffic(res, sys.argv[3], sys.argv[4],
                       os.path.join(os.path.dirname(sys.argv[2]) or ".", "traffic.json"),
                       int(sys.argv[5]) if len(sys.argv) > 5 else None)
