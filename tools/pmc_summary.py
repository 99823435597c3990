#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_*/run_counter_collection.csv)
per kernel and write profiles/traffic_<config>.json for bench.py's
roofline.traffic.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE tallies 128-B fabric read requests at 64 B
(TCC_EA0_RDREQ x 64 B), so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE x
1024 is exact for full-line stores.  Infinity-Cache hits are counted by these
fabric counters, so this is memory-side (L2-miss) traffic, an upper bound on
DRAM bytes.

    python tools/pmc_summary.py [--dir gpurun_out] [--config c2] [--kernel k_render]
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--config", default="c2")
    ap.add_argument("--kernel", default="k_render<false")
    ap.add_argument("--out", default=None)
    ap.add_argument("--fpl", type=int, default=8, help="frames per launch of the profiled bench run")
    ap.add_argument("--prefix", default="", help="pass directories pmc_<prefix>* only (tools/measure.sh pmc: TAG + config)")
    ap.add_argument("--grid", type=int, default=0, help="dispatches of this Grid_Size only (-1: the largest, i.e. the full-group launches)")
    ap.add_argument("--l1", default=None, help="print every counter's per-launch mean of the passes <dir>/<L1>* (measure.sh pmc-l1)")
    a = ap.parse_args()
    if a.l1:
        vals = collections.defaultdict(list)
        for f in glob.glob(os.path.join(a.dir, f"{a.l1}*", "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if a.kernel in row["Kernel_Name"]:
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
        if not vals:
            raise SystemExit("no counter rows for " + a.kernel)
        for k in sorted(vals):
            print(f"{k:40s} {sum(vals[k]) / len(vals[k]):16.0f}  ({len(vals[k])} launches)")
        return
    vals = collections.defaultdict(list)
    files = glob.glob(os.path.join(a.dir, f"pmc_{a.prefix}*", "*counter_collection.csv"))
    if a.grid < 0:   # the largest grid of the kernel: the full-group launches of a grouped loop
        a.grid = max(int(row.get("Grid_Size", 0)) for f in files for row in csv.DictReader(open(f))
                     if a.kernel in row["Kernel_Name"])
    for f in files:
        for row in csv.DictReader(open(f)):
            name = row["Kernel_Name"]
            if a.kernel not in name or (a.grid and int(row.get("Grid_Size", 0)) != a.grid):
                continue
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    if "FETCH_SIZE" not in avg:
        raise SystemExit("no FETCH_SIZE rows for " + a.kernel)
    read_b = 2.0 * avg["FETCH_SIZE"] * 1024
    write_b = avg.get("WRITE_SIZE", 0.0) * 1024
    out = {"kernel": a.kernel, "config": a.config, "frames_per_launch": a.fpl, "launches": len(vals.get("FETCH_SIZE", [])),
           "hbm_bytes_per_launch": int(read_b + write_b),
           "read_bytes_per_launch": int(read_b), "write_bytes_per_launch": int(write_b),
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 64-B tally of 128-B requests), write = WRITE_SIZE KiB",
           "counters_avg_per_launch": avg}
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    path = a.out or os.path.join(ROOT, "profiles", f"traffic_{a.config}.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in out.items() if k != "counters_avg_per_launch"}))


if __name__ == "__main__":
    main()
